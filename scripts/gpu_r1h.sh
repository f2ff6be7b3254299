# Round-1h: parity of the new A/B policies (46-51), then interleaved A/B timings.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "46 or 47 or 48 or 49 or 50 or 51" > gpurun_out/t_r1h.log 2>&1 || { tail -30 gpurun_out/t_r1h.log; exit 1; }
tail -3 gpurun_out/t_r1h.log
timeout -k 10 300 python scripts/ablate.py 37,46,47,48,49,0 > gpurun_out/ab_r1h_nc.txt 2>&1 || exit 1
cat gpurun_out/ab_r1h_nc.txt
timeout -k 10 300 python scripts/ablate.py 0,50,51,21 causal > gpurun_out/ab_r1h_c.txt 2>&1 || exit 1
cat gpurun_out/ab_r1h_c.txt
