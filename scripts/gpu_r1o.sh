# Round-1o: parity of policies 59/60 (Q prescale + C-initialised scores), interleaved A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "59 or 60" > gpurun_out/t_r1o.log 2>&1 || { tail -40 gpurun_out/t_r1o.log; exit 1; }
tail -3 gpurun_out/t_r1o.log
timeout -k 10 300 python scripts/ablate.py 0,59,60,0,59,60 > gpurun_out/ab_r1o.txt 2>&1 || exit 1
cat gpurun_out/ab_r1o.txt
