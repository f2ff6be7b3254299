# Round-1i: parity of policies 50-53 (causal pairing) and the new causal default; A/B at d=128.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "0] or 50 or 51 or 52 or 53 or causal" > gpurun_out/t_r1i.log 2>&1 || { tail -30 gpurun_out/t_r1i.log; exit 1; }
tail -3 gpurun_out/t_r1i.log
timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 causal 0,52,53,33,52,0 > gpurun_out/ab_r1i_d128c.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/shape_bench.py 1 16 16384 128 causal 0,52,53,0,52 >> gpurun_out/ab_r1i_d128c.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/shape_bench.py 1 16 16384 64 causal 21,0,50,51,0 >> gpurun_out/ab_r1i_d128c.txt 2>&1 || exit 1
cat gpurun_out/ab_r1i_d128c.txt
