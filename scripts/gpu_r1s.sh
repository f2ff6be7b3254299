# Round-1s: causal pair order light-first (policies 63/64 v4, 65 d128): parity, A/B, PMC traffic.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "fast_policies_vs_oracle and (50 or 51 or 53 or 63 or 64 or 65) or long_causal" > gpurun_out/t_r1s.log 2>&1 || { tail -30 gpurun_out/t_r1s.log; exit 1; }
tail -3 gpurun_out/t_r1s.log
: > gpurun_out/ab_r1s.txt
timeout -k 10 120 python scripts/shape_bench.py 8 16 4096 64 causal 0,63,50,63,0,63 >> gpurun_out/ab_r1s.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/shape_bench.py 1 16 16384 64 causal 0,64,51,64,0,64 >> gpurun_out/ab_r1s.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/shape_bench.py 8 16 4096 128 causal 0,65,0,65,0,65 >> gpurun_out/ab_r1s.txt 2>&1 || exit 1
timeout -k 10 120 python scripts/shape_bench.py 1 16 16384 128 causal 0,65,0,65 >> gpurun_out/ab_r1s.txt 2>&1 || exit 1
cat gpurun_out/ab_r1s.txt
POL=63 TAG=r1s_p63c CAUSAL=1 PMC_GROUPS=traffic bash scripts/gpu_pmc.sh || exit 1
POL=50 TAG=r1s_p50c CAUSAL=1 PMC_GROUPS=traffic bash scripts/gpu_pmc.sh || exit 1
