# Round-1r: parity of bwd policy 62 (q64 dK/dV, one wave per SIMD, no spills), A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "bwd_policies" > gpurun_out/t_r1r.log 2>&1 || { tail -30 gpurun_out/t_r1r.log; exit 1; }
tail -3 gpurun_out/t_r1r.log
timeout -k 10 300 python scripts/ablate_bwd.py 0,62,43,0,62 > gpurun_out/ab_r1r.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/ablate_bwd.py 0,62 causal >> gpurun_out/ab_r1r.txt 2>&1 || exit 1
cat gpurun_out/ab_r1r.txt
