# Round-1u: parity of bwd policy 66 (64-query dK/dV with Q / dO images by LDS-DMA), A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "bwd_policies" > gpurun_out/t_r1u.log 2>&1 || { tail -30 gpurun_out/t_r1u.log; exit 1; }
tail -3 gpurun_out/t_r1u.log
timeout -k 10 300 python scripts/ablate_bwd.py 0,66,42,0,66 > gpurun_out/ab_r1u.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/ablate_bwd.py 0,66 causal >> gpurun_out/ab_r1u.txt 2>&1 || exit 1
cat gpurun_out/ab_r1u.txt
