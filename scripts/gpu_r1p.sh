# Round-1p: parity of policy 61 (56 + LDS-DMA from inline asm), interleaved A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "61" > gpurun_out/t_r1p.log 2>&1 || { tail -30 gpurun_out/t_r1p.log; exit 1; }
tail -3 gpurun_out/t_r1p.log
timeout -k 10 300 python scripts/ablate.py 0,61,0,61 > gpurun_out/ab_r1p.txt 2>&1 || exit 1
cat gpurun_out/ab_r1p.txt
