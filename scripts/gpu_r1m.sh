# Round-1m: parity of policies 57/58 (LDS reads 3/4 MFMAs ahead), interleaved A/B vs 56.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "57 or 58" > gpurun_out/t_r1m.log 2>&1 || { tail -30 gpurun_out/t_r1m.log; exit 1; }
tail -3 gpurun_out/t_r1m.log
timeout -k 10 300 python scripts/ablate.py 56,57,58,0,56,57,58 > gpurun_out/ab_r1m.txt 2>&1 || exit 1
cat gpurun_out/ab_r1m.txt
