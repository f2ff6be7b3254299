# Round-1k: parity of policies 54/55 (Vᵀ fragments kept from P2 to P4), interleaved A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "54 or 55" > gpurun_out/t_r1k.log 2>&1 || { tail -30 gpurun_out/t_r1k.log; exit 1; }
tail -3 gpurun_out/t_r1k.log
timeout -k 10 300 python scripts/ablate.py 0,54,55,39,54 > gpurun_out/ab_r1k.txt 2>&1 || exit 1
cat gpurun_out/ab_r1k.txt
