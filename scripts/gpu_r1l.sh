# Round-1l: parity of policy 56 (54 + deferred row-sum add / bf16 pack), interleaved A/B.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_gpu.py -k "56" > gpurun_out/t_r1l.log 2>&1 || { tail -30 gpurun_out/t_r1l.log; exit 1; }
tail -3 gpurun_out/t_r1l.log
timeout -k 10 300 python scripts/ablate.py 0,54,56,55,56,54 > gpurun_out/ab_r1l.txt 2>&1 || exit 1
cat gpurun_out/ab_r1l.txt
