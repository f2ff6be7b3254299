# fp32 d = 32 ring forward: parity tests, then A/B vs the two-barrier kernel at (8,16,1024,32).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py tests/test_transformer_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "fp32 or golden or random or mha or transformer or decoder or deterministic" > gpurun_out/tests_d32.log 2>&1
rc=$?
tail -3 gpurun_out/tests_d32.log
[ $rc -eq 0 ] || exit $rc
DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,109 x 8,16,1024,32 9 > gpurun_out/ab_d32.txt 2>&1 \
 && DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,109 causal 8,16,1024,32 9 >> gpurun_out/ab_d32.txt 2>&1
rc=$?
cat gpurun_out/ab_d32.txt
exit $rc
