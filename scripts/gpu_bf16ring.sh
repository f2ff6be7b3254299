# bf16 d < 64 ring forward: parity tests, then A/B vs the two-barrier generic kernel (policy 109).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "random or golden or fp32 or variants or mha or policies" > gpurun_out/tests_bf16ring.log 2>&1
rc=$?
tail -3 gpurun_out/tests_bf16ring.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/ab_fwd.py 0,109 x 8,16,1024,32 7 > gpurun_out/ab_bf16ring.txt 2>&1 \
 && timeout -k 10 200 python scripts/ab_fwd.py 0,109 causal 8,16,1024,48 7 >> gpurun_out/ab_bf16ring.txt 2>&1
rc=$?
cat gpurun_out/ab_bf16ring.txt
exit $rc
