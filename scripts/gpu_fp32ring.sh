# fp32 forward ring kernel: fp32 parity tests, then interleaved A/B vs the two-barrier kernel (policy 109).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-f32ring}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "fp32_fwd_policies or config2" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,115 x 8,16,1024,64 9 > gpurun_out/ab_$TAG.txt 2>&1 \
 && DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,115 causal 8,16,1024,64 9 >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
exit $rc
