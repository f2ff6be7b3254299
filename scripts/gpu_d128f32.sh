# fp32 d = 128 ring forward: parity, then A/B vs the two-barrier kernel (policy 109).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "random or golden or fp32 or variants" > gpurun_out/tests_d128f32.log 2>&1
rc=$?
tail -3 gpurun_out/tests_d128f32.log
[ $rc -eq 0 ] || exit $rc
DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,110 causal 8,16,1024,64 7 > gpurun_out/ab_d128f32.txt 2>&1 \
 && DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,109 causal 8,16,1024,128 7 >> gpurun_out/ab_d128f32.txt 2>&1 \
 && DTYPE=fp32 timeout -k 10 200 python scripts/ab_fwd.py 0,109 x 8,16,1024,128 7 >> gpurun_out/ab_d128f32.txt 2>&1
rc=$?
cat gpurun_out/ab_d128f32.txt
exit $rc
