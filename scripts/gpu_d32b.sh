# fp32 d = 32 ring backward: parity tests, then A/B vs the LDS-row kernels (policy 114) at (8,16,1024,32).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py tests/test_transformer_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "generic_causal_bwd or fp32 or golden or random or mha or transformer or decoder or variants or policies" > gpurun_out/tests_d32b.log 2>&1
rc=$?
tail -3 gpurun_out/tests_d32b.log
[ $rc -eq 0 ] || exit $rc
SHAPE=8,16,1024,32 timeout -k 10 300 python scripts/ablate_bwd.py 0,114 > gpurun_out/ab_d32b.txt 2>&1 \
 && SHAPE=8,16,1024,48 timeout -k 10 300 python scripts/ablate_bwd.py 0,114 causal >> gpurun_out/ab_d32b.txt 2>&1 \
 && SHAPE=8,16,1024,64 DTYPE=fp32 timeout -k 10 300 python scripts/ablate_bwd.py 0,114 >> gpurun_out/ab_d32b.txt 2>&1
rc=$?
cat gpurun_out/ab_d32b.txt
exit $rc
