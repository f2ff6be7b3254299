# Generic (fp32 / bf16 d != 64) backward: parity tests, then timing at C2 fp32 and (8,16,4096,128) bf16.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-genbwd}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "generic_causal_bwd or random_fwd_bwd or golden or mha or config2" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
SHAPE=8,16,1024,64 DTYPE=fp32 timeout -k 10 300 python scripts/ablate_bwd.py 0,114 causal > gpurun_out/ab_$TAG.txt 2>&1 \
 && SHAPE=8,16,1024,64 DTYPE=fp32 timeout -k 10 300 python scripts/ablate_bwd.py 0,114 >> gpurun_out/ab_$TAG.txt 2>&1 \
 && SHAPE=8,16,4096,128 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
exit $rc
