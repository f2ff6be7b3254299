# bf16 backward: parity tests of every bwd policy, then an interleaved A/B at C3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-bwd}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
   -k "bwd_policies or random_fwd_bwd or config3" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,40,43} > gpurun_out/ab_$TAG.txt 2>&1 \
 && timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,40,43} causal >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
exit $rc
