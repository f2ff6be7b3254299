# Fused backward (policy 120): parity vs the oracle, then interleaved A/B against the split
# default at C3 (non-causal and causal) and a kernel-trace profile of the A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fused}
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "bwd_policies and 120" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,120} > gpurun_out/ab_$TAG.txt 2>&1 \
 && timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,120} causal >> gpurun_out/ab_$TAG.txt 2>&1 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
      -- python3 scripts/ablate_bwd.py ${POLS:-0,120} > gpurun_out/prof_$TAG.log 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
exit $rc
