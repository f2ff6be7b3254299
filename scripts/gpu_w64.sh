# One-wave-per-SIMD dK/dV (policy 72): parity of the bwd policies, interleaved A/B at C3,
# and a kernel-trace of both forms (dK/dV vs dQ time).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-w64}
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "bwd_policies and (72 or 69)" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-69,72} > gpurun_out/ab_$TAG.txt 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/scripts/ablate_bwd.py ${POLS:-69,72} > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT && find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -12
exit $rc
