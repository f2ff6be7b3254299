# Quick GPU iteration: one test file (FILE), then an interleaved bwd A/B (POLS, causal if CAUSAL=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-quick}
timeout -k 10 600 python -u -m pytest ${FILE:-tests/test_flash_gpu.py} -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider \
   ${KSEL:+-k "$KSEL"} > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$POLS" ]; then
  timeout -k 10 300 python scripts/ablate_bwd.py $POLS ${CAUSAL:+causal} > gpurun_out/ab_$TAG.txt 2>&1
  rc=$?
  cat gpurun_out/ab_$TAG.txt
fi
exit $rc
