# Paired causal backward (policies 107 / 108): parity vs the oracle, then interleaved A/B at C3 causal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pair}
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "bwd_policies and (107 or 108 or -0-)" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,74,107,108} causal > gpurun_out/ab_$TAG.txt 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
exit $rc
