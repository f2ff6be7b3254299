# GPU pytest subset (TESTS = pytest args, default the varlen + flash golden + fused bwd tests)
# then, with AB=1, the interleaved fused-vs-split backward A/B and its kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
TESTS=${TESTS:-"tests/test_varlen_gpu.py tests/test_flash_gpu.py"}
K=${K:-"golden_fp32 or varlen or bwd_policies"}
timeout -k 10 600 python -u -m pytest $TESTS -k "$K" -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
if [ "${AB:-0}" = "1" ]; then
  timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,120} > gpurun_out/ab_$TAG.txt 2>&1 \
   && timeout -k 10 300 python scripts/ablate_bwd.py ${POLS:-0,120} causal >> gpurun_out/ab_$TAG.txt 2>&1 \
   && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
        -- python3 scripts/ablate_bwd.py ${POLS:-0,120} causal > gpurun_out/prof_$TAG.log 2>&1
  rc=$?
  cat gpurun_out/ab_$TAG.txt
fi
exit $rc
