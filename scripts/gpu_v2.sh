# v2 forward: parity tests for every fast policy, then interleaved A/B timing.
mkdir -p gpurun_out
TAG=${1:-v2}
timeout -k 10 600 python -m pytest tests/test_flash_gpu.py -q -x -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 \
  && timeout -k 10 300 python scripts/ablate.py ${POLS:-0,7,8,9} > gpurun_out/ab_$TAG.txt 2>&1 \
  && timeout -k 10 300 python scripts/ablate.py ${POLS:-0,7,8,9} causal >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
tail -3 gpurun_out/t_$TAG.log; cat gpurun_out/ab_$TAG.txt
exit $rc
