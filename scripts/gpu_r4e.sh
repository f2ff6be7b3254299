# round 4: the d = 128 split backward (parity + timing), then the fused-bwd A/B forms, the
# forward stamps, the C5 census and step.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4e}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "d128 or random_fwd_bwd" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_d128_$TAG.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/tests_d128_$TAG.log | tail -40; [ $rc -eq 0 ] || exit $rc
SHAPE=8,16,4096,128 timeout -k 10 300 python scripts/ablate_bwd.py 0,1 > gpurun_out/ab_d128_$TAG.txt 2>&1 && SHAPE=8,16,4096,128 timeout -k 10 300 python scripts/ablate_bwd.py 0,1 causal >> gpurun_out/ab_d128_$TAG.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_d128_$TAG.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r4d.sh
