# round 4: the d = 128 backward with operand prefetch (parity + timing), the fused d = 64
# backward's per-case default forms (rotated non-causal), the backward tests.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4f}
timeout -k 10 900 python -u -m pytest tests/test_flash_gpu.py -k "d128 or bwd or grads or determin" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_bwd_$TAG.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error|assert" gpurun_out/tests_bwd_$TAG.log | tail -30; [ $rc -eq 0 ] || exit $rc
SHAPE=8,16,4096,128 timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_d128_$TAG.txt 2>&1 && SHAPE=8,16,4096,128 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128_$TAG.txt 2>&1 \
 && timeout -k 10 300 python scripts/ablate_bwd.py 0 >> gpurun_out/ab_d128_$TAG.txt 2>&1 && timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128_$TAG.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_d128_$TAG.txt; [ $rc -eq 0 ] || exit $rc
