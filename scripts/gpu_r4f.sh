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
timeout -k 10 600 python -u -m pytest tests/test_minitorch_gpu.py tests/test_transformer_gpu.py tests/test_optim_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_mt_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/tests_mt_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_op_census.py > gpurun_out/c5_census_$TAG.txt 2>&1 && head -40 gpurun_out/c5_census_$TAG.txt
timeout -k 10 300 python scripts/mt_step_bench.py 20 > gpurun_out/c5_$TAG.json 2>&1 && cat gpurun_out/c5_$TAG.json
