# round 4: the causal W4 default under the flash tests; fp32-output causal W4 A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4n}
timeout -k 10 900 python -u -m pytest tests/test_flash_gpu.py tests/test_varlen_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_flash_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed" gpurun_out/tests_flash_$TAG.log | tail -8; [ $rc -eq 0 ] || exit $rc
OUT=f32 ROUNDS=10 MT_DIAG=1 ENVAB=MT_KNOB:0,4,6 timeout -k 10 300 python scripts/ablate.py 142 causal > gpurun_out/ab_causal_f32_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_causal_f32_$TAG.txt; [ $rc -eq 0 ] || exit $rc
ROUNDS=10 timeout -k 10 300 python scripts/ablate.py 0 causal > gpurun_out/ab_causal_default_$TAG.txt 2>&1; grep -v amdgpu.ids gpurun_out/ab_causal_default_$TAG.txt
