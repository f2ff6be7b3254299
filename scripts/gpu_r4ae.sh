# round 4: the non-causal d = 128 dQ pass in 8-wave workgroups as the product: parity (product
# library), then A/B against the 4-wave dQ pass (knob 50) and a 5-ahead operand ring (knob 49)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4ae}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "d128 or random_fwd_bwd" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_d128_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/tests_d128_$TAG.log | tail -8; [ $rc -eq 0 ] || exit $rc
DIAGLIB=$PWD/llmsys-project-flashattn_amd/minitorch/_lib/diag/libminitorch_hip_diag.so
MT_HIP_LIB=$DIAGLIB MT_KNOB=51 timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "d128_vs_oracle or d128_paired" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_d128k51_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/tests_d128k51_$TAG.log | tail -4; [ $rc -eq 0 ] || exit $rc
MT_HIP_LIB=$DIAGLIB MT_KNOB=49 timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "d128_vs_oracle" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_d128k49_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/tests_d128k49_$TAG.log | tail -4; [ $rc -eq 0 ] || exit $rc
SHAPE=8,16,4096,128 ROUNDS=8 MT_DIAG=1 ENVAB=MT_KNOB:0,50,49 timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_d128w_$TAG.txt 2>&1 && SHAPE=2,8,1024,128 ROUNDS=8 MT_DIAG=1 ENVAB=MT_KNOB:0,50 timeout -k 10 300 python scripts/ablate_bwd.py 0 >> gpurun_out/ab_d128w_$TAG.txt 2>&1 && SHAPE=8,16,4096,128 ROUNDS=8 MT_DIAG=1 ENVAB=MT_KNOB:0,51 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128w_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_d128w_$TAG.txt; exit $rc
