# round 4: the d = 128 dQ pass as 8-wave workgroups, causal too (knob 48: operand ring 2
# ahead; 46 / 47: 3 ahead, 47 also causal): parity (knob 48), interleaved timing
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4ad}
DIAGLIB=$PWD/llmsys-project-flashattn_amd/minitorch/_lib/diag/libminitorch_hip_diag.so
MT_HIP_LIB=$DIAGLIB MT_KNOB=48 timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "d128" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_d128w_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/tests_d128w_$TAG.log | tail -8; [ $rc -eq 0 ] || exit $rc
SHAPE=8,16,4096,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,46,48 timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_d128w_$TAG.txt 2>&1 && SHAPE=8,16,4096,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,47,48 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128w_$TAG.txt 2>&1 && SHAPE=4,32,1100,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,48 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128w_$TAG.txt 2>&1 && SHAPE=4,32,1100,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,48 timeout -k 10 300 python scripts/ablate_bwd.py 0 >> gpurun_out/ab_d128w_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_d128w_$TAG.txt; exit $rc
