# round 4: v6 with the packed scale-and-shift (knob 7) vs the default, 10 rounds, C3; the d = 128
# backward's operand-read distance (knobs 12 / 14 / 15 = 2 / 4 / 5 slots; 0 = 3)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4o}
ROUNDS=10 MT_DIAG=1 ENVAB=MT_KNOB:0,7 timeout -k 10 300 python scripts/ablate.py 140 > gpurun_out/ab_pk_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_pk_$TAG.txt; [ $rc -eq 0 ] || exit $rc
SHAPE=8,16,4096,128 MT_DIAG=1 ENVAB=MT_KNOB:0,12,14,15 timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_d128ah_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_d128ah_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./scripts/valu_rate_bench 2.1 > gpurun_out/valu_rate_$TAG.txt 2>&1; cat gpurun_out/valu_rate_$TAG.txt
MT_DIAG=1 ENVAB=MT_KNOB:0,96 ROUNDS=8 timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_bwdpk_$TAG.txt 2>&1 && MT_DIAG=1 ENVAB=MT_KNOB:0,80 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_bwdpk_$TAG.txt 2>&1; grep -v amdgpu.ids gpurun_out/ab_bwdpk_$TAG.txt
timeout -k 10 300 python -u -m pytest tests/test_varlen_gpu.py -k paired -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_varlen_pair_$TAG.log 2>&1; tail -3 gpurun_out/tests_varlen_pair_$TAG.log
