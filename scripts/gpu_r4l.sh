# round 4: v6 with 4-wave workgroups, two per CU (knob 4 of policy 140), against the 8-wave default
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4l}
MT_DIAG=1 ENVAB=MT_KNOB:0,4 timeout -k 10 300 python scripts/ablate.py 140 > gpurun_out/ab_w4_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_w4_$TAG.txt; [ $rc -eq 0 ] || exit $rc
MT_DIAG=1 ENVAB=MT_KNOB:0,5 timeout -k 10 300 python scripts/ablate.py 142 causal > gpurun_out/ab_causal_nokeep_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_causal_nokeep_$TAG.txt; exit $rc
