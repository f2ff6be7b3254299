# round 4: A/B of the fused backward's dQ hand-off forms (diagnostics build, MT_KNOB):
# 0 the in-kernel last-arriver reduce, 16 the round-3 form (separate reduce kernel),
# 1 / 2 / 3 without the reduction / arrivals / both (timing only), 4 plain stores, 8 global atomic
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4d}
MT_DIAG=1 ENVAB=MT_KNOB:0,16,1,2,3,4,8 timeout -k 10 300 python scripts/ablate_bwd.py 120 > gpurun_out/ab_$TAG.txt 2>&1 \
 && MT_DIAG=1 ENVAB=MT_KNOB:0,16,1,2,3,4,8 timeout -k 10 300 python scripts/ablate_bwd.py 120 causal >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ab_$TAG.txt
exit $rc
timeout -k 10 300 python scripts/c5_op_census.py > gpurun_out/c5_census_$TAG.txt 2>&1 && head -80 gpurun_out/c5_census_$TAG.txt
