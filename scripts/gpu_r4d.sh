# round 4: A/B of the fused backward's dQ hand-off forms (diagnostics build, MT_KNOB):
# 0 the in-kernel last-arriver reduce, 16 the round-3 form (separate reduce kernel),
# 1 / 2 / 3 without the reduction / arrivals / both (timing only), 4 plain stores, 8 global atomic
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4d}
MT_DIAG=1 ENVAB=MT_KNOB:0,16,1,2,3,4,8,32,40,33 timeout -k 10 300 python scripts/ablate_bwd.py 120 > gpurun_out/ab_$TAG.txt 2>&1 \
 && MT_DIAG=1 ENVAB=MT_KNOB:0,16,1,2,3,4,8,32,40,33 timeout -k 10 300 python scripts/ablate_bwd.py 120 causal >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/ab_$TAG.txt
[ $rc -eq 0 ] || exit $rc
MT_DIAG=1 timeout -k 10 300 python scripts/probe_fused_var.py > gpurun_out/probe_var_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/probe_var_$TAG.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_op_census.py > gpurun_out/c5_census_$TAG.txt 2>&1 && head -80 gpurun_out/c5_census_$TAG.txt
timeout -k 10 600 python -u -m pytest tests/test_minitorch_gpu.py tests/test_transformer_gpu.py tests/test_varlen_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_mt_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/tests_mt_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mt_step_bench.py 20 > gpurun_out/c5_$TAG.json 2>&1 && cat gpurun_out/c5_$TAG.json
MT_DIAG=1 timeout -k 10 120 python scripts/stamp_fwd.py --json gpurun_out/stamp_fwd_$TAG.json > gpurun_out/stamp_fwd_$TAG.txt 2>&1; grep -v amdgpu.ids gpurun_out/stamp_fwd_$TAG.txt
