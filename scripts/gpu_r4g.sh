# round 4: v6 forward with the tile's LDS-DMA issued by the older half only (knob 1), A/B and
# stamps; the C5 step launches after the matmul-transpose / gradient-copy changes (rocprof)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4g}
MT_DIAG=1 ENVAB=MT_KNOB:0,1 timeout -k 10 300 python scripts/ablate.py 140 > gpurun_out/ab_odma_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_odma_$TAG.txt; [ $rc -eq 0 ] || exit $rc
MT_DIAG=1 MT_KNOB=1 timeout -k 10 120 python scripts/stamp_fwd.py --json gpurun_out/stamp_odma_$TAG.json > gpurun_out/stamp_odma_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/stamp_odma_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_minitorch_gpu.py tests/test_transformer_gpu.py tests/test_optim_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_mt_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/tests_mt_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_op_census.py > gpurun_out/c5_census_$TAG.txt 2>&1 && head -12 gpurun_out/c5_census_$TAG.txt
timeout -k 10 300 python scripts/mt_step_bench.py 20 > gpurun_out/c5_$TAG.json 2>&1 && cat gpurun_out/c5_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_$TAG -o c5 -- python3 scripts/mt_step_bench.py 10 > gpurun_out/c5prof_$TAG.log 2>&1; echo rocprof rc=$?
