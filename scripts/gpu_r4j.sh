# round 4: C5 host copies cached, column reductions with 128-row chunks
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4j}
timeout -k 10 600 python -u -m pytest tests/test_minitorch_gpu.py tests/test_transformer_gpu.py tests/test_varlen_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_mt_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed" gpurun_out/tests_mt_$TAG.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_op_census.py > gpurun_out/c5_census_$TAG.txt 2>&1 && grep -E "to_cuda|calls in one" gpurun_out/c5_census_$TAG.txt
timeout -k 10 300 python scripts/mt_step_bench.py 20 > gpurun_out/c5_$TAG.json 2>&1 && cat gpurun_out/c5_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_$TAG -o c5 -- python3 scripts/mt_step_bench.py 10 > gpurun_out/c5prof_$TAG.log 2>&1; echo rocprof rc=$?
timeout -k 10 300 python scripts/mt_step_bench.py 10 --prof gpurun_out/c5_host_$TAG.txt > /dev/null 2>&1; echo hostprof rc=$?
timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_bwd_$TAG.txt 2>&1 && timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_bwd_$TAG.txt 2>&1; grep -v amdgpu.ids gpurun_out/ab_bwd_$TAG.txt
