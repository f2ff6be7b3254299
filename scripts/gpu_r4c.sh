# round 4: everything changed this session in one GPU call: backward parity + A/B vs the
# round-3 library, fp16-PV forward parity + timing, the minitorch fused ops, the C5 step
# (time, launches per step under a kernel trace).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4c}
timeout -k 10 900 python -u -m pytest tests/test_flash_gpu.py tests/test_varlen_gpu.py tests/test_minitorch_gpu.py tests/test_optim_gpu.py tests/test_transformer_gpu.py -k "${K:-bwd or grads or varlen or deterministic or fp16pv or config3_bf16_full_size or zip_map or bias_gelu or dropout or adam or transformer or decoder or generic_ops}" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_$TAG.log | tail -80; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_$TAG.txt
for r in 1 2; do
  for lib in abl/lib_r3.so llmsys-project-flashattn_amd/minitorch/_lib/libminitorch_hip.so; do
    for c in "" causal; do
      timeout -k 10 120 python scripts/bwd_lib_time.py $lib $c >> gpurun_out/ab_$TAG.txt 2>&1 || exit 1
    done
  done
done
cat gpurun_out/ab_$TAG.txt
OUT=both ROUNDS=2 timeout -k 10 120 python scripts/shape_bench.py 8 16 4096 64 causal > gpurun_out/causal_out32_$TAG.txt 2>&1 || exit 1
cat gpurun_out/causal_out32_$TAG.txt
timeout -k 10 300 python scripts/mt_step_bench.py 20 > gpurun_out/c5_$TAG.json 2>&1 || exit 1
cat gpurun_out/c5_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bwd_$TAG -o run --output-format csv \
  -- python3 scripts/bwd_lib_time.py llmsys-project-flashattn_amd/minitorch/_lib/libminitorch_hip.so > gpurun_out/prof_bwd_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv \
  -- python3 scripts/mt_step_bench.py 10 > gpurun_out/prof_c5_$TAG.log 2>&1
rc=$?
for f in $(find gpurun_out/prof_bwd_$TAG gpurun_out/prof_c5_$TAG -name "*kernel_stats.csv"); do echo $f; head -12 $f | cut -c1-200; done
exit $rc
