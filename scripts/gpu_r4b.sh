# round 4: the fused backward with the in-kernel dQ reduce; parity subset, then a same-box
# A/B against the round-3 library (abl/lib_r3.so) and a kernel-trace of the new backward.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4b}
timeout -k 10 900 python -u -m pytest tests/test_flash_gpu.py tests/test_varlen_gpu.py -k "${K:-bwd or grads or varlen or deterministic or fp16pv or config3_bf16_full_size}" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -25 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_$TAG.txt
for r in 1 2; do
  for lib in abl/lib_r3.so llmsys-project-flashattn_amd/minitorch/_lib/libminitorch_hip.so; do
    for c in "" causal; do
      timeout -k 10 120 python scripts/bwd_lib_time.py $lib $c >> gpurun_out/ab_$TAG.txt 2>&1 || exit 1
    done
  done
done
cat gpurun_out/ab_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
  -- python3 scripts/bwd_lib_time.py llmsys-project-flashattn_amd/minitorch/_lib/libminitorch_hip.so > gpurun_out/prof_$TAG.log 2>&1
rc=$?
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec head -8 {} \;
exit $rc
