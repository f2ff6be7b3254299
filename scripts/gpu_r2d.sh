# Round-2d: v5 causal (paired blocks, pipelined per-wave diagonal) parity + A/B timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export MT_PARITY_OUT=gpurun_out/parity_r2d.json
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
   -k "v5_causal or fast_policies_vs_oracle or huge_spike or spiked_rescale or kernel_variants or config3" > gpurun_out/tests_r2d.log 2>&1
rc=$?
tail -5 gpurun_out/tests_r2d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_fwd.py 63,64,67,68 causal 8,16,4096,64 > gpurun_out/ab_r2d.txt 2>&1 \
 && timeout -k 10 300 python scripts/ab_fwd.py 64,67,68 causal 1,16,16384,64 >> gpurun_out/ab_r2d.txt 2>&1 \
 && timeout -k 10 300 python scripts/ab_fwd.py 63,67 causal 4,16,2048,64 >> gpurun_out/ab_r2d.txt 2>&1
rc=$?
cat gpurun_out/ab_r2d.txt
exit $rc
