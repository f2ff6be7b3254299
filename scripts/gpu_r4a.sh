set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "fp16pv or config3_bf16_full_size or fp32_out_option or huge_spike or spiked_rescale or golden" -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4a_tests.log; [ $rc -eq 0 ] || exit $rc
OUT=both ROUNDS=3 timeout -k 10 120 python scripts/shape_bench.py 8 16 4096 64 causal > gpurun_out/r4a_causal_out32.txt 2>&1; rc=$?
cat gpurun_out/r4a_causal_out32.txt; exit $rc
