# Round-2b: the new GPU tests (sharded fwd/bwd over RCCL, transformer parity, companion
# fixtures, host-ASan C ABI).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export MT_PARITY_OUT=gpurun_out/parity_r2b.json
timeout -k 10 900 python -u -m pytest tests/test_shard_gpu.py tests/test_transformer_gpu.py \
  tests/test_asan.py "tests/test_minitorch_gpu.py::test_attn_softmax_vs_reference_fixtures" \
  "tests/test_minitorch_gpu.py::test_layernorm_vs_reference_fixtures" \
  -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_r2b.log 2>&1
rc=$?
tail -40 gpurun_out/tests_r2b.log
exit $rc
