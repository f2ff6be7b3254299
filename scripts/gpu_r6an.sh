# round 6: backend 0 (rocBLAS, the X3 128x128 GEMM on the LM-head-forward class) against 4
# (rocBLAS only) and 2 (X3 everywhere): the tests that run minitorch's matmuls under the default,
# then config 5's step legs of bench.py, interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6an.txt
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_transformer_gpu.py tests/test_graphs_gpu.py tests/test_optim_gpu.py tests/test_xent_gpu.py tests/test_minitorch_gpu.py \
  > gpurun_out/r6an_tests.txt 2>&1 || { tail -40 gpurun_out/r6an_tests.txt; exit 1; }
tail -2 gpurun_out/r6an_tests.txt >> $out
for r in 1 2 3; do
  for b in 0 4 2; do
    MT_GEMM_BACKEND=$b timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/r6an_b$b.json 2>/dev/null || { echo "bench $b failed" >> $out; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r6an_b$b.json'))['extra']
print('backend $b round $r:', {k: d[k] for k in ('c5_step_ms','c5_gpu_ms','c5_graph_step_ms','c5_loss','c5_graph_loss') if k in d})" >> $out
  done
done
cat $out
