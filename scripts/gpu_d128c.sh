mkdir -p gpurun_out
{
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 x 33,32,44,33,32,44 &&
  timeout -k 10 300 python scripts/shape_bench.py 1 16 16384 128 x 33,32,33,32 &&
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 causal 33,32,33,32 &&
  timeout -k 10 300 python scripts/shape_bench.py 2 16 2048 128 x 33,32,33,32 &&
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 64 causal 21,22,21,22
} > gpurun_out/sb_d128c.txt 2>&1
rc=$?; cat gpurun_out/sb_d128c.txt; exit $rc
