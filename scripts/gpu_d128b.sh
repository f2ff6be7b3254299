mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_flash_gpu.py -q -x -p no:cacheprovider > gpurun_out/t_d128b.log 2>&1
rc=$?; tail -3 gpurun_out/t_d128b.log; [ $rc -ne 0 ] && exit $rc
{
  timeout -k 10 300 python scripts/shape_bench.py 8 16 16384 128 x 32,44,32,44 &&
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 x 33,45,32,44 &&
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 causal 33,45
} > gpurun_out/sb_d128b.txt 2>&1
rc=$?; cat gpurun_out/sb_d128b.txt; exit $rc
