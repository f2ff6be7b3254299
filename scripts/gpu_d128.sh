# d = 128 forward: parity tests, then timing of the d = 128 policies at C4-like shapes,
# then the d = 64 unroll A/B.
mkdir -p gpurun_out
TAG=${1:-d128}
timeout -k 10 900 python -m pytest tests/test_flash_gpu.py -q -x -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && exit $rc
{
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 x 0,33,2 &&
  timeout -k 10 300 python scripts/shape_bench.py 1 16 16384 128 x 0,33,2 &&
  timeout -k 10 300 python scripts/shape_bench.py 8 16 16384 128 x 0,33,2 &&
  timeout -k 10 300 python scripts/shape_bench.py 8 16 4096 128 causal 0,33,2 &&
  timeout -k 10 300 python scripts/ablate.py 0,31
} > gpurun_out/sb_$TAG.txt 2>&1
rc=$?
cat gpurun_out/sb_$TAG.txt
exit $rc
