# Round-2a: first GPU check of the re-entry tree: gpu tests (with the parity record),
# smoke, a kernel-trace profile of the bench, the default bench line.
set -o pipefail
TAG=${1:-r2c}
mkdir -p gpurun_out
export TMPDIR=/tmp
export MT_PARITY_OUT=gpurun_out/parity_$TAG.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
       -- python3 bench.py --steps 100 --warmup 20 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 \
  && timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/tests_$TAG.log
cat gpurun_out/smoke_$TAG.log gpurun_out/bench_$TAG.json 2>/dev/null
exit $rc
