# GPU session: parity tests, smoke, kernel-trace profile of the bench, full bench line.
# Usage (from the repo root on the GPU box): bash scripts/gpu_check.sh [TAG]
set -o pipefail
TAG=${1:-r1}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1 \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
       -- python3 bench.py --steps 100 --warmup 20 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 \
  && timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/tests_$TAG.log
cat gpurun_out/smoke_$TAG.log gpurun_out/bench_$TAG.json 2>/dev/null
exit $rc
