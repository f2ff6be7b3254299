# Full check of the tree on a fresh box: every GPU test, smoke, a kernel-trace profile of the
# bench, the bench line, and the HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the default
# C3 backward. Usage: TAG=r4k STAGE=tests|bench bash scripts/gpu_final.sh (two calls: each fits
# one gpurun limit)
set -o pipefail
TAG=${TAG:-r4k}
STAGE=${STAGE:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$STAGE" = tests ]; then
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; grep -E "FAILED|ERROR" gpurun_out/tests_$TAG.log | head; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/parity.json gpurun_out/parity_$TAG.json 2>/dev/null
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
exit 0
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 100 --warmup 20 --no-cpu > gpurun_out/prof_$TAG.log 2>&1; rc=$?; echo prof rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "fa_bwd" -d gpurun_out/pmcbwd_${TAG}_$c -o run --output-format csv -- python3 scripts/ablate_bwd.py 0 > gpurun_out/pmcbwd_${TAG}_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo pmc ok
