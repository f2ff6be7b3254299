# fp32 / generic-kernel parity, then the config-2 fp32 forward timing (A/B against the
# previous build kept as PREV_LIB when given) and a kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fp32}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
   -k "fp32 or golden or generic or variants_agree or minitorch or transformer or config2" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 200 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
python3 -c "import json; j=json.load(open('gpurun_out/bench_$TAG.json')); print(j['value'], j['extra'])"
exit $rc
