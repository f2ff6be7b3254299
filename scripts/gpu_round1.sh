# Round-1 GPU session script: parity tests, bench (A/B kernel policies), rocprof.
set -x
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_flash_gpu.py -q -p no:cacheprovider > gpurun_out/t3.log 2>&1; echo "PYTEST_EXIT $?" >> gpurun_out/t3.log
for pol in 0 2 1; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-extra --policy $pol > gpurun_out/bench3_p$pol.json 2> gpurun_out/bench3_p$pol.err || break
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --no-extra --policy $pol --causal > gpurun_out/bench3c_p$pol.json 2>> gpurun_out/bench3_p$pol.err || break
done
tail -5 gpurun_out/t3.log; cat gpurun_out/bench3*.json
