set -x
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_flash_gpu.py -q -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "PYTEST_EXIT $?" >> gpurun_out/t2.log
timeout -k 10 300 python bench.py > gpurun_out/bench2.json 2> gpurun_out/bench2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/prof2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc2_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extra > gpurun_out/pmc2a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc2_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extra > gpurun_out/pmc2b.log 2>&1
echo "ALL_EXIT $?"
tail -5 gpurun_out/t2.log; cat gpurun_out/bench2.json; tail -3 gpurun_out/bench2.err
