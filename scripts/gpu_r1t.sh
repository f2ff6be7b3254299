# Round-1t: full gpu suite + smoke on the light-first causal default, bench lines, rocprof
# kernel-trace stats of the default bench, PMC traffic of the default causal forward.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/t_r1t.log 2>&1 || { tail -30 gpurun_out/t_r1t.log; exit 1; }
tail -3 gpurun_out/t_r1t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_r1t.json 2> gpurun_out/bench_r1t.err || { tail gpurun_out/bench_r1t.err; exit 1; }
cat gpurun_out/bench_r1t.json
timeout -k 10 300 python bench.py --causal --no-cpu > gpurun_out/bench_r1t_causal.json 2>> gpurun_out/bench_r1t.err || exit 1
cat gpurun_out/bench_r1t_causal.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1t -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_r1t.log 2>&1 || exit 1
POL=0 TAG=r1t_causal CAUSAL=1 PMC_GROUPS=traffic bash scripts/gpu_pmc.sh || exit 1
