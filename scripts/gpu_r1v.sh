# Round-1v: rocprofv3 kernel-trace stats of the default bench on the restored tree.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1v -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_r1v.log 2>&1 || { tail -20 gpurun_out/prof_r1v.log; exit 1; }
grep '^{' gpurun_out/prof_r1v.log > gpurun_out/bench_r1v_prof.json || true
find gpurun_out/prof_r1v -name '*kernel_stats.csv' | head -1
