# round 6: kernel times of the X3 GEMM against rocBLAS on config 5's shapes (rocprofv3 stats)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6ag -o run --output-format csv \
  -- python3 scripts/gemm_x3_probe.py > gpurun_out/r6ag.txt 2>&1 || { tail -20 gpurun_out/r6ag.txt; exit 1; }
python3 - >> gpurun_out/r6ag.txt <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_r6ag/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {float(r['AverageNs'])/1000:9.1f} us x{r['Calls']:>4} {r['Name'][:110]}")
PY
grep -v amdgpu.ids gpurun_out/r6ag.txt
