# round 6: the 128x128 X3 GEMM tile against the 64x64 one and rocBLAS on config 5's shapes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6am -o run --output-format csv \
  -- python3 scripts/gemm_x3_probe.py > gpurun_out/r6am.txt 2>&1 || { tail -20 gpurun_out/r6am.txt; exit 1; }
python3 - >> gpurun_out/r6am.txt <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_r6am/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"  {float(r['AverageNs'])/1000:9.1f} us x{r['Calls']:>4} {r['Name'][:110]}")
PY
grep -v amdgpu.ids gpurun_out/r6am.txt
