# round 6: backend 2's 128x128 X3 GEMM tile: the matmul tests, then the probe against the 64x64
# tile and rocBLAS (kernel stats)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ao.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_minitorch_gpu.py -k matmul \
  > gpurun_out/r6ao_tests.txt 2>&1 || { tail -30 gpurun_out/r6ao_tests.txt; exit 1; }
tail -1 gpurun_out/r6ao_tests.txt > $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6ao -o run --output-format csv \
  -- python3 scripts/gemm_x3_probe.py >> $out 2>&1 || { tail -20 $out; exit 1; }
python3 - >> $out <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_r6ao/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm" in r["Name"] or "Cijk" in r["Name"] or "splitk" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1000:9.1f} us x{r['Calls']:>4} {r['Name'][:110]}")
PY
grep -v -e amdgpu.ids -e "^W2026" -e "^E2026" $out
