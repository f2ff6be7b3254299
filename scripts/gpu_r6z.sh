# round 6: causal fused d = 64 backward, head groups of 128 / 64 / 32 (MT_FUSED_GROUP): repeated
# interleaved A/B and per-kernel times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1
out=gpurun_out/r6z.txt
: > $out
ROUNDS=15 ENVAB=MT_FUSED_GROUP:128,32,64 timeout -k 10 300 python -u scripts/ablate_bwd.py 0 causal >> $out 2>&1 || { tail -30 $out; exit 1; }
ROUNDS=15 ENVAB=MT_FUSED_GROUP:128,64,32 timeout -k 10 300 python -u scripts/ablate_bwd.py 0 >> $out 2>&1 || { tail -30 $out; exit 1; }
for g in 128 32; do
  MT_FUSED_GROUP=$g ROUNDS=2 ENVAB=MT_FUSED_GROUP:$g timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6z_$g -o run --output-format csv \
    -- python3 scripts/ablate_bwd.py 0 causal > /dev/null 2>&1 || { echo "prof $g failed"; exit 1; }
  echo "== causal group $g" >> $out
  python3 - gpurun_out/prof_r6z_$g >> $out <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bwd" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1000:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
done
grep -v amdgpu.ids $out
