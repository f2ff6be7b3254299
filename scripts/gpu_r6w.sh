# round 6: per-kernel times of the fused fp32 backward at C2 (non-causal, causal paired, causal
# unpaired = MT_KNOB 61) against the split ring (MT_KNOB 60)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 DTYPE=fp32 SHAPE=${SHAPE:-8,16,1024,64} ROUNDS=3
out=gpurun_out/r6w.txt
: > $out
for c in nc causal; do
  cc=""; [ $c = causal ] && cc=causal
  ENVAB=MT_KNOB:0,60,61 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 $cc >> $out 2>&1 || { tail -30 $out; exit 1; }
  for kn in 0 60 61; do
    MT_KNOB=$kn ENVAB=MT_KNOB:$kn timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6w_${c}_$kn -o run --output-format csv \
      -- python3 scripts/ablate_bwd.py 0 $cc > /dev/null 2>&1 || { echo "prof $c $kn failed"; exit 1; }
    echo "== $c knob $kn" >> $out
    python3 - gpurun_out/prof_r6w_${c}_$kn >> $out <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bwd" in r["Name"] or "prep" in r["Name"]:
            print(f"  {float(r['AverageNs'])/1000:9.1f} us x{r['Calls']:>4} {r['Name'][:90]}")
PY
  done
done
grep -v amdgpu.ids $out
