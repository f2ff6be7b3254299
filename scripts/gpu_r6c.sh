# round 6: W4 (4-wave workgroups, two per CU) vs the 8-wave v6<66> non-causal default, bf16
# and fp32 output, longer interleaved A/B (20 launches per arm per round)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=20
out=gpurun_out/ab_r6c_w4.txt
: > $out
for shp in 8,16,4096,64 4,16,8192,64 16,16,2048,64 2,16,16384,64 8,16,4032,64; do
  for o32 in 0 1; do
    OUT32=$o32 ENVAB=MT_KNOB:0,4 timeout -k 10 200 python scripts/ab_fwd.py 140 nc $shp 11 >> $out 2>&1 || { cat $out; exit 1; }
    echo "OUT32=$o32" >> $out
  done
done
cat $out
