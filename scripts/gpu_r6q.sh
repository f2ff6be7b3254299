# round 6: the per-GPU C3 shards of the scaling run (N = 8: (1,16,4096,64), N = 4: (2,16,4096,64),
# N = 2: (4,16,4096,64)) with the fp32 O of the headline: default vs the v6 forms
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=40 OUT32=1
out=gpurun_out/ab_r6q_shards.txt
: > $out
for shp in 1,16,4096,64 2,16,4096,64 4,16,4096,64; do
  timeout -k 10 200 python scripts/ab_fwd.py 0,140,140:4,105,141 nc $shp 9 >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
