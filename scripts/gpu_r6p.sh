# round 6: causal fp32-O forward: 142 = the default 610 (8-wave, fp16 PV), 142:4 = W4 with fp16
# PV (16994, spills), 142:6 = W4 fp16 PV without the V^T reuse (16998), 142:5 = 610 without reuse
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=20 OUT32=1
out=gpurun_out/ab_r6p_causal_f32o.txt
: > $out
for shp in 8,16,4096,64 4,16,4096,64 2,16,8192,64 16,16,2048,64; do
  timeout -k 10 200 python scripts/ab_fwd.py 142,142:4,142:6,142:5 causal $shp 9 >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
