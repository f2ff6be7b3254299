# round 6: small causal grids, where v4 is still the default: v4 paired
# light-first 4 / 8 waves (policies 63 / 64) against v6's causal forms (142: 8-wave, 142:4 the
# 4-wave W4 blocks), bf16 and fp32 output, interleaved on one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=20
out=gpurun_out/ab_r6h_small_causal.txt
: > $out
for shp in 4,16,2048,64 1,16,4096,64 2,16,2048,64 8,16,1024,64 1,16,8192,64 2,16,4096,64 4,16,4096,64; do
  for o32 in 0 1; do
    OUT32=$o32 timeout -k 10 200 python scripts/ab_fwd.py 63,64,142,142:4 causal $shp 9 >> $out 2>&1 || { cat $out; exit 1; }
    echo "OUT32=$o32" >> $out
  done
done
grep -v amdgpu.ids $out
