# round 6: W4 non-causal with the first pair's second workgroup started late (MT_KNOB 100 + n:
# n x 8128 cycles of s_sleep) so the two workgroups of a CU issue their O stores at different
# times; knob 4 = W4 without the code, 0 = 8-wave. C3 bf16 / fp32 out, interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=20
out=gpurun_out/ab_r6j_stagger.txt
: > $out
for shp in 8,16,4096,64 16,16,2048,64; do
for o32 in 0 1; do
  OUT32=$o32 ENVAB=MT_KNOB:4,100,101,102,104,108 timeout -k 10 200 python scripts/ab_fwd.py 140 nc $shp 9 >> $out 2>&1 || { cat $out; exit 1; }
  echo "OUT32=$o32" >> $out
done
done
grep -v amdgpu.ids $out
