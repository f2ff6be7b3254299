# round 6: one wave per SIMD with v6's stream (W4, LDS padded so one workgroup fits a CU:
# MT_KNOB 8) against the 8-wave default (0) and W4 two per CU (4), C3 bf16 / fp32 out
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=20
out=gpurun_out/ab_r6f_onewave.txt
: > $out
for o32 in 0 1; do
  OUT32=$o32 ENVAB=MT_KNOB:0,4,8 timeout -k 10 200 python scripts/ab_fwd.py 140 nc 8,16,4096,64 9 >> $out 2>&1 || { cat $out; exit 1; }
  echo "OUT32=$o32" >> $out
done
grep -v amdgpu.ids $out
