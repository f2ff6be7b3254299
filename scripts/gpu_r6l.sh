# round 6: non-temporal O stores (abl_fa_fwd_v6_1.so, -DV6NT=1) against the product library,
# fp32 and bf16 O, C3 and (16,16,2048,64), same process interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=llmsys-project-flashattn_amd/minitorch/_lib
out=gpurun_out/ab_r6l_nt.txt
: > $out
for o in f32 bf16; do
  for shp in 8,16,4096,64 16,16,2048,64; do
    OUT=$o SHAPE=$shp timeout -k 10 200 python scripts/fwd_lib_ab.py $L/libminitorch_hip.so $L/diag/abl_fa_fwd_v6_1.so >> $out 2>&1 || { cat $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
