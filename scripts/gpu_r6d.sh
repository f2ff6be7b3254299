# round 6: the epilogue store tail priced: product v6<66> vs the no-O-store ablation
# (timing only), bf16 and fp32 output, same process interleaved
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=llmsys-project-flashattn_amd/minitorch/_lib
out=gpurun_out/ab_r6d_nostore.txt
: > $out
for o in bf16 f32; do
  OUT=$o timeout -k 10 200 python scripts/fwd_lib_ab.py $L/libminitorch_hip.so $L/diag/abl_fa_fwd_v6_16.so >> $out 2>&1 || { cat $out; exit 1; }
  OUT=$o SHAPE=16,16,2048,64 timeout -k 10 200 python scripts/fwd_lib_ab.py $L/libminitorch_hip.so $L/diag/abl_fa_fwd_v6_16.so >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
