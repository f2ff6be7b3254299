# round 6: confirmation of the v6 non-temporal O stores (product) against plain stores
# (abl_fa_fwd_v6_0.so, -DV6NT=0) over more shapes, causal included
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=llmsys-project-flashattn_amd/minitorch/_lib
out=gpurun_out/ab_r6n_nt_confirm.txt
: > $out
for cfg in "f32 8,16,4096,64 0" "bf16 8,16,4096,64 0" "f32 8,16,4096,64 1" "bf16 8,16,4096,64 1" "f32 4,16,8192,64 0" "f32 2,16,16384,64 0" "f32 16,16,2048,64 0"; do
  set -- $cfg
  OUT=$1 SHAPE=$2 CAUSAL=$3 ROUNDS=15 timeout -k 10 300 python scripts/fwd_lib_ab.py $L/libminitorch_hip.so $L/diag/abl_fa_fwd_v6_0.so >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
out2=gpurun_out/ab_r6n_bwd_nt.txt
: > $out2
for c in 0 1; do
  CAUSAL=$c timeout -k 10 300 python scripts/bwd_lib_ab.py $L/libminitorch_hip.so $L/diag/abl_fa_bwd_fused_1.so >> $out2 2>&1 || { cat $out2; exit 1; }
done
grep -v amdgpu.ids $out2
