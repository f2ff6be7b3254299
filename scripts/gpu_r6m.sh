# round 6: d = 128 forward O stores non-temporal (product) vs plain (abl_fa_fwd_d128v2_0.so)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=llmsys-project-flashattn_amd/minitorch/_lib
out=gpurun_out/ab_r6m_nt_d128.txt
: > $out
for cfg in "bf16 8,16,16384,128 3" "bf16 8,16,4096,128 20" "f32 8,16,4096,128 20"; do
  set -- $cfg
  OUT=$1 SHAPE=$2 REPS=$3 timeout -k 10 300 python scripts/fwd_lib_ab.py $L/libminitorch_hip.so $L/diag/abl_fa_fwd_d128v2_0.so >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
