# round 6: the fused d = 64 backward over smaller head groups (MT_FUSED_GROUP heads per launch,
# diagnostics build): does a group's partial slab staying in the Infinity Cache pay?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 ROUNDS=7
out=gpurun_out/r6y.txt
: > $out
for c in "" causal; do
  ENVAB=MT_FUSED_GROUP:128,64,32,16 timeout -k 10 300 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v amdgpu.ids $out
