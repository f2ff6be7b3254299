# round 6: the non-causal fused fp32 backward compiled from the causal-template code with a
# runtime causal flag of 0 (diag knob 68) against the default, C2, interleaved; bitwise check
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1
out=gpurun_out/r6as.txt
: > $out
for r in 1 2; do
  SHAPE=8,16,1024,64 DTYPE=fp32 ROUNDS=15 ENVAB=MT_KNOB:0,68 timeout -k 10 120 python -u scripts/ablate_bwd.py 0 >> $out 2>&1 || { tail -30 $out; exit 1; }
done
cat $out
