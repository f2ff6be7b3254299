# round 6: the fp32 forward with its products on the bf16 MFMA in three pieces per operand
# (X3, MT_KNOB 63 = 32-key slots, 64 = 64-key slots) against the fp32-MFMA ring (knob 0): errors
# against the C oracle on every C2 head, then interleaved timing at C2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ac.txt
: > $out
for c in "" causal; do
  DTYPE=fp32 MT_KNOBS=0,63,64 timeout -k 10 300 python -u scripts/probe_knob_fwd.py 8,16,1024,64 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
  DTYPE=fp32 MT_KNOBS=0,63 timeout -k 10 300 python -u scripts/probe_knob_fwd.py 2,3,1000,48 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
for c in nc causal; do
  MT_DIAG=1 DTYPE=fp32 ENVAB=MT_KNOB:0,63,64 timeout -k 10 200 python -u scripts/ab_fwd.py 0 $c 8,16,1024,64 11 >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v amdgpu.ids $out
