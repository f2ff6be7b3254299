# round 6: the fused fp32 backward forming its own row constants (PREP, no prep launch) against
# the prep kernel ahead of it (MT_KNOB 62); parity tests first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6aa.txt
: > $out
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "fused_ring or fp32 or generic or multihead or deterministic" >> $out 2>&1 || { tail -40 $out; exit 1; }
for c in "" causal; do
  MT_DIAG=1 DTYPE=fp32 SHAPE=8,16,1024,64 ROUNDS=11 ENVAB=MT_KNOB:0,62,60 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v amdgpu.ids $out | tail -12
