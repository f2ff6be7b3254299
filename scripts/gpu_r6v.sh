# round 6: the fused fp32 backward (fa_bwd_fused_ring): parity tests, the fp32 / minitorch
# tests that route through it, and an interleaved A/B against the split ring (MT_KNOB 60) at C2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6v.txt
: > $out
timeout -k 10 500 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py tests/test_transformer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "fused_ring or fp32 or generic or random_fwd_bwd or multihead or transformer or deterministic or config2" >> $out 2>&1 || { tail -40 $out; exit 1; }
for c in "" causal; do
  MT_DIAG=1 DTYPE=fp32 SHAPE=8,16,1024,64 ROUNDS=7 ENVAB=MT_KNOB:0,60 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v amdgpu.ids $out | tail -20
