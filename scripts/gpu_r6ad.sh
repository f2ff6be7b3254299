# round 6: the fp32 forward and the fused fp32 backward on the bf16 MFMA in three pieces (X3,
# the defaults): parity tests of the fp32 paths, then A/B against the fp32-MFMA forms (MT_KNOB
# 65) and the prep-kernel order (62)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ad.txt
: > $out
timeout -k 10 500 python -u -m pytest tests/test_flash_gpu.py tests/test_minitorch_gpu.py tests/test_transformer_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "fused_ring or fp32 or generic or random_fwd_bwd or multihead or transformer or config2 or oracle_golden or c1" >> $out 2>&1 || { tail -40 $out; exit 1; }
for c in nc causal; do
  MT_DIAG=1 DTYPE=fp32 ENVAB=MT_KNOB:0,65 timeout -k 10 200 python -u scripts/ab_fwd.py 0 $c 8,16,1024,64 11 >> $out 2>&1 || { tail -30 $out; exit 1; }
done
for c in "" causal; do
  MT_DIAG=1 DTYPE=fp32 SHAPE=8,16,1024,64 ROUNDS=11 ENVAB=MT_KNOB:0,65,60 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v amdgpu.ids $out | tail -16
