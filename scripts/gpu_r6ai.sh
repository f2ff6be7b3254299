# round 6: X3 split ring backward: error against float64, the MHA tests, and interleaved A/B vs
# the fp32-MFMA form (diag knob 65)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ai.txt
: > $out
MT_DIAG=1 timeout -k 10 200 python -u scripts/probe_x3_ring.py >> $out 2>&1 || { tail -30 $out; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_minitorch_gpu.py \
  > gpurun_out/r6ai_tests.txt 2>&1 || { tail -40 gpurun_out/r6ai_tests.txt; exit 1; }
tail -2 gpurun_out/r6ai_tests.txt >> $out
export MT_DIAG=1
for sh in 8,16,1024,32 2,16,1024,64; do
  for c in "" causal; do
    SHAPE=$sh DTYPE=fp32 ROUNDS=11 ENVAB=MT_KNOB:0,65 timeout -k 10 120 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
