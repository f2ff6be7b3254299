# round 6: X3 split ring backward with per-k-step sums: MHA X.grad against torch fp32 / float64,
# per-tensor errors on the MHA test's inputs (B=2: split ring; B=8: fused ring), the GPU tests
# that run it, and interleaved A/B timing against the fp32-MFMA form (knob 65)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6aj.txt
: > $out
MT_DIAG=1 KNOBS=0,65 timeout -k 10 300 python -u scripts/probe_mha_x3.py >> $out 2>&1 || { tail -30 $out; exit 1; }
MT_DIAG=1 BATCH=2 timeout -k 10 300 python -u scripts/probe_x3_ring2.py >> $out 2>&1 || { tail -30 $out; exit 1; }
MT_DIAG=1 BATCH=8 timeout -k 10 300 python -u scripts/probe_x3_ring2.py >> $out 2>&1 || { tail -30 $out; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_gpu.py tests/test_minitorch_gpu.py \
  > gpurun_out/r6aj_tests.txt 2>&1 || { tail -40 gpurun_out/r6aj_tests.txt; exit 1; }
tail -2 gpurun_out/r6aj_tests.txt >> $out
export MT_DIAG=1
for sh in 8,16,1024,32 2,16,1024,64; do
  for c in "" causal; do
    SHAPE=$sh DTYPE=fp32 ROUNDS=11 ENVAB=MT_KNOB:0,65 timeout -k 10 120 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
  done
done
grep -v -e amdgpu.ids -e Warning -e detach -e "msg.append" $out
