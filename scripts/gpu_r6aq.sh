# round 6: fused fp32 backward, X3 form with K read from the Kᵀ image and fresh per-k-step dK/dV
# sums (the non-causal launch on the causal-template code): tests, accuracy on the MHA inputs,
# interleaved A/B against the fp32-MFMA form (knob 65)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6aq.txt
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_flash_gpu.py tests/test_minitorch_gpu.py \
  > gpurun_out/r6aq_tests.txt 2>&1 || { tail -40 gpurun_out/r6aq_tests.txt; exit 1; }
tail -1 gpurun_out/r6aq_tests.txt >> $out
MT_DIAG=1 MHA=8,1024,1024,16 timeout -k 10 300 python -u scripts/probe_x3_ring2.py >> $out 2>&1 || { tail -30 $out; exit 1; }
MT_DIAG=1 timeout -k 10 200 python -u scripts/probe_x3_ring.py >> $out 2>&1 || { tail -30 $out; exit 1; }
export MT_DIAG=1
for c in "" causal; do
  SHAPE=8,16,1024,64 DTYPE=fp32 ROUNDS=15 ENVAB=MT_KNOB:0,65 timeout -k 10 120 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v -e amdgpu.ids -e Warning -e detach -e "msg.append" $out
