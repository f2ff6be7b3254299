# round 6: X3 form of the fp32 split ring backward (fa_bwd_dkv_ring / fa_bwd_dq_ring): the GPU
# tests that run it, then interleaved A/B against the fp32-MFMA form (diag knob 65)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ah.txt
: > $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_flash_gpu.py tests/test_minitorch_gpu.py \
  > gpurun_out/r6ah_tests.txt 2>&1 || { tail -40 gpurun_out/r6ah_tests.txt; exit 1; }
tail -3 gpurun_out/r6ah_tests.txt >> $out
export MT_DIAG=1
for sh in 8,16,1024,32 2,4,1024,64 1,4,4096,64 4,8,512,48; do
  for c in "" causal; do
    SHAPE=$sh DTYPE=fp32 ROUNDS=11 ENVAB=MT_KNOB:0,65 timeout -k 10 120 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
