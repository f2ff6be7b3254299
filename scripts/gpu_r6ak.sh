# round 6: the X3 split ring backward (per-k-step sums): MHA X.grad against torch fp32 (GPU and
# CPU) and float64, the GPU tests that run it, and interleaved A/B timing against the fp32-MFMA
# form (knob 65)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ak.txt
: > $out
true
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_minitorch_gpu.py -k multihead > gpurun_out/r6ak_mha.txt 2>&1; tail -15 gpurun_out/r6ak_mha.txt >> $out; MT_HIP_LIB=$PWD/llmsys-project-flashattn_amd/minitorch/_lib/diag/libminitorch_hip_diag.so MT_KNOB=65 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_minitorch_gpu.py -k multihead_attention_flash > gpurun_out/r6ak_mha65.txt 2>&1; tail -15 gpurun_out/r6ak_mha65.txt >> $out
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flash_gpu.py tests/test_minitorch_gpu.py \
  > gpurun_out/r6ak_tests.txt 2>&1 || { tail -40 gpurun_out/r6ak_tests.txt; exit 1; }
tail -2 gpurun_out/r6ak_tests.txt >> $out
export MT_DIAG=1
for sh in 8,16,1024,32 2,16,1024,64 1,4,4096,64; do
  for c in "" causal; do
    SHAPE=$sh DTYPE=fp32 ROUNDS=11 ENVAB=MT_KNOB:0,65 timeout -k 10 120 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
  done
done
grep -v -e amdgpu.ids -e Warning -e detach -e "msg.append" $out
