# round 4: the 4-wave-workgroup v6 (knob 4, spill-free) against the default, 15 interleaved rounds at C3 and three other grids
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4m}
: > gpurun_out/ab_w4_$TAG.txt
for sh in 8,16,4096,64 4,16,4096,64 16,16,4096,64 2,16,8192,64; do
  echo "shape $sh" >> gpurun_out/ab_w4_$TAG.txt
  SHAPE=$sh ROUNDS=15 MT_DIAG=1 ENVAB=MT_KNOB:0,4 timeout -k 10 300 python scripts/ablate.py 140 >> gpurun_out/ab_w4_$TAG.txt 2>&1 || { echo "A/B $sh failed"; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ab_w4_$TAG.txt
echo "causal (policy 142): 0 default, 4 W4, 5 no V reuse, 6 W4 + no V reuse" >> gpurun_out/ab_w4_$TAG.txt
ROUNDS=15 MT_DIAG=1 ENVAB=MT_KNOB:0,4,5,6 timeout -k 10 300 python scripts/ablate.py 142 causal >> gpurun_out/ab_w4_$TAG.txt 2>&1 || { echo "causal A/B failed"; exit 1; }
tail -5 gpurun_out/ab_w4_$TAG.txt
