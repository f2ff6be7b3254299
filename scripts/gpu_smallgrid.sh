set -o pipefail
# r5: small-grid d = 64 shapes: the default (v5 split / v5 4-wave / v4) against v6 forms
mkdir -p gpurun_out
export MT_DIAG=1
: > gpurun_out/smallgrid.txt
for shp in 1,8,4096,64 2,4,2048,64 1,4,8192,64 4,8,1024,64 1,16,2048,64; do
  timeout -k 10 120 python -u scripts/ab_fwd.py 0,105,140 x $shp 5 >> gpurun_out/smallgrid.txt 2>&1 || exit 1
  ENVAB=MT_KNOB:0,4 timeout -k 10 120 python -u scripts/ab_fwd.py 140 x $shp 5 >> gpurun_out/smallgrid.txt 2>&1 || exit 1
  ENVAB=MT_KNOB:0,4 timeout -k 10 120 python -u scripts/ab_fwd.py 142 causal $shp 5 >> gpurun_out/smallgrid.txt 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/ab_fwd.py 0 causal $shp 5 >> gpurun_out/smallgrid.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/smallgrid.txt
