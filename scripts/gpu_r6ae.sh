# round 6: accuracy and bias of the X3 fp32 forms against the fp32-MFMA forms and the C oracle
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6ae.txt
: > $out
for shp in 8,16,1024,64 4,16,4096,64; do
  for c in "" causal; do
    echo "== $shp $c" >> $out
    timeout -k 10 300 python -u scripts/probe_x3_bias.py $shp $c >> $out 2>&1 || { tail -30 $out; exit 1; }
  done
done
grep -v amdgpu.ids $out
