# Same-box A/B of two builds of the product library (separate processes, alternating):
# LIBS="a.so b.so"; SCRIPT (default scripts/ablate_bwd.py) run with each of ARGSETS
# (';'-separated argument lists, default "0;0 causal").
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-libab}
: > gpurun_out/$TAG.txt
for r in 1 2 3; do
  for lib in $LIBS; do
    IFS=';' read -ra SETS <<< "${ARGSETS:-0;0 causal}"
    for a in "${SETS[@]}"; do
      echo "== $lib round $r args $a" >> gpurun_out/$TAG.txt
      MT_HIP_LIB=$lib timeout -k 10 120 python ${SCRIPT:-scripts/ablate_bwd.py} $a 2>&1 | grep -v amdgpu.ids >> gpurun_out/$TAG.txt || exit 1
    done
  done
done
cat gpurun_out/$TAG.txt
