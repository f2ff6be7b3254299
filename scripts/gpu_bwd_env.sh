# Interleaved A/B of an environment knob of the default backward (ENVAB=NAME:v1,v2,..),
# non-causal and causal, then a kernel-trace profile of each arm (causal and not).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-env}
timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_$TAG.txt 2>&1 \
 && timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_$TAG.txt 2>&1
rc=$?
cat gpurun_out/ab_$TAG.txt
[ $rc -eq 0 ] || exit $rc
NAME=${ENVAB%%:*}
VALS=${ENVAB#*:}
unset ENVAB
for v in $(echo $VALS | tr , ' '); do
  for c in "" causal; do
    export $NAME=$v
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$v$c -o run --output-format csv \
      -- python3 scripts/ablate_bwd.py 0 $c > gpurun_out/prof_${TAG}_$v$c.log 2>&1 || exit 1
  done
done
