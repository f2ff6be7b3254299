# round 6: the d = 128 backward with the prep folded into the dQ pass (dQ pass first): d = 128
# backward tests, bitwise/diff probe against the round-4 order (MT_KNOB 54), interleaved A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r6t.txt
: > $out
timeout -k 10 400 python -u -m pytest tests/test_flash_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "d128 or padded or random_fwd_bwd" >> $out 2>&1 || { tail -30 $out; exit 1; }
MT_DIAG=1 HEAD_DIM=128 timeout -k 10 200 python -u scripts/probe_bwd_knob.py 54 >> $out 2>&1 || { tail -30 $out; exit 1; }
for c in "" causal; do
  MT_DIAG=1 SHAPE=8,16,4096,128 ROUNDS=7 ENVAB=MT_KNOB:0,54 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 $c >> $out 2>&1 || { tail -30 $out; exit 1; }
done
grep -v amdgpu.ids $out | tail -40
