# round 4: PMC passes of the one-wave-per-SIMD d = 128 backward at (8,16,4096,128)
# (KNOB: the diagnostics knob, default 0 = the product form)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
export MT_DIAG=1 MT_KNOB=${KNOB:-0} ROUNDS=1 SHAPE=8,16,4096,128
TAG=${TAG:-d128w} REGEX=d128w CMD="python3 scripts/ablate_bwd.py 0" bash scripts/gpu_pmc.sh
