# round 4: PMC passes of the d = 128 backward kernels (stall/issue breakdown, instruction mix,
# LDS bank conflicts, HBM bytes) at (8,16,4096,128)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=d128bwd REGEX=fa_bwd_d128 CMD="python3 scripts/ablate_bwd.py 0" SHAPE=8,16,4096,128 bash scripts/gpu_pmc.sh
