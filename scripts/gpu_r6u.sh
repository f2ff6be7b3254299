# round 6: fresh PMC of the current backward kernels: the fused d = 64 pass
# (C3 non-causal and causal, with the causal dQ reduce) and the d = 128 passes at (8,16,4096,128)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp ROUNDS=1
TAG=bwd_fused_c3 REGEX=fa_bwd CMD="python3 scripts/ablate_bwd.py 0" bash scripts/gpu_pmc.sh > /dev/null || exit 1
TAG=bwd_fused_c3_causal REGEX=fa_bwd CMD="python3 scripts/ablate_bwd.py 0 causal" bash scripts/gpu_pmc.sh > /dev/null || exit 1
export SHAPE=8,16,4096,128
TAG=bwd_d128 REGEX=fa_bwd CMD="python3 scripts/ablate_bwd.py 0" bash scripts/gpu_pmc.sh > /dev/null || exit 1
TAG=bwd_d128_causal REGEX=fa_bwd CMD="python3 scripts/ablate_bwd.py 0 causal" bash scripts/gpu_pmc.sh > /dev/null || exit 1
for t in bwd_fused_c3 bwd_fused_c3_causal bwd_d128 bwd_d128_causal; do echo "== $t"; cat gpurun_out/pmc_${t}_summary.txt; done
