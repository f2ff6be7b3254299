# PMC passes (kernel trace only, one counter group per pass) on the C3 default forward:
# HBM traffic (FETCH_SIZE, WRITE_SIZE) and MFMA busy / clock / instruction mix, folded into
# gpurun_out/pmc_fwd_bf16_c3.json by scripts/pmc_traffic.py (copy it to profiles/ to commit).
# Env: NEEDLE (kernel-name substring, default the v6 default kernel), TAG (default fwd_bf16_c3).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NEEDLE=${NEEDLE:-fa_fwd_bf16_v6<2>}
TAG=${TAG:-fwd_bf16_c3}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_fwd -d gpurun_out/pmcd_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extra > gpurun_out/pmcd_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 scripts/pmc_traffic.py $TAG "$NEEDLE" gpurun_out/pmcd_${TAG}_* && cp profiles/pmc_$TAG.json gpurun_out/
