# PMC passes (kernel trace only, one counter group per pass) on the config-2 fp32 forward
# (fa_fwd_generic_ring, the fp32 default) -> gpurun_out/pmc_fwd_f32_c2.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NEEDLE=${NEEDLE:-fa_fwd_generic_ring<float, 64, 2, false, true>}
TAG=${TAG:-fwd_f32_c2}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_fwd -d gpurun_out/pmcd_${TAG}_$i -o run --output-format csv -- python3 scripts/fp32_leg.py 5 > gpurun_out/pmcd_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 scripts/pmc_traffic.py $TAG "$NEEDLE" gpurun_out/pmcd_${TAG}_* && cp profiles/pmc_$TAG.json gpurun_out/
