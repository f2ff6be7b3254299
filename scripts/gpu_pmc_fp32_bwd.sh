# PMC passes on the config-2 fp32 backward ring kernels (fa_bwd_ring.hip) ->
# gpurun_out/pmc_bwd_f32_c2_{dkv,dq}.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex ring -d gpurun_out/pmcb_f32_$i -o run --output-format csv -- python3 scripts/fp32_leg.py 5 > gpurun_out/pmcb_f32_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 scripts/pmc_traffic.py bwd_f32_c2_dkv "fa_bwd_dkv_ring<false" gpurun_out/pmcb_f32_* && cp profiles/pmc_bwd_f32_c2_dkv.json gpurun_out/ \
 && python3 scripts/pmc_traffic.py bwd_f32_c2_dq "fa_bwd_dq_ring<false" gpurun_out/pmcb_f32_* && cp profiles/pmc_bwd_f32_c2_dq.json gpurun_out/
