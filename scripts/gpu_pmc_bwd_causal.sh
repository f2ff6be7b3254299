# PMC passes on the paired causal bf16 backward at C3 -> gpurun_out/pmc_bwd_bf16_c3_causal_{dkv,dq}.json.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_bwd -d gpurun_out/pmcc_$i -o run --output-format csv -- python3 scripts/ablate_bwd.py 0 causal > gpurun_out/pmcc_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 scripts/pmc_traffic.py bwd_bf16_c3_causal_dkv "fa_bwd_dkv_bf16<true, true>" gpurun_out/pmcc_* && cp profiles/pmc_bwd_bf16_c3_causal_dkv.json gpurun_out/ \
 && python3 scripts/pmc_traffic.py bwd_bf16_c3_causal_dq "fa_bwd_dq_bf16<true, 4, false, true>" gpurun_out/pmcc_* && cp profiles/pmc_bwd_bf16_c3_causal_dq.json gpurun_out/
