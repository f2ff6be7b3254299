# Round-2h: PMC of the causal v5 default and of the fp32 (config 2) kernels; default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CAUSAL=1 TAG=c3causal bash scripts/gpu_pmc.sh > /dev/null 2>&1 || { echo "causal pmc failed"; exit 1; }
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
i=0
for grp in "$G1" "$G2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "fa_fwd_generic|fa_bwd" -d gpurun_out/pmc_fp32_$i -o run --output-format csv -- python3 scripts/fp32_leg.py 5 > gpurun_out/pmc_fp32_$i.log 2>&1 || { echo "fp32 group $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_fp32_* > gpurun_out/pmc_fp32_summary.txt 2>&1
python3 scripts/pmc_traffic.py fwd_f32_c2 fa_fwd_generic gpurun_out/pmc_fp32_* > /dev/null
python3 scripts/pmc_traffic.py fwd_bf16_c3_causal "fa_fwd_bf16_v5<2, 99332, true" gpurun_out/pmc_c3causal_* > /dev/null
cp profiles/pmc_fwd_f32_c2.json profiles/pmc_fwd_bf16_c3_causal.json gpurun_out/
timeout -k 10 300 python bench.py > gpurun_out/bench_r2h.json 2> gpurun_out/bench_r2h.err
rc=$?
cat gpurun_out/bench_r2h.json
exit $rc
