# PMC counter passes on the forward kernel (one rocprofv3 --pmc pass per group).
mkdir -p gpurun_out
export TMPDIR=/tmp
POL=${POL:-2}
TAG=${TAG:-p$POL}
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_fwd -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extra --policy $POL > gpurun_out/pmc_${TAG}_$i.log 2>&1 || echo "group $i failed"
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_* > gpurun_out/pmc_${TAG}_summary.txt 2>&1
cat gpurun_out/pmc_${TAG}_summary.txt
