# PMC counter passes on the d = 128 forward at the config-4 per-GPU shard (8,16,16384,128).
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-d128}
set -- "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
       "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
       "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM" "FETCH_SIZE" "WRITE_SIZE"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_fwd -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra --shape 8 16 16384 128 > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "group $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_* > gpurun_out/pmc_${TAG}_summary.txt 2>&1
cat gpurun_out/pmc_${TAG}_summary.txt
