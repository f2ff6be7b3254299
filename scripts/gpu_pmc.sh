# PMC counter passes on the forward kernel (one rocprofv3 --pmc pass per group, kernel
# trace only: never combined with sys/runtime tracing).
# Env: POL (kernel policy, default 0), TAG (output tag), CAUSAL=1 for the causal leg,
#      PMC_GROUPS=all|sq|traffic (sq = the three SQ passes, traffic = FETCH_SIZE and WRITE_SIZE).
mkdir -p gpurun_out
export TMPDIR=/tmp
POL=${POL:-0}
TAG=${TAG:-p$POL}
EXTRA=""
[ "${CAUSAL:-0}" = "1" ] && EXTRA="--causal"
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM"
if [ "${PMC_GROUPS:-all}" = "sq" ]; then
  set -- "$SQ1" "$SQ2" "$SQ3"
elif [ "${PMC_GROUPS:-all}" = "traffic" ]; then
  set -- "FETCH_SIZE" "WRITE_SIZE"
else
  set -- "$SQ1" "$SQ2" "$SQ3" "FETCH_SIZE" "WRITE_SIZE"
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_fwd -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extra --policy $POL $EXTRA > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "group $i failed"; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_* > gpurun_out/pmc_${TAG}_summary.txt 2>&1
cat gpurun_out/pmc_${TAG}_summary.txt
