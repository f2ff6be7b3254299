# PMC passes (kernel trace + one counter group per pass, no tracing domains) on one kernel:
# stall / issue breakdown, instruction mix, LDS, HBM bytes. Env: TAG, REGEX (kernel-name regex
# for --kernel-include-regex), CMD (the program after --, default the C3 bench forward).
# Summary: gpurun_out/pmc_${TAG}_summary.txt (scripts/pmc_summary.py).
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-fwd_v6}
REGEX=${REGEX:-fa_fwd}
CMD=${CMD:-"python3 bench.py --steps 3 --warmup 1 --no-cpu --no-extra"}
set -- "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
       "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
       "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA" "FETCH_SIZE" "WRITE_SIZE"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "$REGEX" -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_* > gpurun_out/pmc_${TAG}_summary.txt 2>&1
cat gpurun_out/pmc_${TAG}_summary.txt
