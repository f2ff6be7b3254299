# round 6: bench with the fp32-O headline, its kernel trace on the same lease and the PMC
# passes of the fp32-O headline kernel (profiles/pmc_fwd_bf16_c3_f32out.json)
set -o pipefail
TAG=${1:-r6k}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
       -- python3 bench.py --steps 2000 --warmup 20 --no-cpu --no-extra > gpurun_out/prof_$TAG.log 2>&1
rc=$?
cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex fa_fwd_bf16_v6 -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-extra > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo pmc done
