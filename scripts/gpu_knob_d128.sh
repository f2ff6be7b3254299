# d = 128 forward key-walk order A/B (MT_KNOB 4, diagnostics library): numerics, interleaved
# timing at the C4 shard, and HBM traffic per launch (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${SHAPE:-8,16,16384,128}
MT_KNOBS=0,4 timeout -k 10 300 python -u scripts/probe_knob_fwd.py $S > gpurun_out/knob_d128.txt 2>&1 || exit 1
MT_DIAG=1 ENVAB=MT_KNOB:0,4 timeout -k 10 300 python -u scripts/ab_fwd.py 0 nc $S 5 >> gpurun_out/knob_d128.txt 2>&1 || exit 1
for kn in 0 4; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    MT_KNOBS=$kn timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex d128 \
      -d gpurun_out/pmc_knob${kn}_$grp -o run --output-format csv -- python3 scripts/probe_knob_fwd.py $S 3 \
      > gpurun_out/pmc_knob${kn}_$grp.log 2>&1 || { echo "pmc $kn $grp failed"; exit 1; }
  done
done
python3 scripts/pmc_summary.py gpurun_out/pmc_knob0_* > gpurun_out/pmc_knob0_summary.txt 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmc_knob4_* > gpurun_out/pmc_knob4_summary.txt 2>&1
cat gpurun_out/knob_d128.txt gpurun_out/pmc_knob0_summary.txt gpurun_out/pmc_knob4_summary.txt
