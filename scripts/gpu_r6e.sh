# round 6: d = 128 forward with reversed key walks on odd rounds (VAR 512): parity, same-box
# A/B against the forward walk (diagnostics policy 130 = VAR 0), FETCH/WRITE PMC of both
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DIAG=$PWD/llmsys-project-flashattn_amd/minitorch/_lib/diag/libminitorch_hip_diag.so
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py tests/test_config4_gpu.py -k "d128 or config4 or c4 or spike or huge" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_r6e.log 2>&1
rc=$?
tail -3 gpurun_out/tests_r6e.log
[ $rc -eq 0 ] || exit $rc
MT_DIAG=1 REPS=3 timeout -k 10 300 python scripts/ab_fwd.py 0,130 nc 8,16,16384,128 9 > gpurun_out/ab_r6e_d128rev.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab_r6e_d128rev.txt
for pol in 0 130; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    MT_HIP_LIB=$DIAG timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex d128v2 -d gpurun_out/pmc_r6e_p${pol}_$grp -o run --output-format csv -- python3 bench.py --shape 8 16 16384 128 --steps 3 --warmup 1 --no-cpu --no-extra --policy $pol > gpurun_out/pmc_r6e_p${pol}_$grp.log 2>&1 || { echo "pmc $pol $grp failed"; tail -5 gpurun_out/pmc_r6e_p${pol}_$grp.log; exit 1; }
  done
  python3 scripts/pmc_traffic.py c4shard_p$pol d128v2 gpurun_out/pmc_r6e_p${pol}_* > gpurun_out/pmc_r6e_p$pol.txt 2>&1
  cat gpurun_out/pmc_r6e_p$pol.txt
done
