# round 4: C5 step with rocBLAS (default) vs the library's own GEMM, alternating
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4q}
: > gpurun_out/c5_gemm_$TAG.txt
for r in 1 2; do
  for g in rocblas own; do
    echo "== $g" >> gpurun_out/c5_gemm_$TAG.txt
    MT_GEMM=$g timeout -k 10 300 python scripts/mt_step_bench.py 20 >> gpurun_out/c5_gemm_$TAG.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/c5_gemm_$TAG.txt
MT_GEMM=own timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof_own_$TAG -o c5 -- python3 scripts/mt_step_bench.py 10 > gpurun_out/c5prof_own_$TAG.log 2>&1; echo rocprof rc=$?
