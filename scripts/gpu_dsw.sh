# dS-image half swizzle: bitwise check against the previous build, then interleaved timing
set -e
mkdir -p gpurun_out
D=llmsys-project-flashattn_amd/minitorch/_lib
MT_HIP_LIB=$D/diag/before_dsw.so timeout -k 10 120 python -u scripts/bwd_dump.py /tmp/before.pt > gpurun_out/dsw_cmp.log 2>&1
MT_HIP_LIB=$D/libminitorch_hip.so timeout -k 10 120 python -u scripts/bwd_dump.py /tmp/after.pt cmp /tmp/before.pt >> gpurun_out/dsw_cmp.log 2>&1
LIBS="$D/diag/before_dsw.so $D/libminitorch_hip.so" TAG=dsw_ab timeout -k 10 500 bash scripts/gpu_lib_ab.sh > /dev/null 2>&1
