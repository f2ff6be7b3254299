# Timing-only ablation libraries of the v6 forward (WRONG results): the product objects with
# fa_fwd_v6.hip rebuilt under -DV6ABL=n, into minitorch/_lib/diag/abl_fwd_n.so (CPU, no GPU).
set -e
cd "$(dirname "$0")/../llmsys-project-flashattn_amd"
make -j8 >/dev/null
mkdir -p build/abl minitorch/_lib/diag
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -fno-honor-nans -fno-slp-vectorize \
    -mllvm -amdgpu-sched-strategy=max-ilp -DV6ABL=$n -c csrc/fa_fwd_v6.hip -o build/abl/fa_fwd_v6_$n.o
  objs=$(ls build/*.o | grep -v fa_fwd_v6.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 $objs build/abl/fa_fwd_v6_$n.o -o minitorch/_lib/diag/abl_fwd_$n.so \
    -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
done
