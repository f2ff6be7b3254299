# Timing-only ablation libraries (WRONG results): the product objects with one source rebuilt
# under -D<MACRO>=n, into minitorch/_lib/diag/abl_<src>_n.so (CPU, no GPU).
# usage: scripts/build_abl.sh SRC MACRO n [n ...]   e.g. scripts/build_abl.sh fa_bwd_fused BWDABL 1 2
set -e
cd "$(dirname "$0")/../llmsys-project-flashattn_amd"
src=$1; macro=$2; shift 2
make -j8 >/dev/null
flags=$(make -pn 2>/dev/null | grep -E "^build/$src.o: EXTRA_FLAGS" | head -1 | sed 's/.*:= //')
mkdir -p build/abl minitorch/_lib/diag
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags \
    -D$macro=$n -c csrc/$src.hip -o build/abl/${src}_$n.o
  objs=$(ls build/*.o | grep -v "build/$src.o")
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 $objs build/abl/${src}_$n.o -o minitorch/_lib/diag/abl_${src}_$n.so \
    -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
done
