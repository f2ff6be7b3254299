# round 6: small non-causal grids with N % 128 != 0, where the default falls to
# v4 (policy 21, 4 waves): v6's 8-wave ragged form (140:9 = 66 | 65536) and the default (0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1 REPS=20
out=gpurun_out/ab_r6o_smallgrid_ragged.txt
: > $out
for shp in 1,16,1088,64 2,16,1088,64 4,16,320,64 1,16,2112,64 2,8,4032,64; do
  timeout -k 10 200 python scripts/ab_fwd.py 0,21,140:9 nc $shp 9 >> $out 2>&1 || { cat $out; exit 1; }
done
grep -v amdgpu.ids $out
