# Quick forward-policy check: the parity tests of the policies in $POLS, then interleaved A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-quick}
KEXPR=$(python3 -c "import sys; print(' or '.join(f'policies_vs_oracle[{p}] or [{p}-64] or keys_vs_oracle[{p}] or pairs_vs_oracle[{p}]' for p in sys.argv[1].split(',')))" ${POLS:-0})
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
   -k "$KEXPR" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_$TAG.txt
for shp in ${SHAPES:-8,16,4096,64 1,16,8192,64}; do
  timeout -k 10 200 python scripts/ab_fwd.py ${POLS:-0} ${MODE:-nc} $shp 7 >> gpurun_out/ab_$TAG.txt 2>&1 || exit 1
done
cat gpurun_out/ab_$TAG.txt
