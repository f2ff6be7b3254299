# A/B of a forward policy against the default: parity of every forward policy, then interleaved A/B at C3 and (1,16,8192).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-v6}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
   -k "fast_policies or huge_spike or spiked_rescale or variants_agree or config3 or split_keys" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_$TAG.txt
for shp in 8,16,4096,64 1,16,8192,64; do
  timeout -k 10 200 python scripts/ab_fwd.py ${POLS:-0,100} nc $shp 7 >> gpurun_out/ab_$TAG.txt 2>&1 || exit 1
done
cat gpurun_out/ab_$TAG.txt
