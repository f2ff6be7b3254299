# Reproduce tests/native/bin/capi_asan on the GPU box with its full stdout/stderr kept.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export ASAN_OPTIONS=${ASAN_OPTIONS:-detect_leaks=1:verify_asan_link_order=0:abort_on_error=0}
export LSAN_OPTIONS=suppressions=$PWD/tests/native/lsan.supp
timeout -k 10 300 tests/native/bin/capi_asan > gpurun_out/asan_stdout.txt 2> gpurun_out/asan_stderr.txt
rc=$?
echo "asan rc=$rc"
grep -n "ERROR\|SUMMARY" gpurun_out/asan_stderr.txt || true
exit 0
