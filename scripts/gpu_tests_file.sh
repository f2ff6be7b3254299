# GPU pytest subset: FILES (default tests/test_flash_gpu.py), K (pytest -k expression, default all)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-sub}
timeout -k 10 800 python -u -m pytest ${FILES:-tests/test_flash_gpu.py} ${K:+-k "$K"} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "FAILED|Error|error" gpurun_out/tests_$TAG.log | head -20
tail -3 gpurun_out/tests_$TAG.log
exit $rc
