# round 4: the one-wave-per-SIMD d = 128 backward as the product form: parity (product library),
# then A/B against the two-wave form (knob 34) and without pairing (knob 1)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r4w}
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "d128 or random_fwd_bwd" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_d128_$TAG.log 2>&1; rc=$?; grep -E "FAILED|Error|passed|failed|assert" gpurun_out/tests_d128_$TAG.log | tail -8; [ $rc -eq 0 ] || exit $rc
SHAPE=8,16,4096,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,34 timeout -k 10 300 python scripts/ablate_bwd.py 0 > gpurun_out/ab_d128_$TAG.txt 2>&1 && SHAPE=8,16,4096,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,34,1 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128_$TAG.txt 2>&1 && SHAPE=4,32,1100,128 ROUNDS=6 MT_DIAG=1 ENVAB=MT_KNOB:0,34 timeout -k 10 300 python scripts/ablate_bwd.py 0 causal >> gpurun_out/ab_d128_$TAG.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_d128_$TAG.txt; exit $rc
