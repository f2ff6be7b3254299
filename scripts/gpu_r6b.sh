# round 6: padded-d head groups / scratch bound tests, then the fp32-output forward A/B
# (8-wave v6<66> vs the 4-wave form W4, two workgroups per CU) on the diagnostics build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_flash_gpu.py -k "padded or golden or random_fwd_bwd" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_r6b.log 2>&1
rc=$?
tail -5 gpurun_out/tests_r6b.log
[ $rc -eq 0 ] || exit $rc
MT_DIAG=1 OUT32=1 ENVAB=MT_KNOB:0,4 timeout -k 10 300 python scripts/ab_fwd.py 140 nc 8,16,4096,64 9 > gpurun_out/ab_r6b_f32out_w4.txt 2>&1 \
 && MT_DIAG=1 ENVAB=MT_KNOB:0,4 timeout -k 10 300 python scripts/ab_fwd.py 140 nc 8,16,4096,64 9 >> gpurun_out/ab_r6b_f32out_w4.txt 2>&1 \
 && MT_DIAG=1 OUT32=1 ENVAB=MT_KNOB:0,4 timeout -k 10 300 python scripts/ab_fwd.py 140 nc 4,16,8192,64 7 >> gpurun_out/ab_r6b_f32out_w4.txt 2>&1
rc=$?
cat gpurun_out/ab_r6b_f32out_w4.txt
exit $rc
