# causal fused backward: the round-3 hand-off (MT_KNOB 16) against rotated walks with the
# in-kernel reduce (32), diagnostics build: bitwise check, then interleaved timing
set -e
export MT_DIAG=1
timeout -k 10 200 python -u scripts/probe_bwd_knob.py 16,32 > gpurun_out/bwdrot_probe.log 2>&1
ENVAB=MT_KNOB:16,32,16,32 ROUNDS=6 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 causal > gpurun_out/bwdrot_ab.log 2>&1
ENVAB=MT_KNOB:16,32 ROUNDS=4 timeout -k 10 200 python -u scripts/ablate_bwd.py 0 > gpurun_out/bwdrot_ab_nc.log 2>&1
