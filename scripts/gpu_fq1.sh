set -o pipefail
mkdir -p gpurun_out
export MT_DIAG=1
timeout -k 10 240 python -u scripts/probe_fq.py 140 8 > gpurun_out/fq_probe.txt 2>&1 &&
timeout -k 10 240 python -u scripts/probe_fq.py 142 8 causal >> gpurun_out/fq_probe.txt 2>&1 &&
ENVAB=MT_KNOB:0,8 timeout -k 10 200 python -u scripts/ab_fwd.py 140 > gpurun_out/fq_ab.txt 2>&1 &&
ENVAB=MT_KNOB:0,8,4,9 timeout -k 10 200 python -u scripts/ab_fwd.py 142 causal >> gpurun_out/fq_ab.txt 2>&1
cat gpurun_out/fq_probe.txt gpurun_out/fq_ab.txt
