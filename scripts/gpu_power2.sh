set -o pipefail
# r5 power probe of the other legs: backward C3 (causal and not), d = 128 forward and backward
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/power2.txt
PROBE_BWD=1 timeout -k 10 200 python -u scripts/power_probe.py 0 >> gpurun_out/power2.txt 2>&1 &&
PROBE_BWD=1 timeout -k 10 200 python -u scripts/power_probe.py 0 0 causal >> gpurun_out/power2.txt 2>&1 &&
timeout -k 10 200 python -u scripts/power_probe.py 0 0 causal >> gpurun_out/power2.txt 2>&1 &&
PROBE_SHAPE=8,16,4096,128 timeout -k 10 200 python -u scripts/power_probe.py 0 >> gpurun_out/power2.txt 2>&1 &&
PROBE_SHAPE=8,16,4096,128 PROBE_BWD=1 timeout -k 10 200 python -u scripts/power_probe.py 0 >> gpurun_out/power2.txt 2>&1
grep -v amdgpu.ids gpurun_out/power2.txt
