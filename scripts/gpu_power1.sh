set -o pipefail
# r5 power probe (profiles/r5_power_probe.txt). The fp16-QK knob 8 of policy 140 it timed was removed after that measurement.
mkdir -p gpurun_out
export TMPDIR=/tmp MT_DIAG=1
ls /sys/class/drm/card*/device/hwmon/hwmon*/power1_* > gpurun_out/pw.txt 2>&1; cat /sys/class/drm/card*/device/hwmon/hwmon*/power1_cap* >> gpurun_out/pw.txt 2>&1
timeout -k 10 200 python -u scripts/power_probe.py 140 0 > gpurun_out/power1.txt 2>&1 &&
timeout -k 10 200 python -u scripts/power_probe.py 140 8 >> gpurun_out/power1.txt 2>&1 &&
for kn in 0 8; do
  MT_KNOB=$kn timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --kernel-trace --kernel-include-regex fa_fwd -d gpurun_out/pw_pmc_$kn -o run --output-format csv -- python3 scripts/ab_fwd.py 140 x 8,16,4096,64 2 > gpurun_out/pw_pmc_$kn.log 2>&1 || exit 1
done
cat gpurun_out/power1.txt gpurun_out/pw.txt
