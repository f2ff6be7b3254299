# eager config-5 step, host-side A/B: the package in abtmp/old against the tree's, alternating
set -e
for r in 1 2 3; do
  MT_PKG_ROOT=$PWD/abtmp/old/llmsys-project-flashattn_amd timeout -k 10 120 python -u scripts/mt_step_bench.py 10 >> gpurun_out/c5host_old.log 2>&1
  timeout -k 10 120 python -u scripts/mt_step_bench.py 10 >> gpurun_out/c5host_new.log 2>&1
done
