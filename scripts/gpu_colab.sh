# config-5 A/B under rocprofv3 (kernel time per step): the default against MT_RIGHT_T=0
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0 1 0; do
  MT_RIGHT_T=$v timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/colab_rt$v -o run$RANDOM -- python -u scripts/c5_graph_probe.py 10 >> gpurun_out/colab_rt$v.log 2>&1
done
