# column-reduction A/B at config 5's shapes (reduce_probe under rocprofv3, per-kernel medians)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/colab_probe -o run -- python -u scripts/reduce_probe.py > gpurun_out/colab_probe.log 2>&1
timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/colab_c5 -o run -- python -u scripts/c5_graph_probe.py 10 > gpurun_out/colab_c5.log 2>&1
