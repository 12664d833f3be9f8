cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for env in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "HIP_FORCE_DEV_KERNARG=1"; do
  env $env timeout -k 10 120 python scripts/probe_graph_launch.py 12 >> gpurun_out/probe_launch.log 2>&1 || exit 1
done
