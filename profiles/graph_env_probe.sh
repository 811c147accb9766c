#!/bin/bash
# graph_branch_probe.py under the HIP runtime's graph-execution knobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for env in "" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  echo "== $env"
  env $env timeout -k 10 60 python profiles/graph_branch_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
