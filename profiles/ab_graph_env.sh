#!/bin/bash
# bench.py ms/step under graph-execution variants, interleaved A/B on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --throughput-batch 0 --no-extras --no-roofline"
for rep in 1 2; do
  for env in "X=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "VAESNE_STREAMS=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2"; do
    r=$(env $env timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])") || exit 1
    echo "$env rep$rep: $r"
  done
done
