#!/bin/bash
# interleaved A/B of bench.py ms/step under environment variants given as arguments:
#   bash profiles/ab_env.sh "X=0" "VAESNE_PREFETCH_DROPOUT=0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS="${AB_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --throughput-batch 0 --no-extras --no-roofline}"
for rep in 1 2 3; do
  for env in "$@"; do
    r=$(env $env timeout -k 10 200 python bench.py $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])") || exit 1
    echo "$env rep$rep: $r"
  done
done
