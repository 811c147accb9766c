#!/bin/bash
# Step-level A/B of environment settings (tuning hooks) on one box, interleaved,
# two rounds:  profiles/ab_env.sh "" "VAESNE_ATTN_FUSED_DQ=0"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for E in "$@"; do
    env $E timeout -k 10 180 python bench.py --no-cpu-baseline --no-roofline --throughput-batch 0 > gpurun_out/abe_$i.json 2>/dev/null || { echo "variant '$E' failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abe_$i.json')); print(repr('$E'), d['ms_per_step'], d['value'])"
    i=$((i+1))
  done
done
