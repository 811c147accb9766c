#!/bin/bash
# Step-level A/B of environment settings: bench.py (20 timed steps, hipGraph) once per
# setting, interleaved, two rounds.  Each argument is one setting, e.g.
#   profiles/ab_env_list.sh "VAESNE_REP_ATTN=0" "VAESNE_REP=0,4,256,1,16,768"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for S in "$@"; do
    i=$((i + 1))
    env $S timeout -k 10 180 python bench.py --no-cpu-baseline --no-roofline --throughput-batch 0 --no-extras > gpurun_out/abe_$i.json 2>/dev/null || { echo "setting $S failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abe_$i.json')); print('$S', d['ms_per_step'], d['value'])"
  done
done
