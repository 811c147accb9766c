#!/bin/bash
# Step-level A/B of library variants (VAESNE_HIP_LIB=vaesne-dev_amd/lib/ab/<V>.so):
# bench.py (20 timed steps, hipGraph) once per variant, interleaved, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in "$@"; do
    VAESNE_HIP_LIB=$PWD/vaesne-dev_amd/lib/ab/$V.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-roofline --throughput-batch 0 > gpurun_out/abb_$V.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abb_$V.json')); print('$V', d['ms_per_step'], d['value'])"
  done
done
