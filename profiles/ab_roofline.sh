#!/bin/bash
# A/B timing of library variants (VAESNE_HIP_LIB) on the roofline launches, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in "$@"; do
    VAESNE_HIP_LIB=$PWD/vaesne-dev_amd/lib/ab/$V.so timeout -k 10 120 python bench.py --roofline-only > gpurun_out/ab_$V.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$V.json')); print('$V', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
  done
done
