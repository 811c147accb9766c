#!/bin/bash
# interleaved roofline timing of VAESNE_ATTN_MFMA_FWD variants: bash tools/mfma_ab.sh 0 4 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do for V in "$@"; do
  VAESNE_ATTN_MFMA_FWD=$V timeout -k 10 120 python bench.py --roofline-only > gpurun_out/ab_m$V.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_m$V.json')); print('mfma=$V', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
done; done
