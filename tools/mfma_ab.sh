#!/bin/bash
# interleaved roofline timing of the matrix-core attention variants:
#   bash tools/mfma_ab.sh 0 4 8                          (VAESNE_ATTN_MFMA_FWD)
#   VAR=VAESNE_ATTN_MFMA_BWD bash tools/mfma_ab.sh 0 4 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=${VAR:-VAESNE_ATTN_MFMA_FWD}
for rep in 1 2 3; do for V in "$@"; do
  env "$VAR=$V" timeout -k 10 120 python bench.py --roofline-only > gpurun_out/ab_m$V.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_m$V.json')); print('$VAR=$V', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
done; done
