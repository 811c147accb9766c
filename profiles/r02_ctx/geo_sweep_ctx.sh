#!/bin/bash
# batch-stacked encoder context attention (B=64 x 983 tokens) under forced geometries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for geo in auto "256,2" "128,2" "64,2" "256,1" "128,1" "64,1"; do
  if [ "$geo" = auto ]; then e=""; else e="VAESNE_ATTN_GEO=$geo"; fi
  echo "geo $geo: $(env $e timeout -k 10 100 python profiles/r02_ctx/ctx_attn_bench.py 2>&1 | tail -1)" || exit 1
done
