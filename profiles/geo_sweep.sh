#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for geo in "256,2" "128,2" "64,2" "256,1" "128,1" "256,4" "128,4" "64,4"; do
  VAESNE_ATTN_GEO=$geo timeout -k 10 120 python bench.py --roofline-only > gpurun_out/geo_$geo.json 2> gpurun_out/geo_$geo.err || { echo "geo $geo failed rc=$?"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/geo_$geo.json')); print('$geo', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
done
