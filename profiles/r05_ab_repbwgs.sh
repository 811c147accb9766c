#!/bin/bash
# A/B: block-1 attention backward workgroup target (vaesne_attn_rep_config bwgs) 768 vs 1536 / 3072
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for bw in 768 1536 3072; do
    r=$(timeout -k 10 200 python -c "
import sys
sys.path[:0] = ['.', 'vaesne-dev_amd']
import torch, bench
from VAESNe import _lib
_lib.load()
assert _lib.lib.attn_rep_config(0, 2, 256, 1, 16, $bw, 1) == 0
sys.argv = ['bench.py', '--steps', '30', '--warmup', '5', '--no-cpu-baseline', '--throughput-batch', '0', '--no-extras', '--no-roofline']
bench.main()
" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])") || exit 1
    echo "bwgs $bw rep$rep: $r"
  done
done
