#!/bin/bash
# A/B: block-1 attention backward: ab0 (committed), G (G accumulated over feature pairs: full-pair
# packed FMAs), GQ (G + duplicated Q rows for the score and dK chains)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=$PWD/vaesne-dev_amd/lib
for lib in libvaesne_hip_G.so libvaesne_hip_GQ.so; do
  VAESNE_HIP_LIB=$L/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_rep_attention.py tests/test_gpu_stepgraph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$lib.log 2>&1 || exit 1
  echo "$lib tests: $(tail -1 gpurun_out/t_$lib.log)"
done
for rep in 1 2; do
  for lib in libvaesne_hip_ab0.so libvaesne_hip_G.so libvaesne_hip_GQ.so; do
    VAESNE_HIP_LIB=$L/$lib timeout -k 10 200 python bench.py --roofline-only > gpurun_out/rl_$lib.json 2>/dev/null || exit 2
    python -c "import json; r=json.load(open('gpurun_out/rl_$lib.json')); r=r.get('roofline', r); print('$lib rep$rep rep_bwd', r['detail']['rep_bwd']['ms'], 'rep_fwd', r['detail']['rep_fwd']['ms'])"
  done
done
bash profiles/ab_env.sh "VAESNE_HIP_LIB=$L/libvaesne_hip_ab0.so" "VAESNE_HIP_LIB=$L/libvaesne_hip_G.so" "VAESNE_HIP_LIB=$L/libvaesne_hip_GQ.so" || exit 4
