#!/bin/bash
# A/B: split-f16 forward register budget for 4 waves/SIMD (wpe4, 128 VGPRs, spills 144 B) vs 3
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=$PWD/vaesne-dev_amd/lib
for rep in 1 2; do
  for lib in libvaesne_hip.so libvaesne_hip_wpe4.so; do
    VAESNE_HIP_LIB=$L/$lib timeout -k 10 200 python bench.py --roofline-only > gpurun_out/rl_$lib.json 2>/dev/null || exit 2
    python -c "import json; r=json.load(open('gpurun_out/rl_$lib.json')); r=r.get('roofline', r); print('$lib rep$rep bwd', r['detail']['bwd']['ms'], 'fwd', r['detail']['fwd']['ms'])"
  done
done
VAESNE_HIP_LIB=$L/libvaesne_hip_wpe4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sf16.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_wpe4.log 2>&1 || exit 1
bash profiles/ab_env.sh "VAESNE_HIP_LIB=$L/libvaesne_hip.so" "VAESNE_HIP_LIB=$L/libvaesne_hip_wpe4.so" || exit 4
