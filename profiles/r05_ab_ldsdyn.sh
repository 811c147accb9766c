#!/bin/bash
# A/B: split-f16 backward with LDS sized by its wave count (dynamic) vs static 8-wave LDS (ab0)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/vaesne-dev_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_sf16.py tests/test_gpu_kernels.py tests/test_gpu_stepgraph.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_lds.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in libvaesne_hip_ab0.so libvaesne_hip.so; do
    VAESNE_HIP_LIB=$L/$lib timeout -k 10 200 python bench.py --roofline-only > gpurun_out/rl_$lib.json 2>/dev/null || exit 2
    python -c "import json; r=json.load(open('gpurun_out/rl_$lib.json')); r=r.get('roofline', r); print('$lib rep$rep bwd', r['detail']['bwd']['ms'], 'fwd', r['detail']['fwd']['ms'])"
    VAESNE_HIP_LIB=$L/$lib VAESNE_STAMPS=1 timeout -k 10 200 python tools/stamps.py --batch 2 > gpurun_out/b2_$lib.txt 2>/dev/null || exit 3
    echo "$lib rep$rep b2 $(tail -1 gpurun_out/b2_$lib.txt)"
  done
done
bash profiles/ab_env.sh "VAESNE_HIP_LIB=$L/libvaesne_hip_ab0.so" "VAESNE_HIP_LIB=$L/libvaesne_hip.so" || exit 4
