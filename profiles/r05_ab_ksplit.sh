#!/bin/bash
# A/B: split-f16 backward key split down to 1 wave per workgroup, target 512 workgroups
# (libvaesne_hip.so) vs down to 2 waves, target 256 (ab0)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
L=$PWD/vaesne-dev_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_sf16.py tests/test_gpu_kernels.py tests/test_gpu_stepgraph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ks.log 2>&1 || exit 1
echo "tests: $(tail -1 gpurun_out/t_ks.log)"
for rep in 1 2; do
  for lib in libvaesne_hip_ab0.so libvaesne_hip.so; do
    VAESNE_HIP_LIB=$L/$lib VAESNE_STAMPS=1 timeout -k 10 200 python tools/stamps.py --batch 2 > gpurun_out/b2_$lib.txt 2>/dev/null || exit 3
    echo "$lib rep$rep b2 $(tail -1 gpurun_out/b2_$lib.txt)"
  done
done
bash profiles/ab_env.sh "VAESNE_HIP_LIB=$L/libvaesne_hip_ab0.so" "VAESNE_HIP_LIB=$L/libvaesne_hip.so" || exit 4
