#!/bin/bash
# Step-level A/B of Python package variants: abpkg/<V>/VAESNe vs the working tree ("cur"),
# same libvaesne_hip.so unless abpkg/<V>/libvaesne_hip.so exists, interleaved, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in cur "$@"; do
    if [ "$V" = cur ]; then env=""; else
      lib=$PWD/vaesne-dev_amd/lib/libvaesne_hip.so; [ -f abpkg/$V/libvaesne_hip.so ] && lib=$PWD/abpkg/$V/libvaesne_hip.so
      env="VAESNE_PKG_DIR=$PWD/abpkg/$V VAESNE_HIP_LIB=$lib"; fi
    env $env timeout -k 10 180 python bench.py --no-cpu-baseline --no-roofline --throughput-batch 0 > gpurun_out/abp_$V.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abp_$V.json')); print('$V', d['ms_per_step'], d['value'])"
  done
done
