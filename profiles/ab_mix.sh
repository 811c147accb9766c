#!/bin/bash
# Step-level A/B mixing environment variants of the working tree with package
# variants abpkg/<V>: arguments are "env:<VAR=VAL ...>" or "pkg:<V>"; interleaved, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for A in "$@"; do
    case $A in
      env:*) env=${A#env:};;
      pkg:*) V=${A#pkg:}; lib=$PWD/vaesne-dev_amd/lib/libvaesne_hip.so
             [ -f abpkg/$V/libvaesne_hip.so ] && lib=$PWD/abpkg/$V/libvaesne_hip.so
             env="VAESNE_PKG_DIR=$PWD/abpkg/$V VAESNE_HIP_LIB=$lib";;
    esac
    env $env timeout -k 10 180 python bench.py --no-cpu-baseline --no-roofline --throughput-batch 0 --no-extras > gpurun_out/abm_$i.json 2>/dev/null || { echo "variant '$A' failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abm_$i.json')); print(repr('$A'), d['ms_per_step'], d['value'])"
    i=$((i+1))
  done
done
