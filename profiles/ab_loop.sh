#!/bin/bash
# The unchanged script's loop (bench.py training_step_script: captured B = 16, eager, B = 2)
# for the working tree ("cur") and abpkg/<V> package variants, interleaved, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for V in cur "$@"; do
    env=""; [ $V != cur ] && env="VAESNE_PKG_DIR=$PWD/abpkg/$V VAESNE_HIP_LIB=$PWD/abpkg/$V/libvaesne_hip.so"
    env $env timeout -k 10 300 python -c "
import json, torch, bench
r = bench.training_step_script(torch.device('cuda:0'))
print(json.dumps({k: r[k]['ms_per_step'] for k in ('captured', 'eager', 'b2')}))" > gpurun_out/abl_$V.json 2>/dev/null || { echo "variant $V failed"; exit 1; }
    echo "$V $(cat gpurun_out/abl_$V.json)"
  done
done
