#!/bin/bash
# Kernel-level A/B: bench.py --roofline-only for the working tree ("cur") and abpkg/<V> variants
# (their own libvaesne_hip.so), interleaved, two rounds; ms per kernel of the decoder-shape launches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for V in cur "$@"; do
    env=""; [ $V != cur ] && env="VAESNE_PKG_DIR=$PWD/abpkg/$V VAESNE_HIP_LIB=$PWD/abpkg/$V/libvaesne_hip.so"
    env $env timeout -k 10 150 python bench.py --roofline-only > gpurun_out/abr_$V.json 2>/dev/null || { echo "roofline $V failed"; exit 5; }
    python -c "import json; d=json.load(open('gpurun_out/abr_$V.json')); print('$V', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
  done
done
