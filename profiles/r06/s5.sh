#!/bin/bash
# r06 session 5: rep backward with LDS-DMA keep words: tests, roofline A/B vs r05, step A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rep_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py -q -rf --maxfail=4 --timeout 300 --timeout-method thread > gpurun_out/s5_tests.log 2>&1; rc=$?
tail -4 gpurun_out/s5_tests.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for V in cur r05; do
    env=""; [ $V = r05 ] && env="VAESNE_PKG_DIR=$PWD/abpkg/r05 VAESNE_HIP_LIB=$PWD/abpkg/r05/libvaesne_hip.so"
    env $env timeout -k 10 150 python bench.py --roofline-only > gpurun_out/s5_roof_$V.json 2>/dev/null || { echo "roofline $V failed"; exit 5; }
    python -c "import json; d=json.load(open('gpurun_out/s5_roof_$V.json')); print('$V', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
  done
done
bash profiles/ab_pkg.sh r05 2>&1 | tee gpurun_out/s5_abpkg.txt
