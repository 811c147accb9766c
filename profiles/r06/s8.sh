#!/bin/bash
# r06 session 8: f16-output lo splits (fma_mixlo/hi), padded V image rows: tests, roofline A/B vs cf3, step A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sf16.py tests/test_gpu_rep_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py tests/test_gpu_parity.py -q -rf --maxfail=4 --timeout 300 --timeout-method thread > gpurun_out/s8_tests.log 2>&1; rc=$?
tail -4 gpurun_out/s8_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s8_tests.log && exit 3
for rep in 1 2; do
  for V in cur cf3; do
    env=""; [ $V != cur ] && env="VAESNE_PKG_DIR=$PWD/abpkg/$V VAESNE_HIP_LIB=$PWD/abpkg/$V/libvaesne_hip.so"
    env $env timeout -k 10 150 python bench.py --roofline-only > gpurun_out/s8_roof_$V.json 2>/dev/null || { echo "roofline $V failed"; exit 5; }
    python -c "import json; d=json.load(open('gpurun_out/s8_roof_$V.json')); print('$V', {k:round(v['ms'],4) for k,v in d['detail'].items()})"
  done
done
bash profiles/ab_pkg.sh cf3 2>&1 | tee gpurun_out/s8_abpkg.txt
bash profiles/r06/sq.sh > gpurun_out/s8_sq.log 2>&1 || exit 7
python profiles/sq_json.py gpurun_out/s8_sq.json gpurun_out/pmc_sq1/run_counter_collection.csv gpurun_out/pmc_sq2/run_counter_collection.csv > /dev/null
