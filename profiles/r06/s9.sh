#!/bin/bash
# r06 session 9: conflict-free LDS images (forward V^T pair-word staging at a 24-dword stride,
# XOR-swizzled transposed operand images in the backward kernels): tests, kernel A/B, SQ passes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sf16.py tests/test_gpu_rep_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py tests/test_gpu_parity.py -q -rf --maxfail=4 --timeout 300 --timeout-method thread > gpurun_out/s9_tests.log 2>&1; rc=$?
tail -4 gpurun_out/s9_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s9_tests.log && exit 3
bash profiles/ab_roof.sh cf3 pad || exit 5
bash profiles/r06/sq.sh > gpurun_out/s9_sq.log 2>&1 || exit 7
python profiles/sq_json.py gpurun_out/s9_sq.json gpurun_out/pmc_sq1/run_counter_collection.csv gpurun_out/pmc_sq2/run_counter_collection.csv > /dev/null
bash profiles/ab_pkg.sh cf3
