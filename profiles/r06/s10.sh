#!/bin/bash
# r06 session 10: forward range scales (v' = v 2^ev, balanced q' / k'), conflict-free K image reads
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sf16.py tests/test_gpu_rep_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py tests/test_gpu_parity.py -q -rf --maxfail=4 --timeout 300 --timeout-method thread > gpurun_out/s10_tests.log 2>&1; rc=$?
tail -6 gpurun_out/s10_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s10_tests.log && exit 3
bash profiles/ab_roof.sh cf3 || exit 5
bash profiles/r06/sq.sh > gpurun_out/s10_sq.log 2>&1 || exit 7
python profiles/sq_json.py gpurun_out/s10_sq.json gpurun_out/pmc_sq1/run_counter_collection.csv gpurun_out/pmc_sq2/run_counter_collection.csv > /dev/null
python profiles/sq_show.py gpurun_out/s10_sq.json
bash profiles/ab_pkg.sh cf3
