#!/bin/bash
# r06 session 19: torch-AdamW updater steady-state fast path (one host tensor of step counts):
# optimizer / loop tests, loop A/B vs m16
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_optim.py tests/test_gpu_stepgraph.py tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_boundary.py -q -rf --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/s19_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s19_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s19_tests.log && exit 3
bash profiles/ab_loop.sh m16
timeout -k 10 300 python tools/b2_host_profile.py > gpurun_out/s19_b2_host.txt 2>&1; head -6 gpurun_out/s19_b2_host.txt
