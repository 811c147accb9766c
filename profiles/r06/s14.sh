#!/bin/bash
# r06 session 14: verdicts read two batches late: the training-loop tests, loop A/B vs hsh
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread -k "train or guard or boundary or stepgraph or dp or update or script or determinism" > gpurun_out/s14_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s14_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s14_tests.log && exit 3
bash profiles/ab_loop.sh hsh
