#!/bin/bash
# r06 session 12: attention dropout hash with the row key through one multiply (hoisted) and
# the key-pair mix added: full GPU suite, kernel A/B vs 8cf, step A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/s12_suite.log 2>&1; rc=$?
tail -5 gpurun_out/s12_suite.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s12_suite.log && exit 3
bash profiles/ab_roof.sh 8cf || exit 5
bash profiles/ab_pkg.sh 8cf
