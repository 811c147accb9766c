#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "decoder or tail" > gpurun_out/s23_tests.log 2>&1; rc=$?
tail -1 gpurun_out/s23_tests.log; [ $rc -le 1 ] || exit $rc
bash profiles/ab_pkg.sh fin
