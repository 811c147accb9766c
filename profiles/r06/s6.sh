#!/bin/bash
# r06 session 6: the whole GPU suite, step stamps (B=16, B=2), the script loop's host profile, SQ passes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/s6_suite.log 2>&1; rc=$?
tail -8 gpurun_out/s6_suite.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s6_suite.log && exit 3
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py > gpurun_out/s6_stamps.txt 2> gpurun_out/s6_stamps.err || exit 4
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/s6_b2_stamps.txt 2> gpurun_out/s6_b2_stamps.err || exit 5
timeout -k 10 300 python tools/b2_host_profile.py > gpurun_out/s6_b2_host.txt 2>&1 || exit 6
bash profiles/r06/sq.sh || exit 7
