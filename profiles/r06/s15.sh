#!/bin/bash
# r06 session 15: query-chunked split-f16 backward for few (sequence, head) pairs, the WN
# weight-gradient kernel, verdicts two batches late: full GPU suite, step / loop A/B vs hsh,
# B = 2 and B = 16 stamps
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/s15_suite.log 2>&1; rc=$?
tail -3 gpurun_out/s15_suite.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s15_suite.log && exit 3
bash profiles/ab_pkg.sh hsh || exit 5
bash profiles/ab_loop.sh hsh || exit 6
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/s15_b2_stamps.txt 2> gpurun_out/s15_b2_stamps.err || exit 7
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py > gpurun_out/s15_stamps.txt 2> gpurun_out/s15_stamps.err || exit 8
grep -E "self_bwd|update" gpurun_out/s15_b2_stamps.txt gpurun_out/s15_stamps.txt
