#!/bin/bash
# r06 session 1: the split-f16 repeated-sequence attention, determinism test, then the suite + bench
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rep_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py -v -rf --maxfail=6 --timeout 300 --timeout-method thread > gpurun_out/s1_tests.log 2>&1; rc=$?
echo "targeted rc=$rc"; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s1_tests.log && exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --throughput-batch 0 > gpurun_out/s1_bench.json 2> gpurun_out/s1_bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s1_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras > gpurun_out/s1_prof.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
