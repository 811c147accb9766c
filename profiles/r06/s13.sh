#!/bin/bash
# r06 session 13: the next block's in_proj gradient as one three-slice kernel (y read once)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_determinism.py -q -rf --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/s13_tests.log 2>&1; rc=$?
tail -3 gpurun_out/s13_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s13_tests.log && exit 3
bash profiles/ab_pkg.sh hsh || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s13_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --throughput-batch 0 --no-extras > gpurun_out/s13_prof.log 2>&1 || exit 6
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/s13_prof/run_kernel_stats.csv")):
    if "wgrad" in r["Name"] or "dec_tail_bwd_fused" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3, 1))
PY
