#!/bin/bash
# r06 session 22: GELU derivative from the recompute's GELU output in the fused tail backward:
# full GPU suite, bench parity line, kernel trace of the tails, step A/B vs e0
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/s22_suite.log 2>&1; rc=$?
tail -4 gpurun_out/s22_suite.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s22_suite.log && exit 3
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras --no-roofline > gpurun_out/s22_bench.json 2>/dev/null || exit 4
python -c "import json; d=json.loads(open('gpurun_out/s22_bench.json').read().strip().splitlines()[-1]); print('ms', d['ms_per_step'], 'grad_rel_err', d['grad_rel_err'], 'elbo', d['elbo_rel_err'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s22_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --throughput-batch 0 --no-extras > gpurun_out/s22_prof.log 2>&1 || exit 6
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/s22_prof/run_kernel_stats.csv")):
    if "dec_tail" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3, 1))
PY
bash profiles/ab_pkg.sh m16
