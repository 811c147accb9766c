#!/bin/bash
# r06 session 3: split-f16 attention tests (plain + repeated), determinism, bench + trace
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rep_sf16.py tests/test_gpu_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py -v -rf --maxfail=6 --timeout 300 --timeout-method thread > gpurun_out/s3_tests.log 2>&1; rc=$?
tail -12 gpurun_out/s3_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s3_tests.log && exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --throughput-batch 0 > gpurun_out/s3_bench.json 2> gpurun_out/s3_bench.err || exit 4
python -c "import json; d=json.load(open('gpurun_out/s3_bench.json')); print(d['ms_per_step'], d['value'], d['grad_rel_err'], {k: v.get('ms') for k, v in d['roofline']['detail'].items()})"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras > gpurun_out/s3_prof.log 2>&1
