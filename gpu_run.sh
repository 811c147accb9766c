#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = assertion failures, not a GPU fault
STAGES="${STAGES:-tests smoke bench prof}"
for s in $STAGES; do
  case $s in
    probe) timeout -k 10 120 python tools/probe/mfma_probe.py > gpurun_out/probe.log 2>&1; rc=$?;;
    tests) timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?;;
    bench2) VAESNE_DP_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench2.json 2> gpurun_out/bench2.err; rc=$?;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras > gpurun_out/prof.log 2>&1; rc=$?;;
    pmc)   timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_fetch.log 2>&1; rc=$?
           [ $rc -eq 0 ] && { timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_write.log 2>&1; rc=$?; };;
  esac
  echo "$s rc=$rc"
  ok $rc || exit $rc
  # a GPU fault inside pytest still exits 1: stop the session there
  if grep -qsE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR" gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.err gpurun_out/bench2.err; then
    echo "GPU fault reported in $s; stopping"; exit 3
  fi
done
