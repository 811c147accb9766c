#!/bin/bash
# rocprofv3 kernel trace of a short bench.py run -> gpurun_out/prof (per-step breakdown:
# python profiles/step_breakdown.py gpurun_out/prof/run_kernel_trace.csv)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras --no-roofline \
  > gpurun_out/prof.log 2>&1
