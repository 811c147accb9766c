#!/bin/bash
# rocprofv3 kernel trace of a short bench.py run under an environment variant:
#   bash profiles/trace_env.sh TAG "VAR=1 VAR2=0"   -> gpurun_out/prof_TAG/run_kernel_trace.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
rm -rf gpurun_out/prof_$tag
env $1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras --no-roofline \
  > gpurun_out/prof_$tag.log 2>&1
