#!/bin/bash
# r05 session 3: GPU suite, bench, B=2 stamps + kernel trace (small-batch decoder tail chunking)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="tests bench" bash gpu_run.sh || exit $?
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/b2_stamps.txt 2> gpurun_out/b2_stamps.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b2 -o run --output-format csv -- python tools/stamps.py --batch 2 --steps 10 > gpurun_out/prof_b2.log 2>&1 || exit 4
echo done
