#!/bin/bash
# r05 second session: softmax peak microbench (bench --roofline-only), B=2 step stamps and
# a kernel trace of the captured B=2 step
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python bench.py --roofline-only > gpurun_out/rl.json 2> gpurun_out/rl.err || exit 2
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/b2_stamps.txt 2> gpurun_out/b2_stamps.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b2 -o run --output-format csv -- python tools/stamps.py --batch 2 --steps 10 > gpurun_out/prof_b2.log 2>&1 || exit 4
echo done
