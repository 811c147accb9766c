#!/bin/bash
# r04 closing profile session (one gpurun call)
cd "${GRAFT_REPO_ROOT:-.}"
STAGES="tests smoke bench bench2 prof pmc" bash gpu_run.sh || exit $?
bash profiles/sq_pass.sh || exit 4
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.txt 2> gpurun_out/stamps.err || exit 5
echo done
