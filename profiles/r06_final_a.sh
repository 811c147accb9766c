#!/bin/bash
# r06 closing session, part A: GPU suite, smoke, bench (1 and 2 ranks), kernel trace
cd "${GRAFT_REPO_ROOT:-.}"
STAGES="tests smoke bench bench2 prof" bash gpu_run.sh || exit $?
echo done
