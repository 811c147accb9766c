#!/bin/bash
# r06 closing session, part B: HBM traffic passes, SQ counter passes over the roofline launches
# (sq_counters.json: bench.py's valu fields), step stamps at B = 16 and B = 2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="pmc" bash gpu_run.sh || exit $?
bash profiles/r06/sq.sh > gpurun_out/sq.log 2>&1 || exit 4
python profiles/sq_json.py gpurun_out/sq_counters.json gpurun_out/pmc_sq1/run_counter_collection.csv gpurun_out/pmc_sq2/run_counter_collection.csv > /dev/null || exit 8
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.txt 2> gpurun_out/stamps.err || exit 5
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/b2_stamps.txt 2> gpurun_out/b2_stamps.err || exit 7
echo done
