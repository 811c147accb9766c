#!/bin/bash
# r05 closing session, part B: HBM traffic passes, SQ counter passes (attention; all kernels
# over three captured steps), step stamps at B = 16 and B = 2
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="pmc" bash gpu_run.sh || exit $?
bash profiles/sq_pass.sh || exit 4
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc_sq3 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-extras --throughput-batch 0 > gpurun_out/pmc_sq3.log 2>&1 || exit 6
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py > gpurun_out/stamps.txt 2> gpurun_out/stamps.err || exit 5
VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/b2_stamps.txt 2> gpurun_out/b2_stamps.err || exit 7
echo done
