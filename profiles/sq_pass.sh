#!/bin/bash
# Two SQ counter passes over bench.py --roofline-only (each its own rocprofv3 run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES -d gpurun_out/pmc_sq1 -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_sq1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2 -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_sq2.log 2>&1 || exit 2
