#!/bin/bash
# SQ counter passes over a short captured-step bench run (each pass its own rocprofv3
# run, at most 8 SQ counters; a failing pass ends the script):
#   bash profiles/pmc_step.sh   -> gpurun_out/pmc_step{1,2}/run_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 2 --no-cpu-baseline --throughput-batch 0 --no-extras --no-roofline"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_step1 -o run --output-format csv -- python $B > gpurun_out/pmc_step1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA -d gpurun_out/pmc_step2 -o run --output-format csv -- python $B > gpurun_out/pmc_step2.log 2>&1 || exit 2
