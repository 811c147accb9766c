#!/bin/bash
# SQ counter passes over a short full training step (bench.py, 2 timed steps): every kernel of
# the step, each pass its own rocprofv3 run
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32"
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --throughput-batch 0 --no-graph --no-extras"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc_st1 -o run --output-format csv -- $B > gpurun_out/pmc_st1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc_st2 -o run --output-format csv -- $B > gpurun_out/pmc_st2.log 2>&1 || exit 2
echo sq step done
python profiles/sq_kernels.py gpurun_out/pmc_st1/run_counter_collection.csv gpurun_out/pmc_st2/run_counter_collection.csv > gpurun_out/sq_step.txt
