#!/bin/bash
# SQ counter passes over bench.py --roofline-only (decoder-shape attention launches), each its
# own rocprofv3 run; the counters offered by this gfx950 are listed first
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/counters_list.txt; }
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
have SQ_INSTS_MFMA && P1="$P1 SQ_INSTS_MFMA"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
have SQ_VALU_MFMA_BUSY_CYCLES && P2="$P2 SQ_VALU_MFMA_BUSY_CYCLES"
have SQ_INSTS_VALU_TRANS_F32 && P2="$P2 SQ_INSTS_VALU_TRANS_F32"
echo "pass1: $P1"; echo "pass2: $P2"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmc_sq1 -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_sq1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmc_sq2 -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_sq2.log 2>&1 || exit 2
echo sq done
