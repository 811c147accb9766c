#!/bin/bash
# SQ counter passes over bench.py --roofline-only for env variants: bash tools/sq_ab.sh "VAR=0" "VAR=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1))
  env $V true   # validate
  export $V
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d gpurun_out/sqab${i}_1 -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/sqab${i}_1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/sqab${i}_2 -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/sqab${i}_2.log 2>&1 || exit 2
  echo "=== $V"
  python profiles/sq_summary.py -k ${KEY:-attn_fwd} $(find gpurun_out/sqab${i}_1 gpurun_out/sqab${i}_2 -name "*counter_collection.csv")
done
