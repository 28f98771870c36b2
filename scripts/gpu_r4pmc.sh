#!/bin/bash
# Round 4: PMC counters of the production K1/K2 dispatch at 1 GiB, chunk CRCs on the i8 and on
# the FP4 matrix cores (one counter pass per form; kernel trace only, nothing else traced).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O="$R/gpurun_out/r4pmc"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && \
DFS_CRC_FP4=0 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  -d "$O/i8" -o i8 --output-format csv -- "$R/build/native/crc_bench" --single 1024 --iters 20 > "$O/i8.log" 2>&1 && \
DFS_CRC_FP4=1 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE \
  -d "$O/fp4" -o fp4 --output-format csv -- "$R/build/native/crc_bench" --single 1024 --iters 20 > "$O/fp4.log" 2>&1
