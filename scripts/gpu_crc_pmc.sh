#!/bin/bash
# Two PMC passes over a short crc_bench run (defaults: scrub on the 3-buffer register ring):
# LDS/VALU counters, then matrix-core busy cycles against GPU-active cycles. Each pass is
# its own rocprofv3 run within the per-block counter limits.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
   SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU \
   -d "$R/gpurun_out/pmc_crc" -o crc --output-format csv -- "$R/build/native/crc_bench" --iters 5 --mib 256 \
   > "$R/gpurun_out/pmc_crc.log" 2>&1) && \
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES \
   SQ_WAVES GRBM_GUI_ACTIVE -d "$R/gpurun_out/pmc_mfma" -o crc --output-format csv -- "$R/build/native/crc_bench" \
   --iters 5 --mib 256 > "$R/gpurun_out/pmc_mfma.log" 2>&1)
echo "gpu_crc_pmc rc=$?"
