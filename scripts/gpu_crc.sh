#!/bin/bash
# CRC kernel session: kernel tests, kernel-only microbenchmark (MFMA vs LDS tables),
# then one PMC pass and one kernel-trace pass over a short crc_bench run.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_replication.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k.log 2>&1 && \
timeout -k 10 300 build/native/crc_bench --iters 50 > gpurun_out/crc_bench.json 2> gpurun_out/crc_bench.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
   SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU \
   -d "$R/gpurun_out/pmc_crc" -o crc --output-format csv -- "$R/build/native/crc_bench" --iters 5 --mib 256 \
   > "$R/gpurun_out/pmc_crc.log" 2>&1) && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$R/gpurun_out/trace_crc" -o crc -- "$R/build/native/crc_bench" --iters 10 --mib 256 \
   > "$R/gpurun_out/trace_crc.log" 2>&1)
echo "gpu_crc rc=$?"
