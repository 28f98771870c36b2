#!/bin/bash
# Round 4 final tree under rocprofv3: kernel trace + stats of crc_bench's default table (FP4
# K1/K2 and K1b next to the i8 and LDS-table forms) and of the chunkserver during the driver's
# N=1 command.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/crc -o crc -- build/native/crc_bench > $O/crc_default.json 2> $O/crc_default.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --profile-dir $O/bench > $O/bench_prof.json 2> $O/bench_prof.err
