#!/bin/bash
# Round 4: how the chunkserver's host threads wait for the device (DFS_HIP_SYNC: the runtime's
# default vs block = sleep until the completion interrupt), on config 5's sustained PUT (cores
# per process, user vs system) and on the driver's N=1 command (latency).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 400 python bench_configs.py config5 --gpu 0 --phase-seconds 5 --parquet-rows 10000 > $O/config5_default.json 2> $O/config5_default.err && \
DFS_HIP_SYNC=block timeout -k 10 400 python bench_configs.py config5 --gpu 0 --phase-seconds 5 --parquet-rows 10000 > $O/config5_block.json 2> $O/config5_block.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err && \
DFS_HIP_SYNC=block timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_block.json 2> $O/bench_block.err
