#!/bin/bash
# Round 4: journal appends through O_DIRECT (DFS_JOURNAL_DIRECT=1: the block goes from the
# registered slot to the device without a page-cache copy) vs buffered, alternating, on the
# driver's N=1 command.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_buf_a.json 2> $O/bench_buf_a.err && \
DFS_JOURNAL_DIRECT=1 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_dio_a.json 2> $O/bench_dio_a.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_buf_b.json 2> $O/bench_buf_b.err && \
DFS_JOURNAL_DIRECT=1 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_dio_b.json 2> $O/bench_dio_b.err
