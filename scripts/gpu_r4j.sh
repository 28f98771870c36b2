#!/bin/bash
# Round 4: where the journal runs' extra time per step goes (closing sync vs between phases),
# 8-part journal vs per-file, the driver's N=1 command.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j4.json 2> $O/bench_j4.err && \
DFS_JOURNAL_PARTS=8 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j8.json 2> $O/bench_j8.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
DFS_JOURNAL_ZERO_FILL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j4_nofill.json 2> $O/bench_j4_nofill.err
