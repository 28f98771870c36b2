#!/bin/bash
# Round 4: journal segment preparation A/B (zero-filled vs fallocated) against the per-file
# path, the driver's N=1 command each, then a long run where the materializer must keep up.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 build/native/io_bench --journal-sweep --dir /tmp/r4c_journal > $O/journal_sweep.json 2> $O/journal_sweep.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_jz1.json 2> $O/bench_jz1.err && \
DFS_JOURNAL_ZERO_FILL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_jz0.json 2> $O/bench_jz0.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_jz1b.json 2> $O/bench_jz1b.err && \
timeout -k 10 900 python bench.py --steps 80 --warmup 5 --remote-steps 0 > $O/bench_long.json 2> $O/bench_long.err
