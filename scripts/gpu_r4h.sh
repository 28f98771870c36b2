#!/bin/bash
# Round 4: where the journal's write time goes. K journals on the one volume (1 / 3 / 7, as
# K chunkservers of a node) with per-journal vs node-wide flush combining; the driver's N=1
# bench with the journal (flush / commit timing in the JSON) and with the per-file path, then
# the journal bench under rocprofv3 (kernel + marker trace: dfs.store.* phases).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 build/native/io_bench --multi-journal --dir /tmp/r4h_mj > $O/multi_journal.json 2> $O/multi_journal.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j1.json 2> $O/bench_j1.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j2.json 2> $O/bench_j2.err && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --remote-steps 0 --profile-dir gpurun_out/r4h/prof > $O/bench_prof.json 2> $O/bench_prof.err
