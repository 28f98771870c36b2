#!/bin/bash
# Round 4: the chunkserver's CPU in config 5's sustained PUT — durable-path counters per phase
# (journal records, bypassed writes, materialized blocks), with the journal and without it.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 100000 > $O/config5.json 2> $O/config5.err && \
DFS_JOURNAL=0 timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 100000 > $O/config5_perfile.json 2> $O/config5_perfile.err
