#!/bin/bash
# Round 4: S3 config 5 at production settings (TLS + SigV4/STS + IAM role + SSE-S3 + audit in the
# native front, 10 s phases, native load generator) and the plain config 5; config 4 at
# BASELINE's shape (60 s stress-write per shard prefix at conc 10, 2 Raft shards, 1,000
# cross-shard renames) with the native dfs_master / dfs_config_server executables.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 400 python bench_configs.py config5 --secure --gpu 0 --phase-seconds 10 > $O/config5_secure.json 2> $O/config5_secure.err && \
timeout -k 10 400 python bench_configs.py config4 --gpu 0 --stress-seconds 60 --stress-concurrency 10 --renames 1000 > $O/config4.json 2> $O/config4.err && \
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 1000000 > $O/config5.json 2> $O/config5.err
