#!/bin/bash
# Configs 4 and 5 with the round-3 native pieces: config 4 (2 Raft shards, stress-write +
# cross-shard Rename) with the native 2PC coordinator and the Python one (A/B), then config 5
# (S3 gateway, one process, native front + native audit writer).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3cfg
mkdir -p $O
for v in 1 0; do
  DFS_NATIVE_2PC=$v timeout -k 10 500 python bench_configs.py config4 --gpu 0 --stress-seconds 15 --renames 1000 \
    > $O/config4_native2pc$v.json 2> $O/config4_native2pc$v.err || exit $?
done
S3_WORKERS=1 timeout -k 10 500 python bench_configs.py config5 --gpu 0 --parquet-rows 2000000 \
  > $O/config5_w1.json 2> $O/config5_w1.err
