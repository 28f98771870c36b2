#!/bin/bash
# Config 5 (S3 gateway) on one MI355X: native front end with one gateway process, then four.
# Each run also drives the gateway from the native load generator (build/native/s3_load).
set -o pipefail
out=gpurun_out/r3_s3
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 1 4; do
  S3_WORKERS=$w timeout -k 10 500 python bench_configs.py config5 --gpu 0 --parquet-rows 2000000 \
    > $out/config5_w${w}_native.json 2> $out/config5_w${w}_native.err || exit $?
  cat $out/config5_w${w}_native.json
done
