#!/bin/bash
# Config 5 (S3 gateway) on one MI355X: native front end, one gateway process and four.
set -o pipefail
out=gpurun_out/r3_s3
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
S3_WORKERS=1 timeout -k 10 500 python bench_configs.py config5 --gpu 0 --parquet-rows 2000000 \
  > $out/config5_w1_native.json 2> $out/config5_w1_native.err || exit $?
cat $out/config5_w1_native.json
S3_WORKERS=4 timeout -k 10 500 python bench_configs.py config5 --gpu 0 --parquet-rows 2000000 \
  > $out/config5_w4_native.json 2> $out/config5_w4_native.err || exit $?
cat $out/config5_w4_native.json
