#!/bin/bash
# Config 5 alone (one gateway process, native front): native audit writer vs the Python one.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3s3
mkdir -p $O
for a in 1 0; do
  DFS_AUDIT_NATIVE=$a S3_WORKERS=1 timeout -k 10 500 python bench_configs.py config5 --gpu 0 --parquet-rows 1000000 \
    > $O/config5_audit_native$a.json 2> $O/config5_audit_native$a.err || exit $?
done
