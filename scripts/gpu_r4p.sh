#!/bin/bash
# Round 4: where the CPU goes in the S3 phases (cores per process: gateway, chunkserver, master,
# load generator; the job's cgroup quota and throttling), plain and production settings.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 100000 > $O/config5.json 2> $O/config5.err && \
timeout -k 10 500 python bench_configs.py config5 --secure --gpu 0 --phase-seconds 10 > $O/config5_secure.json 2> $O/config5_secure.err
