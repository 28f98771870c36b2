#!/bin/bash
# Round 4: the closing device sync's latency (chunkserver-side hipDeviceSynchronize vs the
# request) in two journal runs; then the S3 / config-4 / transport / roofline steps of r4g.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j4a.json 2> $O/bench_j4a.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j4b.json 2> $O/bench_j4b.err && \
bash scripts/gpu_r4g.sh
