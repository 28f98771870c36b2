#!/bin/bash
# Remote-client (gRPC/TCP) phase with and without the registered ReadBlock reply pool,
# alternating on one box.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ab_pool
for rep in 1 2; do
  for p in 0 1; do
    DFS_GRPC_REPLY_POOL=$p timeout -k 10 300 python bench.py --steps 3 --warmup 1 --remote-steps 6 \
      > gpurun_out/ab_pool/pool${p}_$rep.json 2> gpurun_out/ab_pool/pool${p}_$rep.err || exit $?
  done
done
echo ab_pool done
