#!/bin/bash
# Round 4: the 2-rank rehearsal (RF 2, 20 steps) with buffered journal appends, O_DIRECT
# appends (cheaper flushes when two chunkservers share the volume), and the per-file path.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4u
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29550 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5 > $O/$name.json 2> $O/$name.err
}
run n2_buffered DFS_JOURNAL_DIRECT=0 && run n2_direct DFS_JOURNAL_DIRECT=1 && run n2_perfile DFS_JOURNAL=0 && \
run n2_direct_b DFS_JOURNAL_DIRECT=1 && run n2_buffered_b DFS_JOURNAL_DIRECT=0
