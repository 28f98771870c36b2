#!/bin/bash
# 7 ranks on the one GPU (7 chunkservers sharing the card, RF=3 over the hipipc device
# transport: 21 pairs), then 2 ranks (RF=2). 7, not 8: every process that imports torch holds
# the GPU open on ROCm, and the 1-GPU box allows 16 GPU processes (8 ranks + torchrun + 8
# chunkservers = 17). Each step has its own timeout.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G --remote-steps 0 \
  --keep --workdir /tmp/dfs_n7 > $O/bench_n7_shared.json 2> $O/bench_n7_shared.err
rc=$?
cp /tmp/dfs_n7/cs0.log /tmp/dfs_n7/cs6.log $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
rm -rf /tmp/dfs_n7
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --gpus 2 --steps 5 --warmup 1 --remote-steps 0 \
  > $O/bench_n2_shared.json 2> $O/bench_n2_shared.err
