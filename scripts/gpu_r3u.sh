#!/bin/bash
# GPU tier + smoke + the driver's N=1 bench command, then an 8-rank rehearsal on the one GPU
# (8 chunkservers sharing the card, RF=3 over the hipipc device transport: 28 pairs, the
# N=8 topology). Each GPU step has its own timeout; && ends at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err && \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 8 --steps 3 --warmup 1 --hbm-capacity 8G --remote-steps 0 \
  > $O/bench_n8_shared.json 2> $O/bench_n8_shared.err
