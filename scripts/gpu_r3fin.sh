#!/bin/bash
# Final check of the session: GPU tier, smoke, the driver's N=1 bench, then the 2-rank and
# 7-rank shared-GPU rehearsals (native heartbeat + futex waits + compaction thread).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3fin
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --gpus 2 --steps 5 --warmup 1 --remote-steps 0 > $O/bench_n2.json 2> $O/bench_n2.err && \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G --remote-steps 0 > $O/bench_n7.json 2> $O/bench_n7.err
