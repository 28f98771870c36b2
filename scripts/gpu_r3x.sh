#!/bin/bash
# hipipc waits on futexes (no polling threads): the device-replication GPU tests, then the
# 2-rank and 7-rank shared-GPU rehearsals (compare cs*_sys with profiles/r3_rehearsal).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_replication.py -m gpu -x -v --timeout 180 \
  --timeout-method thread -p no:cacheprovider > $O/pytest_ipc.log 2>&1 && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --gpus 2 --steps 5 --warmup 1 --remote-steps 0 \
  > $O/bench_n2_shared.json 2> $O/bench_n2_shared.err && \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G --remote-steps 0 \
  > $O/bench_n7_shared.json 2> $O/bench_n7_shared.err
