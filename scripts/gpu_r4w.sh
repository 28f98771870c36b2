#!/bin/bash
# Round 4: replica sends take their pair sequence number only once their first slice is staged
# — the GPU tier (replication, IPC, EC-device tests among it), then the 2-rank rehearsal with
# hbm-ack and nvme-sync, then the driver's N=1 command.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4w
mkdir -p $O
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29550 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5 "$@" > $O/$name.json 2> $O/$name.err
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
run n2_hbmack --durability hbm-ack && run n2_hipipc && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
