#!/bin/bash
# Round 4: what bounds the 2-rank rehearsal — the default (hipipc device forwards, nvme-sync),
# replica forwards over gRPC instead, and hbm-ack (no flush on the ack path at all).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4v
mkdir -p $O
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29550 + RANDOM % 400)) bench.py --gpus 2 --steps 20 --warmup 5 "$@" > $O/$name.json 2> $O/$name.err
}
run n2_hipipc && run n2_grpc --transport grpc && run n2_hbmack --durability hbm-ack && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --durability hbm-ack > $O/n1_hbmack.json 2> $O/n1_hbmack.err
