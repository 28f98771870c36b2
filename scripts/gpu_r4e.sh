#!/bin/bash
# Round 4: PCIe roofline of the fused bench kernels, the driver's N=1 command with the
# journal (fallocated segments, the new default) twice and with the per-file path, a long
# run where the materializer must keep up, and the shared-GPU 2- and 7-rank rehearsals.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4e
mkdir -p $O
df -h /tmp > $O/df.txt 2>&1
timeout -k 10 120 build/native/io_bench --pcie-roofline > $O/pcie_roofline.json 2> $O/pcie_roofline.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j1.json 2> $O/bench_j1.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_j2.json 2> $O/bench_j2.err && \
timeout -k 10 600 python bench.py --steps 80 --warmup 5 --remote-steps 0 > $O/bench_long.json 2> $O/bench_long.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29543 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G > $O/bench_n7.json 2> $O/bench_n7.err && \
DFS_JOURNAL=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29545 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G > $O/bench_n7_perfile.json 2> $O/bench_n7_perfile.err
