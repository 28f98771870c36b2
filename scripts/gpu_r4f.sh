#!/bin/bash
# Round 4: journal with idle zero-fill + pipelined flush rounds (A/B syncers 1 vs 4) against the
# per-file path on one box; PCIe roofline of the fused write/read kernels vs the SDMA path;
# the N=7 shared-GPU rehearsal with both journal modes.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4f
mkdir -p $O
df -h /tmp > $O/df.txt 2>&1
timeout -k 10 120 build/native/io_bench --pcie-roofline > $O/pcie_roofline_fused.json 2> $O/pcie_roofline_fused.err && \
DFS_FUSED_WRITE=0 DFS_FUSED_READ=0 timeout -k 10 120 build/native/io_bench --pcie-roofline > $O/pcie_roofline_sdma.json 2> $O/pcie_roofline_sdma.err && \
timeout -k 10 400 build/native/io_bench --journal-sweep --dir /tmp/r4f_journal > $O/journal_sweep.json 2> $O/journal_sweep.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_s1.json 2> $O/bench_s1.err && \
DFS_JOURNAL_SYNCERS=4 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_s4.json 2> $O/bench_s4.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile2.json 2> $O/bench_perfile2.err && \
DFS_JOURNAL_SYNCERS=4 timeout -k 10 600 python bench.py --steps 80 --warmup 5 --remote-steps 0 > $O/bench_long_s4.json 2> $O/bench_long_s4.err && \
DFS_JOURNAL_SYNCERS=4 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G > $O/bench_n7_s4.json 2> $O/bench_n7_s4.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29545 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G > $O/bench_n7_s1.json 2> $O/bench_n7_s1.err
