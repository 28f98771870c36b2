#!/bin/bash
# Round 4: write-staging roofline (hybrid fused/SDMA at 10 writers, each path at 1 writer);
# S3 config 5 at production settings (TLS + SigV4/STS + IAM role + SSE-S3 + audit in the native
# front, 10 s phases, native load generator) and the plain config 5; config 4 at BASELINE's
# shape (60 s stress-write per shard prefix at conc 10, 2 Raft shards, 1,000 cross-shard
# renames) with the native dfs_master / dfs_config_server executables; last, hipipc
# (host-driven copy-engine copies) vs hipipc-spin (RCCL's execution model: send/recv kernels
# parked on their channel streams until the peer shows up) on the same 2-rank rehearsal.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 120 build/native/io_bench --pcie-roofline > $O/pcie_roofline_hybrid.json 2> $O/pcie_roofline_hybrid.err && \
timeout -k 10 120 build/native/io_bench --pcie-roofline --threads 1 --per 400 > $O/pcie_roofline_hybrid_t1.json 2> $O/pcie_roofline_hybrid_t1.err && \
DFS_FUSED_WRITE_MAX_INFLIGHT=0 timeout -k 10 120 build/native/io_bench --pcie-roofline --threads 1 --per 400 > $O/pcie_roofline_fused_t1.json 2> $O/pcie_roofline_fused_t1.err && \
DFS_FUSED_WRITE=0 timeout -k 10 120 build/native/io_bench --pcie-roofline --threads 1 --per 400 > $O/pcie_roofline_sdma_t1.json 2> $O/pcie_roofline_sdma_t1.err && \
timeout -k 10 400 python bench_configs.py config5 --secure --gpu 0 --phase-seconds 10 > $O/config5_secure.json 2> $O/config5_secure.err && \
timeout -k 10 400 python bench_configs.py config4 --gpu 0 --stress-seconds 60 --stress-concurrency 10 --renames 1000 > $O/config4.json 2> $O/config4.err && \
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 1000000 > $O/config5.json 2> $O/config5.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 5 --warmup 1 --transport hipipc > $O/bench_n2_hipipc.json 2> $O/bench_n2_hipipc.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29553 bench.py --gpus 2 --steps 5 --warmup 1 --transport hipipc-spin > $O/bench_n2_spin.json 2> $O/bench_n2_spin.err
