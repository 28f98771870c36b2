#!/bin/bash
# Round 4: sustained S3 PUT with the materializer waiting for a pause (config 5 plain), the
# remote gateway's native front (config 5 --remote-gateway), the 2-rank rehearsal with 8 / 2
# journal parts, and the driver's N=1 command next to io_bench's 10-writer disk sweep on the
# same volume (VERDICT r3 item 1's "side by side").
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 100000 > $O/config5.json 2> $O/config5.err && \
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 --parquet-rows 100000 --remote-gateway > $O/config5_remote.json 2> $O/config5_remote.err && \
timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/io_bench_disk --cases 10:0,10:0 > $O/disk_sweep_before.json 2> $O/disk_sweep_before.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_a.json 2> $O/bench_a.err && \
timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/io_bench_disk --cases 10:0,10:0 > $O/disk_sweep_after.json 2> $O/disk_sweep_after.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_p8.json 2> $O/bench_n2_p8.err && \
DFS_JOURNAL_PARTS=2 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29553 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_p2.json 2> $O/bench_n2_p2.err
