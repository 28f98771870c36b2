#!/bin/bash
# Round 4 checkpoint: the full GPU test tier and smoke() on the current tree, the driver's N=1
# command twice, the 2-rank rehearsal (native device-sync bracket), and config 4 with the
# per-file durable path for an A/B against r4g's journal run.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_a.json 2> $O/bench_a.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_b.json 2> $O/bench_b.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err && \
DFS_JOURNAL=0 timeout -k 10 400 python bench_configs.py config4 --gpu 0 --stress-seconds 60 --stress-concurrency 10 --renames 1000 > $O/config4_perfile.json 2> $O/config4_perfile.err
