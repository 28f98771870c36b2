#!/bin/bash
# Round 4: the journal striped over 4 part files per segment (per-part group commit) against
# the per-file path, the driver's N=1 command, A/B/A/B on one box; then the N=7 rehearsal and
# the GPU journal / store tests.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_p4a.json 2> $O/bench_p4a.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile_a.json 2> $O/bench_perfile_a.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_p4b.json 2> $O/bench_p4b.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile_b.json 2> $O/bench_perfile_b.err && \
DFS_JOURNAL_PARTS=8 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_p8.json 2> $O/bench_p8.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 7 --steps 3 --warmup 1 --hbm-capacity 8G > $O/bench_n7.json 2> $O/bench_n7.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_cs_restart.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest_store.log 2>&1
