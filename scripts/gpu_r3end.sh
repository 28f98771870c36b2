#!/bin/bash
# End-of-session check: GPU tier, smoke, the driver's N=1 bench, a kernel profile of the
# bench's chunkserver, then config 4 (native 2PC after the compaction fix).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3end
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err && \
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --remote-steps 1 --profile-dir $O/prof > $O/bench_prof.json 2> $O/bench_prof.err && \
timeout -k 10 500 python bench_configs.py config4 --gpu 0 --stress-seconds 15 --renames 1000 > $O/config4.json 2> $O/config4.err
