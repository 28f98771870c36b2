#!/bin/bash
# Round 4: journal A/B on the box's volume, the GPU store / device-EC / multi-GPU tests, and
# the driver's N=1 bench with the journal vs the per-file path (same box).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4b
mkdir -p $O
df -h /tmp . > $O/df.txt 2>&1; mount | grep -E ' / | /tmp ' >> $O/df.txt 2>&1 || true
timeout -k 10 300 build/native/io_bench --journal-sweep --dir /tmp/r4b_journal > $O/journal_sweep.json 2> $O/journal_sweep.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ec_device.py tests/test_gpu_multi.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_new.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_journal.json 2> $O/bench_journal.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_journal2.json 2> $O/bench_journal2.err
