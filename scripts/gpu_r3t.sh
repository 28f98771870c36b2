#!/bin/bash
# Re-entry check after a container rebuild: the box's volumes, GPU tier, smoke, and the
# driver's N=1 bench command. Each GPU step has its own timeout; && ends at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r3t
O=gpurun_out/r3t
{ df -hT; echo; lsblk -o NAME,SIZE,TYPE,MOUNTPOINT,ROTA,MODEL 2>&1; echo; mount | grep -v -e cgroup -e proc -e sysfs; } > $O/volumes.txt 2>&1 || true
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
