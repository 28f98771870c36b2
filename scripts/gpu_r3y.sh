#!/bin/bash
# O_DIRECT data files for fresh durable blocks (DFS_ODIRECT=1) vs buffered + fdatasync:
# the GPU crash-restart / cluster tests with O_DIRECT on, then N=1 benches alternating.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3y
mkdir -p $O
DFS_ODIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_cs_restart.py tests/test_gpu_cluster.py -m gpu -x -v \
  --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_odirect.log 2>&1 || exit $?
for i in 1 2; do
  for d in 0 1; do
    DFS_ODIRECT=$d timeout -k 10 400 python bench.py --steps 10 --warmup 2 --remote-steps 0 \
      > $O/bench_odirect${d}_$i.json 2> $O/bench_odirect${d}_$i.err || exit $?
  done
done
