#!/bin/bash
# O_DIRECT (head data files + replica files) A/B, interleaved: N=1 x3 pairs, then the 2-rank
# rehearsal with and without it.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3z
mkdir -p $O
DFS_ODIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_cs_restart.py -m gpu -x -v \
  --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_odirect.log 2>&1 || exit $?
for i in 1 2 3; do
  for d in 1 0; do
    DFS_ODIRECT=$d timeout -k 10 400 python bench.py --steps 10 --warmup 2 --remote-steps 0 \
      > $O/n1_odirect${d}_$i.json 2> $O/n1_odirect${d}_$i.err || exit $?
  done
done
for d in 1 0; do
  DFS_ODIRECT=$d timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2954$d bench.py --gpus 2 --steps 5 --warmup 1 --remote-steps 0 \
    > $O/n2_odirect$d.json 2> $O/n2_odirect$d.err || exit $?
done
