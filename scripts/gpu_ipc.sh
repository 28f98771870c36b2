#!/bin/bash
# Round 3: device replication between processes on one GPU (hipipc), HBM leak regression,
# then the 4-rank shared-GPU bench rehearsal over hipipc. Every GPU step is time-boxed.
set -o pipefail
out=gpurun_out/r3_ipc
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_replication.py tests/test_gpu_ipc.py -x -v -s \
  --timeout 300 --timeout-method thread -m gpu > $out/pytest_ipc.log 2>&1
rc=$?
tail -30 $out/pytest_ipc.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29537 bench.py --gpus 4 --steps 3 --warmup 1 --remote-steps 0 --hbm-capacity 8G \
  > $out/bench_n4_hipipc.json 2> $out/bench_n4_hipipc.err
rc=$?
cat $out/bench_n4_hipipc.json
exit $rc
