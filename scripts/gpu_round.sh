#!/bin/bash
# One GPU-box session: GPU tests, smoke, 1-GPU bench (nvme-sync + hbm-ack) and a
# rocprofv3 kernel-trace of the ChunkServer during the bench. Every GPU step has its own
# timeout and the steps are chained with && so the first failure ends the session.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
STEP=${1:-all}
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
if [ "$STEP" = "all" ] || [ "$STEP" = "test" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_nvme.json 2> gpurun_out/bench_nvme.err && \
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 --durability hbm-ack > gpurun_out/bench_hbm.json 2> gpurun_out/bench_hbm.err || exit $?
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "prof" ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --profile-dir gpurun_out/prof > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "micro" ]; then
  # native I/O + kernel microbenchmark (C45) under a kernel trace
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$OLDPWD/gpurun_out/prof_io" -o io -- "$OLDPWD/build/native/io_bench" --iters 30) \
     > gpurun_out/io_bench.json 2> gpurun_out/io_bench.err || exit $?
fi
if [ "$STEP" = "sync" ]; then
  # A/B of the durability flush: per-file fdatasync pair vs group-commit syncfs
  DFS_GROUP_SYNC=0 timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_sync0.json 2> gpurun_out/bench_sync0.err && \
  DFS_GROUP_SYNC=1 timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_sync1.json 2> gpurun_out/bench_sync1.err || exit $?
fi
if [ "$STEP" = "quick" ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || exit $?
fi
if [ "$STEP" = "multi" ]; then
  # N=2 rehearsal on a single GPU: two ranks share the device, gRPC replication
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2_shared.json 2> gpurun_out/bench_n2_shared.err || exit $?
fi
if [ "$STEP" = "rccl-fail" ]; then
  # RCCL failure-path rehearsal: two ranks on one GPU cannot form a communicator
  # (duplicate device); both must give up within the deadline and fall back together
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29535 bench.py --gpus 2 --steps 2 --warmup 1 --rehearse-rccl --keep --workdir /tmp/dfs_rccl_rehearsal \
    > gpurun_out/bench_rccl_rehearsal.json 2> gpurun_out/bench_rccl_rehearsal.err; rc=$?
  cp /tmp/dfs_rccl_rehearsal/cs*.log gpurun_out/ 2>/dev/null || true
  [ $rc -eq 0 ] || exit $rc
fi
echo "gpu_round done"
