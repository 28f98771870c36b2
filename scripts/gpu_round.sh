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
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv \
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
if [ "$STEP" = "gate" ]; then
  # Node-wide disk admission (csrc/disk_gate.h): 4 ranks share the GPU and the volume, RF=3,
  # so ~120 durable replica writes are in flight; A/B ungated vs the default gate, then N=1
  DFS_DISK_INFLIGHT=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29537 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/bench_n4_gate0.json 2> gpurun_out/bench_n4_gate0.err && \
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29539 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/bench_n4_gate.json 2> gpurun_out/bench_n4_gate.err && \
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit $?
fi
if [ "$STEP" = "gate2" ]; then
  # interleaved: fresh N=1, N=4 gated, N=4 ungated, N=1 again (the volume throttles after bursts)
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/g2_n1a.json 2> gpurun_out/g2_n1a.err && \
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/g2_n4_gate.json 2> gpurun_out/g2_n4_gate.err && \
  DFS_DISK_INFLIGHT=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29543 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/g2_n4_gate0.json 2> gpurun_out/g2_n4_gate0.err && \
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/g2_n1b.json 2> gpurun_out/g2_n1b.err || exit $?
fi
if [ "$STEP" = "diag" ]; then
  # why does a 1-GPU write get slow (and burn kernel CPU) after a burst of runs?
  D=gpurun_out/diag.txt
  { stat -f . ; grep -v "^overlay\|cgroup\|proc\|sysfs\|devpts\|mqueue" /proc/mounts | head -20; } > $D 2>&1
  { TIMEFORMAT="io_bench 10:0 fresh user=%U sys=%S wall=%R"; time timeout -k 10 120 build/native/io_bench --disk-sweep --dir ./iob --cases "10:0,10:0" ; } >> $D 2>&1 && \
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29545 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/d_n4.json 2> gpurun_out/d_n4.err || exit $?
  { echo "--- after n4"; ps -eo pid,stat,pcpu,etime,comm | awk '$3 > 1.0' ; cat /proc/pressure/io; grep -E "Dirty|Writeback:|MemFree|^Cached" /proc/meminfo; } >> $D 2>&1
  { TIMEFORMAT="io_bench 10:0 after user=%U sys=%S wall=%R"; time timeout -k 10 120 build/native/io_bench --disk-sweep --dir ./iob --cases "10:0,10:0" ; } >> $D 2>&1 && \
  { TIMEFORMAT="io_bench 10:0 tmp-after user=%U sys=%S wall=%R"; time timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/iob --cases "10:0" ; } >> $D 2>&1 && \
  sleep 45 && echo "--- after 45s" >> $D && cat /proc/pressure/io >> $D && \
  { TIMEFORMAT="io_bench 10:0 later user=%U sys=%S wall=%R"; time timeout -k 10 120 build/native/io_bench --disk-sweep --dir ./iob --cases "10:0,10:0" ; } >> $D 2>&1 && \
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/d_n1.json 2> gpurun_out/d_n1.err || exit $?
fi
if [ "$STEP" = "diag2" ]; then
  # buffered vs O_DIRECT durable writes, fresh and after an N=4 burst
  D=gpurun_out/diag2.txt
  C="10:0:0,10:0:1,30:12:0,30:12:1,10:0:0,10:0:1"
  { TIMEFORMAT="fresh user=%U sys=%S wall=%R"; time timeout -k 10 200 build/native/io_bench --disk-sweep --dir ./iob --cases "$C" ; } > $D 2>&1 && \
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29547 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/d2_n4.json 2> gpurun_out/d2_n4.err && \
  { TIMEFORMAT="after user=%U sys=%S wall=%R"; time timeout -k 10 200 build/native/io_bench --disk-sweep --dir ./iob --cases "$C" ; } >> $D 2>&1 && \
  sleep 30 && \
  { TIMEFORMAT="later user=%U sys=%S wall=%R"; time timeout -k 10 200 build/native/io_bench --disk-sweep --dir ./iob --cases "$C" ; } >> $D 2>&1 || exit $?
fi
if [ "$STEP" = "stress" ]; then
  # the reference's published config: stress-write 30 s, 10240 B, concurrency 5 (470 ops/s)
  timeout -k 10 600 python bench.py --steps 1 --warmup 1 --stress-seconds 30 > gpurun_out/bench_stress_nvme.json 2> gpurun_out/bench_stress_nvme.err && \
  timeout -k 10 600 python bench.py --steps 1 --warmup 1 --stress-seconds 30 --durability hbm-ack > gpurun_out/bench_stress_hbm.json 2> gpurun_out/bench_stress_hbm.err && \
  timeout -k 10 600 python bench.py --steps 1 --warmup 1 --stress-seconds 60 --stress-size 1048576 --stress-concurrency 10 > gpurun_out/bench_stress_1m.json 2> gpurun_out/bench_stress_1m.err || exit $?
fi
echo "gpu_round done"
if [ "$STEP" = "gate3" ]; then
  # FIFO disk admission: N=4 ranks sharing the GPU and the volume (RF=3, shm fan-out), then N=1
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29551 bench.py --gpus 4 --steps 3 --warmup 1 --hbm-capacity 16G > gpurun_out/g3_n4.json 2> gpurun_out/g3_n4.err && \
  timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/g3_n1.json 2> gpurun_out/g3_n1.err || exit $?
fi
if [ "$STEP" = "grpcab" ]; then
  # remote-client phase with the ChunkServerService on the native nghttp2 server vs grpcio
  DFS_CS_GRPC=grpcio timeout -k 10 600 python bench.py --steps 2 --warmup 1 --remote-steps 3 > gpurun_out/ab_grpcio.json 2> gpurun_out/ab_grpcio.err && \
  DFS_CS_GRPC=native timeout -k 10 600 python bench.py --steps 2 --warmup 1 --remote-steps 3 > gpurun_out/ab_native.json 2> gpurun_out/ab_native.err || exit $?
fi
if [ "$STEP" = "mgrpcab" ]; then
  # remote-client phase: MasterService on grpcio vs the native server (chunkserver native in both)
  DFS_MASTER_GRPC=grpcio timeout -k 10 600 python bench.py --steps 2 --warmup 1 --remote-steps 4 > gpurun_out/mab_grpcio.json 2> gpurun_out/mab_grpcio.err && \
  DFS_MASTER_GRPC=native timeout -k 10 600 python bench.py --steps 2 --warmup 1 --remote-steps 4 > gpurun_out/mab_native.json 2> gpurun_out/mab_native.err || exit $?
fi
if [ "$STEP" = "remoteab" ]; then
  # remote-client phase: Python grpcio client vs the native C++ client (servers native in both)
  DFS_NATIVE_REMOTE=0 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --remote-steps 4 > gpurun_out/rab_python.json 2> gpurun_out/rab_python.err && \
  DFS_NATIVE_REMOTE=1 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --remote-steps 4 > gpurun_out/rab_native.json 2> gpurun_out/rab_native.err || exit $?
fi
if [ "$STEP" = "s3" ]; then
  # config 5 with the single-process gateway vs the multi-process one (A/B of S3_WORKERS)
  S3_WORKERS=1 timeout -k 10 400 python bench_configs.py config5 --gpu 0 > gpurun_out/config5_w1.json 2> gpurun_out/config5_w1.err && \
  S3_WORKERS=8 timeout -k 10 400 python bench_configs.py config5 --gpu 0 > gpurun_out/config5_w8.json 2> gpurun_out/config5_w8.err && \
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit $?
fi

if [ "$STEP" = "configs" ]; then
  # BASELINE configs 4 (2-shard stress-write + cross-shard Rename) and 5 (S3 + Parquet) on the GPU
  timeout -k 10 500 python bench_configs.py config4 --gpu 0 > gpurun_out/config4.json 2> gpurun_out/config4.err && \
  timeout -k 10 500 python bench_configs.py config5 --gpu 0 > gpurun_out/config5.json 2> gpurun_out/config5.err || exit $?
fi
