#!/bin/bash
# Round 4: the wide K1/K2 kernel on the FP4 matrix cores (zlib numerics, i8 vs FP4 A/B with a
# same-size streaming read); the driver's N=1 command three times with the journal settled before the warm-up and
# no cyclic GC inside the timed region, once with the per-file path; the 2-rank rehearsal at
# the driver's step count; the 7-rank rehearsal with the job's cgroup CPU (cores used, quota,
# throttled time) to show what bounds it; config 4 on a fixed two-shard map.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4m
mkdir -p $O
{ nproc; python -c 'import os; print(len(os.sched_getaffinity(0)))'; cat /proc/self/cgroup;
  cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us 2>&1;
  df -h . /tmp /dev/shm; free -g; } > $O/box.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_kernels.log 2>&1 && \
timeout -k 10 300 build/native/crc_bench --fp4-ab > $O/crc_fp4_ab.json 2> $O/crc_fp4_ab.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_a.json 2> $O/bench_a.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_b.json 2> $O/bench_b.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_c.json 2> $O/bench_c.err && \
DFS_JOURNAL=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_perfile.json 2> $O/bench_perfile.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2.json 2> $O/bench_n2.err && \
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 \
  --master-port 29553 bench.py --gpus 7 --steps 3 --warmup 1 > $O/bench_n7.json 2> $O/bench_n7.err && \
timeout -k 10 400 python bench_configs.py config4 --gpu 0 --stress-seconds 60 --stress-concurrency 10 --renames 1000 > $O/config4.json 2> $O/config4.err
