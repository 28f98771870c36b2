#!/bin/bash
# One GPU-box session, parameterized: `scripts/gpu.sh <out-dir> <step> [<step> ...]`.
# Every GPU step runs under its own `timeout -k`, and the steps are chained so the first
# failure ends the session (no further GPU work after a fault, an abort or a time limit).
#
#   test      pytest -m gpu (one process) + smoke()
#   bench     the driver's N=1 command (--steps 20 --warmup 5), twice
#   sustain   1 MiB stress-write for 6 s after the timed steps (longer than 3x a round-4 journal)
#   exportab  the driver's command with the exporter forced active (60 s windows at 256 MB/s),
#             off (never) and the round-4 idle mode
#   n2        2 ranks sharing the GPU (hipipc, RF 2)
#   n2hbm     the same with hbm-ack durability (the shared volume out of the ack path)
#   n4        the driver's N=4 command on 4 ranks sharing the GPU
#   reclaim   4 ranks deleting each step's files after the read-back (bench's short-volume mode)
#   ipctest   the device-replication GPU tests only
#   pullab    replica hops, receiver pull vs push (hbm-ack, conc 10 and 1)
#   pullhost  2 ranks nvme-sync: pulled replicas appended from the kernel's host copy vs HBM vs push
#   prof      rocprofv3 kernel trace of the chunkserver during a short bench
#   configs   BASELINE configs 4 and 5
#   config3 / config4   one of them (config 4 at the reference's compose topology: 4 chunkservers, RF 3)
#   secure    config 5 at production settings (TLS + SigV4/STS + IAM + SSE-S3 + audit)
#   crcpmc    two rocprofv3 PMC passes over crc_bench (LDS/VALU, then MFMA busy vs GPU-active)
#   probe     the box's block devices and mounts (where per-rank journals could live)
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:?out dir}
shift
mkdir -p "$O"
run() {  # run <name> <seconds> <cmd...>: stdout -> $O/<name>.json, stderr -> $O/<name>.err
  local name=$1 secs=$2
  shift 2
  echo "[gpu.sh] $name: $*" >&2
  timeout -k 10 "$secs" "$@" > "$O/$name.json" 2> "$O/$name.err"
  local rc=$?
  [ $rc -eq 0 ] || { echo "[gpu.sh] $name failed rc=$rc" >&2; tail -20 "$O/$name.err" >&2; }
  return $rc
}
for step in "$@"; do
  case "$step" in
    test)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
      tail -3 "$O/pytest_gpu.log"
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1 ;;
    bench)
      run bench_a 600 python bench.py --steps 20 --warmup 5 && \
      run bench_b 600 python bench.py --steps 20 --warmup 5 || exit 1 ;;
    sustain)
      run sustain 600 python bench.py --steps 5 --warmup 1 --remote-steps 0 --stress-seconds 6 \
        --stress-size 1048576 --stress-concurrency 10 || exit 1 ;;
    exportab)
      DFS_EXPORT_MBPS=256 DFS_EXPORT_HEADROOM_MB=1 run export_active 600 python bench.py --steps 20 --warmup 5 && \
      DFS_JOURNAL_EXPORT=never run export_never 600 python bench.py --steps 20 --warmup 5 && \
      DFS_JOURNAL_EXPORT=idle run export_idle 600 python bench.py --steps 20 --warmup 5 || exit 1 ;;
    n2)
      run n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 || exit 1 ;;
    n2hbm)  # the same 2 ranks with the volume out of the ack path: what the channels carry
      run n2_hbm 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack || exit 1 ;;
    n2lat)  # what one forward costs without queueing (concurrency 1), and with host waits that sleep
      run n2_hbm_c1 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --concurrency 1 && \
      run n1_hbm_c1 600 python bench.py --steps 10 --warmup 2 --durability hbm-ack --concurrency 1 && \
      DFS_HIP_SYNC=block run n2_hbm_block 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack || exit 1 ;;
    n2phase)  # replica hop phases (repl_phase_us) at concurrency 1 and 10, hbm-ack
      run n2p_c1 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --concurrency 1 && \
      run n2p_c10 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack || exit 1 ;;
    ipctest)  # the device-replication GPU tests only (hipipc pull / push / spin, multi-GPU)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_replication.py tests/test_gpu_multi.py \
        -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$O/pytest_ipc.log" 2>&1 || \
        { tail -30 "$O/pytest_ipc.log"; exit 1; }
      tail -3 "$O/pytest_ipc.log" ;;
    pullab)   # replica hops at hbm-ack: receiver pull (one kernel per hop) vs the round-5 push + checksum
      run n2_pull 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack && \
      DFS_IPC_PULL=0 run n2_push 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack && \
      run n2_pull_c1 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --concurrency 1 && \
      DFS_IPC_PULL=0 run n2_push_c1 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack \
        --concurrency 1 || exit 1 ;;
    pullrep)  # receiver pull vs push at 2 ranks, interleaved, 3 reps each, nvme-sync then hbm-ack
      for i in 1 2 3; do
        run n2pull_nv_$i 600 python bench.py --gpus 2 --steps 10 --warmup 2 && \
        DFS_IPC_PULL=0 run n2push_nv_$i 600 python bench.py --gpus 2 --steps 10 --warmup 2 && \
        run n2pull_hbm_$i 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack && \
        DFS_IPC_PULL=0 run n2push_hbm_$i 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack \
          || exit 1
      done ;;
    pullhost) # 2 ranks nvme-sync: pulled replicas appended from the kernel's host copy / from HBM / push
      DFS_PULL_HOST=1 run n2_pullhost 600 python bench.py --gpus 2 --steps 10 --warmup 2 && \
      run n2_pulldev 600 python bench.py --gpus 2 --steps 10 --warmup 2 && \
      DFS_IPC_PULL=0 run n2_pushnv 600 python bench.py --gpus 2 --steps 10 --warmup 2 && \
      DFS_PULL_HOST=1 run n2_pullhost_b 600 python bench.py --gpus 2 --steps 10 --warmup 2 || exit 1 ;;
    n2prof)   # rocprofv3 kernel + marker + memory-copy traces of both chunkservers, 2 ranks, conc 1
      DFS_PROF_EXTRA=--memory-copy-trace run n2prof 600 python bench.py --gpus 2 --steps 5 --warmup 1 \
        --durability hbm-ack --concurrency 1 --remote-steps 0 --profile-dir "$O/n2prof" || exit 1 ;;
    reclaim)  # 4 ranks with each step's files deleted after the read-back (what a short volume triggers)
      DFS_BENCH_RECLAIM=1 run n4_reclaim 900 python bench.py --gpus 4 --steps 10 --warmup 2 || exit 1 ;;
    n4)     # the driver's N=4 command, 4 ranks sharing the GPU
      run n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 || exit 1 ;;
    prof)
      run prof 600 python bench.py --steps 3 --warmup 1 --profile-dir "$O/prof" || exit 1 ;;
    profcopy) # the N=1 profile with the memory-copy trace (which copies still use the copy engines)
      DFS_PROF_EXTRA=--memory-copy-trace run profcopy 600 python bench.py --steps 3 --warmup 1 --remote-steps 0 \
        --profile-dir "$O/profcopy" || exit 1 ;;
    syncab)   # how host threads wait for the GPU: runtime default, blocking (interrupt), yield
      run sync_default 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 && \
      DFS_HIP_SYNC=block run sync_block 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 && \
      DFS_HIP_SYNC=yield run sync_yield 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 && \
      DFS_HIP_SYNC=block run sync_block_n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 --remote-steps 0 && \
      run sync_default_n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 --remote-steps 0 || exit 1 ;;
    volab)    # 4 ranks on one volume: exporter off, O_DIRECT journal, and the N=1 command with O_DIRECT
      run vol_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_EXPORT=never run vol_n4_noexport 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_DIRECT=1 run vol_n4_direct 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_DIRECT=1 run vol_n1_direct 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 && \
      run vol_n1 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 || exit 1 ;;
    sliceab)  # 1 MiB replica transfers in one slice instead of four (hbm-ack and nvme-sync)
      DFS_REPL_MIN_SLICE_KIB=1024 run s1m_c1 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --concurrency 1 --remote-steps 0 && \
      DFS_REPL_MIN_SLICE_KIB=1024 run s1m_c10 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --remote-steps 0 && \
      run s256k_c10 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --remote-steps 0 && \
      DFS_REPL_MIN_SLICE_KIB=1024 run s1m_n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 --remote-steps 0 && \
      run s256k_n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 --remote-steps 0 || exit 1 ;;
    laneab)   # 8 vs 16 stream contexts per chunkserver, receives taking theirs eagerly or at landing
      DFS_RECV_LANE_EAGER=1 run l8e 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --remote-steps 0 && \
      run l8 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --remote-steps 0 && \
      DFS_CS_LANES=16 run l16 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --remote-steps 0 && \
      DFS_CS_LANES=16 DFS_RECV_LANE_EAGER=1 run l16e 600 python bench.py --gpus 2 --steps 10 --warmup 2 --durability hbm-ack --remote-steps 0 && \
      DFS_CS_LANES=16 run l16_n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 --remote-steps 0 && \
      run l8_n2 600 python bench.py --gpus 2 --steps 10 --warmup 2 --remote-steps 0 && \
      DFS_CS_LANES=16 run l16_n1 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 && \
      run l8_n1 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 || exit 1 ;;
    partab)   # 4 ranks on one volume: fewer journal parts per chunkserver (more records per flush)
      run p8_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_PARTS=2 run p2_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_PARTS=1 run p1_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_SYNC_DELAY_US=300 run d300_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 || exit 1 ;;
    partab2)  # more journal parts: 16 / 32 at 4 ranks, 16 at N=1
      DFS_JOURNAL_PARTS=16 run p16_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_PARTS=32 run p32_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      run p8_n4b 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_PARTS=16 run p16_n1 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 && \
      run p8_n1 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 || exit 1 ;;
    gateab)   # journal appends under the node-wide disk gate (12 / 24 slots) at 4 ranks, and N=1
      run g0_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_GATE=1 run g12_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_GATE=1 DFS_DISK_INFLIGHT=24 run g24_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_GATE=1 DFS_DISK_INFLIGHT=6 run g6_n4 900 python bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 && \
      DFS_JOURNAL_GATE=1 run g12_n1 600 python bench.py --steps 20 --warmup 5 --remote-steps 0 || exit 1 ;;
    configs)
      run config4 500 python bench_configs.py config4 --gpu 0 && \
      run config5 500 python bench_configs.py config5 --gpu 0 || exit 1 ;;
    config3)  # 3 chunkservers, RF 3 (sharing the GPU on a 1-GPU box), nvme-sync + hbm-ack
      run config3 600 python bench_configs.py config3 --gpu 0 || exit 1 ;;
    config4)  # 2 shards + 4 chunkservers (RF 3), 60 s stress-write per shard prefix
      run config4 600 python bench_configs.py config4 --gpu 0 || exit 1 ;;
    config5)
      run config5 500 python bench_configs.py config5 --gpu 0 || exit 1 ;;
    secure)
      run config5_secure 600 python bench_configs.py config5 --gpu 0 --secure || exit 1 ;;
    crcpmc)
      R=$PWD
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
         SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU \
         -d "$R/$O/pmc_crc" -o crc --output-format csv -- "$R/build/native/crc_bench" --iters 5 --mib 256 \
         > "$R/$O/pmc_crc.log" 2>&1) && \
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES \
         SQ_WAVES GRBM_GUI_ACTIVE -d "$R/$O/pmc_mfma" -o crc --output-format csv -- "$R/build/native/crc_bench" \
         --iters 5 --mib 256 > "$R/$O/pmc_mfma.log" 2>&1) || exit 1 ;;
    probe)
      { lsblk -o NAME,SIZE,TYPE,MOUNTPOINT,ROTA,MODEL 2>&1; df -h 2>&1; cat /proc/mounts; nproc; free -g; } \
        > "$O/probe.txt" 2>&1 || true ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "[gpu.sh] done" >&2
