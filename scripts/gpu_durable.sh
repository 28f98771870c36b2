#!/bin/bash
# the N=1 nvme-sync write path next to the volume's own 10-writer ceiling
# (io_bench --disk-sweep: 1 MiB + sidecar, write + fdatasync), in one call, and the cost of
# the directory fsync that makes the renames durable (DFS_DIR_SYNC=1 default vs 0), A/B/A/B.
set -o pipefail
out=gpurun_out/r3_durable
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
sweep() { timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/iob --cases "10:0,10:0" > $out/sweep_$1.json 2>&1; }
one() { DFS_DIR_SYNC=$1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --remote-steps 0 > $out/bench_ds$1_$2.json 2> $out/bench_ds$1_$2.err; }
sweep a && one 1 a && one 0 a && one 1 b && one 0 b && sweep b || exit $?
for f in $out/sweep_a.json $out/bench_ds1_a.json $out/bench_ds0_a.json $out/bench_ds1_b.json $out/bench_ds0_b.json $out/sweep_b.json; do
  echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','host_cpu_util_rank0') if k in d} if 'value' in d else d)"
done
