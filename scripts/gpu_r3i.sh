#!/bin/bash
# End-of-milestone benches: N=1 headline (driver defaults, then 20 steps), hbm-ack, and the
# 4-rank shared-GPU rehearsal over hipipc (RF=3, device forwards) with the native agents.
set -o pipefail
out=gpurun_out/r3i
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --remote-steps 5 > $out/bench_nvme.json 2> $out/bench_nvme.err || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --remote-steps 0 --durability hbm-ack > $out/bench_hbm.json 2> $out/bench_hbm.err || exit $?
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 --hbm-capacity 8G \
  > $out/bench_n4_hipipc.json 2> $out/bench_n4_hipipc.err || { tail -30 $out/bench_n4_hipipc.err; exit 1; }
for f in bench_nvme bench_hbm bench_n4_hipipc; do
  echo "== $f"; python -c "import json; d=json.load(open('$out/$f.json')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','write_p99_ms','rccl_forwards','shm_forwards','grpc_forwards','replica_failures','repl_pair_failures','host_cpu_util_rank0','remote_client') if k in d})"
done
