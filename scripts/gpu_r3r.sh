#!/bin/bash
# Round-3 late checkpoint: 4-rank hipipc rehearsal on one GPU (RF=3, device forwards), then the
# N=1 bench under rocprofv3 --kernel-trace --stats (kernel table after the wide CRC kernel).
set -o pipefail
out=gpurun_out/r3r
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 --hbm-capacity 8G --timeout 150 \
  > $out/bench_n4_hipipc.json 2> >(tee $out/bench_n4_hipipc.err >&2) || { tail -60 $out/bench_n4_hipipc.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_n4_hipipc.json')); print({k: d.get(k) for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','read_p50_ms','rccl_forwards','shm_forwards','grpc_forwards','rccl_fallbacks','replica_failures','repl_pair_failures','repl_pairs_up')})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --remote-steps 2 \
  > $out/bench_prof.json 2> $out/bench_prof.err || { tail -30 $out/bench_prof.err; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -3
