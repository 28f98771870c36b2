#!/bin/bash
# 4-rank hipipc rehearsal on one GPU, three runs back to back (an earlier call hung once with
# no output): bench's own watchdog (--timeout 150) prints every process's log tail on a hang.
set -o pipefail
out=gpurun_out/r3s
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2 3; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $((29570 + k)) bench.py --gpus 4 --steps 5 --warmup 2 --remote-steps 0 --hbm-capacity 8G --timeout 150 \
    > $out/bench_n4_$k.json 2> >(tee $out/bench_n4_$k.err >&2) || { echo "run $k failed"; tail -80 $out/bench_n4_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_n4_$k.json')); print($k, {k: d.get(k) for k in ('value','write_mb_per_s','write_p50_ms','rccl_forwards','rccl_fallbacks','repl_pair_failures')})"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --remote-steps 2 \
  > $out/bench_prof.json 2> $out/bench_prof.err || { tail -30 $out/bench_prof.err; exit 1; }
find $out/prof -name "*stats.csv"
