#!/bin/bash
# Full GPU tier, then the bench's remote phase with registered request buffers (A/B: the
# pool disabled through a tiny DFS_GRPC_REPLY_PREWARM has no effect on requests, so compare
# against profiles/r3_bench).
set -o pipefail
out=gpurun_out/r3k
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider \
  > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --remote-steps 10 > $out/bench.json 2> $out/bench.err || exit $?
python -c "import json; d=json.load(open('$out/bench.json')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','remote_client') if k in d})"
