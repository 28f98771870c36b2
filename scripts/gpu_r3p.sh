#!/bin/bash
# Round-3 checkpoint: full GPU tier, smoke, N=1 bench (with remote phase).
set -o pipefail
out=gpurun_out/r3p
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --remote-steps 10 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json; d=json.load(open('$out/bench.json')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','read_p50_ms','host_cpu_util_rank0')}); r=d['remote_client']; print({k: r[k] for k in ('write_mb_per_s','read_mb_per_s','write_p50_ms','read_p50_ms','read_p99_ms')})"
