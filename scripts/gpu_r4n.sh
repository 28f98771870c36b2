#!/bin/bash
# Round 4: FP4 chunk CRCs as the default — the full GPU tier and smoke(), crc_bench's default
# table (K1/K2 by size, K1b scrub in both forms, RS); the driver's N=1 command twice (device
# syncs over one keep-alive connection); config 4 with the masters' logs kept; config 5 plain
# (PUT past the journal's materialize mark takes the per-file path).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 300 build/native/crc_bench > $O/crc_default.json 2> $O/crc_default.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_a.json 2> $O/bench_a.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_b.json 2> $O/bench_b.err && \
DFS_KEEP_LOGS=$O/c4logs DFS_LOG=info timeout -k 10 420 python bench_configs.py config4 --gpu 0 --stress-seconds 60 --stress-concurrency 10 --renames 1000 > $O/config4.json 2> $O/config4.err ; \
timeout -k 10 500 python bench_configs.py config5 --gpu 0 --phase-seconds 10 > $O/config5.json 2> $O/config5.err
