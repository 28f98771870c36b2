#!/bin/bash
# Full GPU tier + smoke, then the K1/K2 grid x ring sweep (where the 64 MiB time goes).
set -o pipefail
out=gpurun_out/r3f
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider \
  > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 300 build/native/crc_bench --sweep --mib 256 --iters 30 > $out/crc_sweep.json 2> $out/crc_sweep.err || exit $?
cat $out/crc_sweep.json
