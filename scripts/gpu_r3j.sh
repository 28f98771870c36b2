#!/bin/bash
# Balanced tile runs in the CRC kernels: correctness tier + the grid x ring sweep + defaults.
set -o pipefail
out=gpurun_out/r3j
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_replication.py -x -q --timeout 120 \
  --timeout-method thread -m gpu > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -2 $out/pytest_kernels.log
timeout -k 10 300 build/native/crc_bench --sweep --mib 256 --iters 30 > $out/crc_sweep.json 2> $out/crc_sweep.err || exit $?
timeout -k 10 300 build/native/crc_bench > $out/crc_default.json 2> $out/crc_default.err || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r3j/crc_sweep.json"))
for r in d["k1k2"]:
    if r["bytes"] in (64 << 20, 256 << 20): print(r)
e = json.load(open("gpurun_out/r3j/crc_default.json"))
for r in e["k1k2"]:
    if r["impl"] == "dispatch": print(r)
print("scrub", e["scrub"][0])
PY
