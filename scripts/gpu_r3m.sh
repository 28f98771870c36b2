#!/bin/bash
# K1/K2 one-workgroup-per-CU A/B (wide 0/1/2) + correctness; storage volumes of the box.
set -o pipefail
out=gpurun_out/r3m
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
(cat /proc/mounts; echo; df -h; echo; lsblk 2>&1; echo TMPDIR=$TMPDIR; df -h /tmp /dev/shm) > $out/mounts.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_replication.py -x -q --timeout 120 \
  --timeout-method thread -m gpu > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -2 $out/pytest_kernels.log
timeout -k 10 300 build/native/crc_bench --wide-ab > $out/wide_ab.json 2> $out/wide_ab.err || exit $?
python3 - <<'PY'
import json
e = json.load(open("gpurun_out/r3m/wide_ab.json"))
print("stream", e["stream_read_GBps"])
for r in e["k1k2"]: print(r["bytes"] >> 20, r["wide"], r["rep"], r["us"], r["GBps"], r["ok"])
PY
timeout -k 10 300 build/native/crc_bench > $out/crc_default.json 2> $out/crc_default.err || exit $?
python3 - <<'PY'
import json
e = json.load(open("gpurun_out/r3m/crc_default.json"))
for r in e["k1k2"]:
    if r["impl"] == "dispatch": print(r)
print("scrub", e["scrub"][0])
PY
