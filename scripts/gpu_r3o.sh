#!/bin/bash
# Wide K1/K2: correctness, wide A/B, production dispatch rows, stagger/priority knob at 64 MiB.
set -o pipefail
out=gpurun_out/r3o
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 \
  --timeout-method thread -m gpu > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -1 $out/pytest_kernels.log
timeout -k 10 300 build/native/crc_bench --wide-ab > $out/wide_ab.json 2> $out/wide_ab.err || exit $?
timeout -k 10 300 build/native/crc_bench > $out/crc_default.json 2> $out/crc_default.err || exit $?
python3 - <<'PY'
import json
e = json.load(open("gpurun_out/r3o/wide_ab.json"))
for r in e["k1k2"]:
    if r["bytes"] >= 32 << 20: print(r["bytes"] >> 20, r["wide"], r["rep"], r["us"], r["GBps"], r["ok"])
e = json.load(open("gpurun_out/r3o/crc_default.json"))
for r in e["k1k2"]:
    if r["impl"] == "dispatch": print(r)
print("scrub", e["scrub"][0])
PY
: > $out/tune.txt
for tune in 0 0x100; do
  r=$(DFS_CRC_WIDE_TUNE=$tune timeout -k 10 60 build/native/crc_bench --single 64 --iters 200 --mib 256) || exit $?
  echo "$tune 64 $r" | tee -a $out/tune.txt
done
