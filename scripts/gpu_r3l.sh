#!/bin/bash
# Interleaved MFMA chains in the CRC kernels: correctness + K1/K2 / scrub throughput.
set -o pipefail
out=gpurun_out/r3l
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_replication.py -x -q --timeout 120 \
  --timeout-method thread -m gpu > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -2 $out/pytest_kernels.log
timeout -k 10 300 build/native/crc_bench > $out/crc_default.json 2> $out/crc_default.err || exit $?
timeout -k 10 300 build/native/crc_bench --sweep --mib 256 --iters 30 > $out/crc_sweep.json 2> $out/crc_sweep.err || exit $?
python3 - <<'PY'
import json
e = json.load(open("gpurun_out/r3l/crc_default.json"))
for r in e["k1k2"]:
    if r["impl"] == "dispatch": print(r)
print("scrub", e["scrub"][0])
d = json.load(open("gpurun_out/r3l/crc_sweep.json"))
for r in d["k1k2"]:
    if r["bytes"] == 64 << 20 and r["ring"] == 2: print(r)
PY
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --remote-steps 10 > $out/bench.json 2> $out/bench.err || exit $?
python -c "import json; d=json.load(open('$out/bench.json')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','client_phase_p50_ms_rank0','remote_client') if k in d})"
