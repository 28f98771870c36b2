#!/bin/bash
# Round 3 batch: GPU kernel + replication tests, CRC bench (size-based dispatch), config 5
# with the native S3 front, durable write path A/B.
set -o pipefail
out=gpurun_out/r3c
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_replication.py -x -q \
  --timeout 120 --timeout-method thread -m gpu > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -3 $out/pytest_kernels.log
timeout -k 10 180 build/native/crc_bench > $out/crc_bench.json 2> $out/crc_bench.err || exit $?
python -c "import json; d=json.load(open('$out/crc_bench.json')); [print(e) for e in d['k1k2']]"
bash scripts/gpu_s3.sh && bash scripts/gpu_durable.sh
