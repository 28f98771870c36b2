#!/bin/bash
# K1/K2 wide kernel with 2 vs 3 groups per CU: correctness (wide-mode tests) then the A/B
# (crc_bench --wide-ab: mode 0 = 12-wave narrow, 1 = 3 groups, 2 = 2 groups).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "wide or crc" > $O/pytest_wide.log 2>&1 && \
timeout -k 10 300 build/native/crc_bench --wide-ab > $O/wide_ab.json 2> $O/wide_ab.err && \
timeout -k 10 300 build/native/crc_bench > $O/crc_default.json 2> $O/crc_default.err
