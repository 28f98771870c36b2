#!/bin/bash
# crc_bench (K1+K2 at several sizes, K1b scrub of 1 GiB) per register-ring depth of the MFMA
# kernels (2 = the 3-waves/SIMD kernels, 3..4 = the deep-ring kernels; the same depth for the
# scrub and for K1/K2 launches of >= 32 MiB), then the GPU kernel tests under each depth in
# TEST_RINGS.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in ${RINGS:-2 3 4}; do
  DFS_CRC_RING=$r DFS_CRC_TILE_RING=$r timeout -k 10 120 build/native/crc_bench --iters 100 > gpurun_out/crc_ring_$r.json 2> gpurun_out/crc_ring_$r.err || exit $?
done
for r in ${TEST_RINGS:-}; do
  DFS_CRC_RING=$r DFS_CRC_TILE_RING=$r timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_kernels.py > gpurun_out/crc_ring_test_$r.log 2>&1 || exit $?
done
