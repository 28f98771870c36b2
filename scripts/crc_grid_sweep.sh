#!/bin/bash
# crc_bench under different minimum tiles per workgroup (small-block launch shape sweep)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for p in 1 2 4 8; do
  DFS_CRC_MIN_TILES_PER_WG=$p timeout -k 10 120 build/native/crc_bench --iters 200 --mib 64 > gpurun_out/crc_grid_$p.json 2> gpurun_out/crc_grid_$p.err || exit $?
done
