#!/bin/bash
# RS(6,3) end-to-end encode (registered host shards -> H2D -> K4 -> D2H) per pipeline chunk
# size (DFS_RS_CHUNK_KIB per shard per step), three runs each.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for kib in ${CHUNKS:-4096 2048 1024 512 256}; do
  for rep in 1 2 3; do
    DFS_RS_CHUNK_KIB=$kib timeout -k 10 120 build/native/io_bench --rs-only --dir /tmp/iob_rs \
      > gpurun_out/rs_chunk_${kib}_$rep.json 2> gpurun_out/rs_chunk_${kib}_$rep.err || exit $?
  done
done
