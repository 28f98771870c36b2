#!/bin/bash
# K3 fused verify+copy read vs verify kernel + SDMA copy, store level (io_bench, registered
# client buffers), alternating; then a kernel trace of the fused run.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/fused
for rep in 1 2; do
  for f in 0 1; do
    DFS_FUSED_READ=$f timeout -k 10 300 build/native/io_bench --iters 30 > gpurun_out/fused/io_f${f}_$rep.json 2> gpurun_out/fused/io_f${f}_$rep.err || exit $?
  done
done
(cd /tmp && export TMPDIR=/tmp && DFS_FUSED_READ=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$OLDPWD/gpurun_out/fused/prof" -o io -- "$OLDPWD/build/native/io_bench" --iters 30) \
   > gpurun_out/fused/io_prof.json 2> gpurun_out/fused/io_prof.err || exit $?
echo fused done
