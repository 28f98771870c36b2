#!/bin/bash
# Is the fresh box's slow durable-write phase tied to time or to bytes first written?
# Ten 10-writer sweeps (600 x 1 MiB + 2 fdatasync each) back to back, with timestamps; no GPU.
set -o pipefail
out=gpurun_out/r3q
mkdir -p $out
t0=$(date +%s.%N)
for k in 1 2 3 4 5 6 7 8 9 10; do
  r=$(timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/r3q_sweep --cases 10:0) || exit $?
  t=$(date +%s.%N)
  echo "$k $(python3 -c "print(round($t-$t0,1))") $(echo $r | tr -d '\n' | cut -c1-160)" | tee -a $out/sweeps.txt
done
rm -rf /tmp/r3q_sweep
