#!/bin/bash
# Wide K1/K2 kernel: start stagger / priority knob sweep (DFS_CRC_WIDE_TUNE) at 64 MiB and 1 GiB.
set -o pipefail
out=gpurun_out/r3n
mkdir -p $out
: > $out/tune.txt
for tune in 0 4 8 16 24 32 0x100 0x108 0x110 0; do
  for mib in 64 1024; do
    r=$(DFS_CRC_WIDE_TUNE=$tune timeout -k 10 60 build/native/crc_bench --single $mib --iters 200 --mib 1024) || exit $?
    echo "$tune $mib $r" | tee -a $out/tune.txt
  done
done
