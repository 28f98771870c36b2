#!/bin/bash
# Sliced head writes with the descriptor announced before the first slice: GPU replication
# tests, then the 64 MiB RF=3 timeline under rocprofv3.
set -o pipefail
out=gpurun_out/r3h
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_replication.py tests/test_gpu_ipc.py tests/test_gpu_cluster.py -x -v \
  --timeout 180 --timeout-method thread -p no:cacheprovider -m gpu > $out/pytest_repl.log 2>&1 || { tail -40 $out/pytest_repl.log; exit 1; }
tail -3 $out/pytest_repl.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
   -d "$OLDPWD/$out/prof_sliced" -o st -- python3 "$OLDPWD/scripts/sliced_timeline.py") > $out/sliced.log 2>&1 || { tail -20 $out/sliced.log; exit 1; }
grep -v "^W2\|^E2" $out/sliced.log | tail -8
python3 scripts/sliced_timeline.py --summary $out/prof_sliced | tee $out/sliced_summary.txt
DFS_SLICED_WRITE_MIN_MIB=0 timeout -k 10 300 python3 scripts/sliced_timeline.py > $out/unsliced.log 2>&1 || { tail -20 $out/unsliced.log; exit 1; }
grep -v "^W2\|^E2" $out/unsliced.log | tail -6
