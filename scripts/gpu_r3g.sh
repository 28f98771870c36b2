#!/bin/bash
# Full GPU tier + smoke, the sliced-write timeline under rocprofv3, the K1/K2 sweep.
set -o pipefail
out=gpurun_out/r3g
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider \
  > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
   -d "$OLDPWD/$out/prof_sliced" -o st -- python3 "$OLDPWD/scripts/sliced_timeline.py") > $out/sliced.log 2>&1 || { tail -20 $out/sliced.log; exit 1; }
cat $out/sliced.log | grep -v "^W2\|^E2" | tail -8
python3 scripts/sliced_timeline.py --summary $out/prof_sliced | tee $out/sliced_summary.txt
timeout -k 10 300 build/native/crc_bench --sweep --mib 256 --iters 30 > $out/crc_sweep.json 2> $out/crc_sweep.err || exit $?
cat $out/crc_sweep.json
bash scripts/gpu_s3.sh
