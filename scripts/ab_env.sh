#!/bin/bash
# Same-box interleaved A/B of one environment knob on the driver's N=1 command:
#   scripts/ab_env.sh <out-dir> <reps> <VAR> <value-a> <value-b> [<value-c>]
# Each rep runs every value once, in order; every run is its own `timeout -k`, and the first
# failure ends the session (no GPU work after a fault, an abort or a time limit).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:?out dir}; reps=${2:?reps}; var=${3:?var}
shift 3
mkdir -p "$O"
for r in $(seq 1 "$reps"); do
  for v in "$@"; do
    echo "[ab_env] rep $r $var=$v" >&2
    env "$var=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/${var}_${v}_$r.json" 2> "$O/${var}_${v}_$r.err" \
      || { echo "[ab_env] $var=$v rep $r failed rc=$?" >&2; tail -20 "$O/${var}_${v}_$r.err" >&2; exit 1; }
    python - "$O/${var}_${v}_$r.json" <<'PY' >&2
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = d["client_phase_p50_ms_rank0"]
print(f"  value {d['value']} write {d['write_mb_per_s']} p50 {d['write_p50_ms']} p99 {d['write_p99_ms']} "
      f"write-phase {ph['write']} complete {ph['complete']} md5_wait {ph['md5_wait']} "
      f"sync/round {d['journal']['sync_ns'] / max(1, d['journal']['sync_rounds']) / 1e6:.3f} ms")
PY
  done
done
echo "[ab_env] done" >&2
