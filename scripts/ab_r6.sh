#!/bin/bash
# Same-box A/B of the driver's N=1 command, interleaved: `scripts/ab_r6.sh <out-dir> <reps> <variant>...`
#   head     this tree
#   oldgrow  this tree with the journal topping up spares under load (round 5's behaviour)
#   r4       the round-4 tree (git worktree at 435766d in ab_r4/, built in place)
#   r5       the round-5 tree (git worktree at 6116051 in ab_r5/, built in place)
#   name:VAR=v[,VAR2=w]  this tree with those environment variables
# Every run is under its own time limit; the first failure ends the session.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:?out dir}
REPS=${2:?reps}
shift 2
mkdir -p "$O"
for i in $(seq 1 "$REPS"); do
  for v in "$@"; do
    case "$v" in
      head)    (timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$O/${v}_$i.json" 2> "$O/${v}_$i.err") ;;
      oldgrow) (DFS_JOURNAL_SPARES_LOW=1000 timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
                  > "$O/${v}_$i.json" 2> "$O/${v}_$i.err") ;;
      r4)      (cd ab_r4 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "../$O/${v}_$i.json" \
                  2> "../$O/${v}_$i.err") ;;
      r5)      (cd ab_r5 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "../$O/${v}_$i.json" \
                  2> "../$O/${v}_$i.err") ;;
      *:*)     (name=${v%%:*}; envs=${v#*:}; env ${envs//,/ } timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
                  > "$O/${v%%:*}_$i.json" 2> "$O/${v%%:*}_$i.err") ;;
      *) echo "unknown variant $v" >&2; exit 2 ;;
    esac
    rc=$?
    v=${v%%:*}
    [ $rc -eq 0 ] || { echo "[ab] $v run $i failed rc=$rc" >&2; tail -20 "$O/${v}_$i.err" >&2; exit 1; }
    python - "$O/${v}_$i.json" "$v" "$i" <<'EOF' >&2
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
j = d.get("journal") or {}
print(f"[ab] {sys.argv[2]} #{sys.argv[3]}: {d['value']} MB/s write {d['write_mb_per_s']} p50 {d['write_p50_ms']} "
      f"p99 {d['write_p99_ms']} complete {d.get('client_phase_p50_ms_rank0', {}).get('complete')} "
      f"exported {j.get('materialized_blocks')} timed {j.get('timed_region')}")
EOF
  done
done
echo "[ab] done" >&2
