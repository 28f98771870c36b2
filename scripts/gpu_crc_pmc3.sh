#!/bin/bash
# Where the K1/K2 tile kernel's cycles go (64 MiB and 256 MiB blocks): wave-state and
# instruction-mix counters, one pass per counter group, each under a hard time limit.
set -o pipefail
out=gpurun_out/r3_pmc
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="$PWD/build/native/crc_bench"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$OLDPWD/$out/avail.txt" 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" "$OLDPWD/$out/avail.txt" | sort -u > "$OLDPWD/$out/sq_counters.txt" || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES"
for mib in 64 256; do
  timeout -s KILL 60 rocprofv3 --pmc $P1 --output-format csv -d "$OLDPWD/$out/p1_$mib" -o p -- "$B" --single $mib --iters 20 \
    > "$OLDPWD/$out/p1_$mib.log" 2>&1 || { tail -5 "$OLDPWD/$out/p1_$mib.log"; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $P2 --output-format csv -d "$OLDPWD/$out/p2_$mib" -o p -- "$B" --single $mib --iters 20 \
    > "$OLDPWD/$out/p2_$mib.log" 2>&1 || { tail -5 "$OLDPWD/$out/p2_$mib.log"; exit 1; }
done
cd "$OLDPWD"
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob("gpurun_out/r3_pmc/p*_*")):
    if not glob.os.path.isdir(d): continue
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "crc_" not in r.get("Kernel_Name", ""): continue
            agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print("==", d)
    for (k, c), v in sorted(agg.items()):
        print(f"  {k:40s} {c:28s} mean/dispatch {sum(v)/len(v):14.0f}  (n={len(v)})")
PY
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --remote-steps 10 > $out/bench_remote.json 2> $out/bench_remote.err || exit $?
python -c "import json; d=json.load(open('$out/bench_remote.json')); print(d['client_phase_p50_ms_rank0']); print(d['remote_client'])"
