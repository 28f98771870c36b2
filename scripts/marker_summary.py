"""Aggregate a rocprofv3 marker trace by phase: roctx range names carry the request id as a
"[rid]" suffix (csrc/trace.h), so the tool's own stats list one row per request. Usage:
python scripts/marker_summary.py <..._marker_api_trace.csv>  -> per-phase count / p50 / p99 / mean (us)"""
import collections
import csv
import re
import sys

durs = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\s*\[[0-9a-f]+\]$", "", r.get("Function") or r.get("Name") or "")
    try:
        durs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    except (KeyError, ValueError):
        continue
print(f"{'phase':<28}{'count':>8}{'p50_us':>10}{'p99_us':>10}{'mean_us':>10}")
for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{name:<28}{len(v):>8}{v[len(v) // 2]:>10.1f}{v[min(len(v) - 1, int(len(v) * 0.99))]:>10.1f}"
          f"{sum(v) / len(v):>10.1f}")
