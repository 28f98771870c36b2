"""Per-phase latency table from a rocprofv3 --marker-trace CSV directory (roctx ranges of
csrc/trace.h: dfs.store.write, dfs.grpc.read_block, ...). Usage: marker_phases.py DIR."""
import csv
import glob
import os
import sys


def main(d: str) -> None:
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                name = r.get("Function") or r.get("Operation") or ""
                if not name.startswith("dfs."):
                    continue
                name = name.split(" [", 1)[0]  # ranges carry "[request id]"
                try:
                    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                except (KeyError, ValueError):
                    continue
                rows.setdefault(name, []).append(us)
    print(f"{'phase':30s} {'count':>6s} {'p50_us':>9s} {'p99_us':>9s} {'mean_us':>9s}")
    for name, v in sorted(rows.items(), key=lambda kv: -len(kv[1])):
        v.sort()
        pick = lambda q: v[min(len(v) - 1, int(len(v) * q))]
        print(f"{name:30s} {len(v):6d} {pick(0.5):9.1f} {pick(0.99):9.1f} {sum(v) / len(v):9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
