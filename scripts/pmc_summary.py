"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (LDS bank conflicts / LDS-active
cycles, VALU/LDS instruction ratio). Usage: python scripts/pmc_summary.py <counter_collection.csv>"""
import collections
import csv
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(\w+)\(", r["Kernel_Name"])
    agg[m.group(1) if m else r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    if not v.get("SQ_LDS_IDX_ACTIVE"):
        continue
    print(f"{k}: bank-conflict/LDS-active = {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.3f}, "
          f"VALU/LDS insts = {v['SQ_INSTS_VALU'] / max(1.0, v['SQ_INSTS_LDS']):.1f}, "
          f"LDS-active cycles = {int(v['SQ_LDS_IDX_ACTIVE'])}, waves = {int(v['SQ_WAVES'])}")
