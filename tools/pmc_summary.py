#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (totals and per wave)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    m = re.search(r"(k_\w+)(?:<(\d+)[^>]*>)?", r["Kernel_Name"])  # k_pool<11, true> -> k_pool<11>
    k = (m.group(1) + (f"<{m.group(2)}>" if m.group(2) else "")) if m else r["Kernel_Name"][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    w = v.get("SQ_WAVES", 0.0)
    print(f"{k}  dispatches={len(disp[k])}")
    for c, val in sorted(v.items()):
        per = f"  per-wave {val / w:.1f}" if w else ""
        print(f"   {c:24s} total {val:.4g}  per-dispatch {val / len(disp[k]):.4g}{per}")
