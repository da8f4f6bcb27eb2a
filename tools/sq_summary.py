#!/usr/bin/env python3
"""SQ counters per kernel from one rocprofv3 --pmc pass (tools/gpu_sq.sh).

usage: sq_summary.py COUNTER_CSV [--label L] > profiles/rNN_sq_c<cfg>.json
Per kernel (templated name kept): dispatches and each counter's total per launch.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
(/opt/skills/guides/MI355X_MICROARCH.md, PMC section); ratios between them are
what bench.py reports.
"""
import argparse
import collections
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        m = re.search(r"(k_\w+)(?:<(\d+)[^>]*>)?", r["Kernel_Name"])  # k_pool<11, true> -> k_pool<11>
        k = (m.group(1) + (f"<{m.group(2)}>" if m.group(2) else "")) if m else r["Kernel_Name"][:40]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {"label": a.label, "per": "launch", "kernels": {}}
    for k in sorted(tot):
        nd = len(disp[k])
        out["kernels"][k] = dict({c: v / nd for c, v in sorted(tot[k].items())}, dispatches=nd)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
