#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: both counters are
in KiB; on gfx950 FETCH_SIZE tallies 128-B memory-side read requests at 64 B, so
it is doubled; WRITE_SIZE is taken as is.  Per kernel (templated name kept):
    traffic_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 / dispatches

usage: traffic.py FETCH_CSV WRITE_CSV [--label L] > profiles/rNN_traffic_*.json
"""
import argparse
import collections
import csv
import json
import re


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(k_\w+)(?:<(\d+)[^>]*>)?", r["Kernel_Name"])  # k_pool<11, true> -> k_pool<11>
        k = (m.group(1) + (f"<{m.group(2)}>" if m.group(2) else "")) if m else r["Kernel_Name"][:40]
        tot[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    f, fd = per_kernel(a.fetch_csv, "FETCH_SIZE")
    w, wd = per_kernel(a.write_csv, "WRITE_SIZE")
    out = {"label": a.label, "formula": "(2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 / dispatches", "kernels": {}}
    for k in sorted(set(f) & set(w)):
        nf, nw = fd[k], wd[k]
        fetch_b = f[k] * 1024 / nf
        write_b = w[k] * 1024 / nw
        out["kernels"][k] = {"dispatches": nf, "fetch_size_kib_per_launch": f[k] / nf,
                             "write_size_kib_per_launch": w[k] / nw,
                             "traffic_bytes_per_launch": 2 * fetch_b + write_b}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
