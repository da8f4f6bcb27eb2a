#!/usr/bin/env python3
"""Enqueue-to-start lag of kernels (diagnostic), from one rocprofv3 run with
--kernel-trace --hip-trace (csv): for each launch of the named kernels, when
the host's launch call returned and when the kernel started / ended on the
device, plus what ran on the device in between.

usage: enqueue_lag.py KERNEL_TRACE.csv HIP_API_TRACE.csv [--kernels k_pool2,k_cand] [--last 40]
Launches are matched by correlation id.  Times in ms from the first record."""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kt")
    ap.add_argument("api")
    ap.add_argument("--kernels", default="k_pool2,k_pool,k_cand,k_flow,k_fit_quad")
    ap.add_argument("--last", type=int, default=60)
    a = ap.parse_args()
    want = a.kernels.split(",")
    api = {}
    t_first = None
    for r in csv.DictReader(open(a.api)):
        cid = r.get("Correlation_Id")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        api[cid] = (s, e, r.get("Function", r.get("Operation", "")))
        t_first = s if t_first is None else min(t_first, s)
    rows = []
    for r in csv.DictReader(open(a.kt)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:24]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        rows.append((s, e, name, r.get("Queue_Id", "?"), r.get("Correlation_Id")))
        t_first = s if t_first is None else min(t_first, s)
    rows.sort()
    ms = lambda v: (v - t_first) / 1e6  # noqa: E731
    sel = [r for r in rows if r[2] in want]
    for s, e, name, q, cid in sel[-a.last:]:
        c = api.get(cid)
        call = f"launched {ms(c[1]):9.3f}" if c else "launched       ?"
        lag = f"lag {((s - c[1]) / 1e3 if c else 0):8.1f} us" if c else ""
        print(f"{name:12s} q{q:>3s} {call}  start {ms(s):9.3f} end {ms(e):9.3f}  {lag}")


if __name__ == "__main__":
    main()
