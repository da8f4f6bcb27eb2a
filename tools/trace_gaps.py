#!/usr/bin/env python3
"""Where a call's wall time goes, from a rocprofv3 kernel trace (diagnostic).

usage: trace_gaps.py KERNEL_TRACE.csv [--call -1] [--head 40] [--gap-us 3]
For the chosen farms call (the k_prep-started calls of the trace; -1 = the last),
prints: the call's span; the time no kernel of the call runs (device idle),
listed by gap; the head (first k_prep to the first pooling launch) and the tail
(the last fit or pooling kernel to the end); per kernel type its launches,
summed and union durations; the first HEAD kernels with start / end offsets
and their queue."""
import argparse
import collections
import csv
import re


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--call", type=int, default=-1)
    ap.add_argument("--head", type=int, default=40)
    ap.add_argument("--gap-us", type=float, default=3.0)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:28]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?")))
    rows.sort()
    preps = [i for i, r in enumerate(rows) if r[2] == "k_prep"]
    lo = preps[a.call]
    hi = preps[a.call + 1] if a.call != -1 and a.call + 1 < len(preps) else len(rows)
    sel = [r for r in rows[lo:hi] if r[2] not in ("k_stats",)]
    t0 = sel[0][0]
    t1 = max(r[1] for r in sel)
    us = lambda v: (v - t0) / 1e3  # noqa: E731
    print(f"call {a.call} of {len(preps)}: span {(t1 - t0) / 1e3:.1f} us, {len(sel)} kernels")
    busy = union([(s, e) for s, e, *_ in sel])
    print(f"device busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
    # idle gaps
    cur = t0
    gaps = []
    for s, e, k, q in sorted(sel):
        if s > cur and (s - cur) / 1e3 >= a.gap_us:
            gaps.append((us(cur), (s - cur) / 1e3, k))
        cur = max(cur, e)
    for g0, d, k in gaps[:30]:
        print(f"  idle at {g0:9.1f} us for {d:7.1f} us (then {k})")
    if len(gaps) > 30:
        print(f"  ... {len(gaps) - 30} more gaps, {sum(d for _, d, _ in gaps[30:]):.1f} us")
    pools = [r for r in sel if r[2].startswith("k_pool") and r[2] not in ("k_pool_desc", "k_pool_compact")]
    fits = [r for r in sel if r[2].startswith("k_fit")]
    if pools:
        print(f"head: first pooling launch at {us(pools[0][0]):.1f} us")
    last_work = max([r[1] for r in pools + fits] or [t1])
    print(f"tail: {(t1 - last_work) / 1e3:.1f} us after the last fit / pooling kernel")
    byk = collections.defaultdict(list)
    for s, e, k, q in sel:
        byk[k].append((s, e))
    for k, iv in sorted(byk.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        print(f"  {k:28s} n={len(iv):5d} sum {sum(e - s for s, e in iv) / 1e3:9.1f} us  union {union(iv) / 1e3:9.1f} us")
    for s, e, k, q in sel[:a.head]:
        print(f"    {us(s):9.1f} .. {us(e):9.1f}  q{q:>3s}  {k}")


if __name__ == "__main__":
    main()
