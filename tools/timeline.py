#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 kernel trace: for the last farms_process call
(between the last k_prep and the last k_pool), busy time per stream, the
overlap of streams, and per-kernel totals (tuning aid)."""
import collections
import csv
import re
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:30],
                 r["Stream_Id"], r["Queue_Id"]))
rows.sort()
preps = [i for i, r in enumerate(rows) if r[2] == "k_prep"]
lo = preps[-1]
t0 = rows[lo][0]
sel = [r for r in rows[lo:] if r[2] != "k_stats"]
t1 = max(r[1] for r in sel)
print(f"span {(t1 - t0) / 1e6:.2f} ms, {len(sel)} kernels")


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


by_stream = collections.defaultdict(list)
by_kernel = collections.defaultdict(list)
for s, e, k, st, q in sel:
    by_stream[(st, q)].append((s, e))
    by_kernel[k].append((s, e))
print(f"any-kernel busy {union([(s, e) for s, e, *_ in sel]) / 1e6:.2f} ms")
for key, iv in sorted(by_stream.items()):
    ks = collections.Counter(k for s, e, k, st, q in sel if (st, q) == key)
    print(f"stream/queue {key}: busy {union(iv) / 1e6:.2f} ms  kernels {dict(ks.most_common(4))}")
for k, iv in sorted(by_kernel.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
    print(f"  {k:24s} n={len(iv):6d} sum {sum(e - s for s, e in iv) / 1e6:8.2f} ms  union {union(iv) / 1e6:8.2f} ms")
