#!/usr/bin/env python3
"""Per-kernel totals and per-stream busy intervals of the last N k_prep-delimited
calls in a rocprofv3 SQLite output (rocpd): where a strip rank's step goes.
usage: rocpd_timeline.py results.db [calls_back]"""
import collections
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
back = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = db.execute("select name, start, end, stream_id from kernels order by start").fetchall()


def short(n):
    m = re.search(r"(k_[a-z_]+)(<[^(]*>)?\(", n)
    return m.group(1) + (m.group(2) or "") if m else n[:40]


preps = [r[1] for r in rows if short(r[0]).startswith("k_prep")]
t0 = preps[-back]
last = [(short(n), (s - t0) / 1e6, (e - t0) / 1e6, sid) for n, s, e, sid in rows if s >= t0]
print(f"window {max(r[2] for r in last):.1f} ms over the last {back} calls")
agg = collections.defaultdict(lambda: [0, 0.0])
for k, s, e, _ in last:
    agg[k][0] += 1
    agg[k][1] += e - s
for k, (cnt, ms) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:40s} {cnt:6d} {ms:9.2f} ms {ms / cnt * 1e3:8.1f} us")
for sid in sorted({r[3] for r in last}):
    segs = []
    for k, s, e, x in last:
        if x != sid:
            continue
        if segs and s - segs[-1][1] < 0.3:
            segs[-1][1] = max(segs[-1][1], e)
        else:
            segs.append([s, e])
    busy = sum(b - a for a, b in segs)
    print(f"stream {sid}: busy {busy:.1f} ms in {len(segs)} stretches:",
          " ".join(f"{a:.1f}-{b:.1f}" for a, b in segs[:24]))
