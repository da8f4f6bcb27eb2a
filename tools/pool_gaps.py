#!/usr/bin/env python3
"""Where the pooling stream waits in the last call of a rocprofv3 kernel trace
(rocpd SQLite): per super-chunk, the k_pool launch, the idle gap before it on
its stream, and the chain-stream kernels (k_flow, k_cand / k_chain,
k_pool_desc) that produced its candidate lists, with the fit launches still
running.  usage: pool_gaps.py results.db"""
import collections
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end, stream_id from kernels order by start").fetchall()


def short(n):
    m = re.search(r"(k_[a-z_]+)(<[^(]*>)?\(", n)
    return m.group(1) + (m.group(2) or "") if m else n[:40]


preps = [r[1] for r in rows if short(r[0]).startswith("k_prep")]
t0 = preps[-1]
last = [(short(n), (s - t0) / 1e3, (e - t0) / 1e3, sid) for n, s, e, sid in rows if s >= t0]
end = max(r[2] for r in last)
print(f"last call: {end / 1e3:.2f} ms from k_prep")
agg = collections.defaultdict(lambda: [0, 0.0])
for k, s, e, _ in last:
    agg[k][0] += 1
    agg[k][1] += e - s
for k, (cnt, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:32s} {cnt:6d} {us / 1e3:9.2f} ms {us / cnt:9.1f} us")
pools = [r for r in last if r[0].startswith("k_pool<")]
psid = pools[0][3]
csid = next(r[3] for r in last if r[0] == "k_pool_desc")
print(f"pool stream {psid}, chain stream {csid}")
prev_end = None
idle = 0.0
for i, (k, s, e, sid) in enumerate(pools):
    gap = s - prev_end if prev_end is not None else s
    idle += gap if prev_end is not None else 0.0
    # chain-stream kernels that ended in (prev pool start, this pool start]
    ch = [r for r in last if r[3] == csid and r[2] <= s and (i == 0 or r[2] > pools[i - 1][1])]
    desc = " ".join(f"{r[0]}:{r[2] - r[1]:.0f}" for r in ch if r[0] != "k_chain")
    fits = sum(1 for r in last if r[0].startswith("k_fit") and r[1] < e and r[2] > s)
    print(f"S{i:3d} start {s / 1e3:8.2f} ms dur {e - s:7.1f} us gap {gap:7.1f} us fits-overlap {fits:3d} | {desc}")
    prev_end = e
print(f"pool stream idle between launches: {idle / 1e3:.2f} ms")
