#!/usr/bin/env python3
"""Phase breakdown of the last traced step in a rocprofv3 kernel trace
(tools/gpu_r05_strips.sh: one x-strip rank step, or the N = 1 step).

The last step starts at the k_prep of its first call: a strip step runs 8
sub-batch calls (8 k_prep), a one-call step one.  For that window it prints the
span, and per phase the kernels' summed durations and their union on the
device timeline:
  prep   k_prep, the sorts, k_link, the work order and descriptors, the plans
  fit    k_fit_quad / k_fit / k_fit_wave / k_fit_prep
  flow   k_flow
  cand   k_cand / k_chain / k_cand_commit / k_cand_list
  pool   k_pool / k_pool2 / k_pool_desc / k_pool_compact / k_true_polar
  halo   k_export_flows / k_import_flows
plus the time no kernel runs (gaps) and each phase's share of the span.

usage: strip_trace.py KERNEL_TRACE_CSV [--label L] [--preps N]
"""
import argparse
import collections
import csv
import re

PHASES = [
    ("fit", ("k_fit_quad", "k_fit_wave", "k_fit_prep", "k_fit")),
    ("flow", ("k_flow",)),
    ("cand", ("k_cand_commit", "k_cand_list", "k_cand_plan", "k_cand", "k_chain")),
    ("pool", ("k_pool_compact", "k_pool_desc", "k_pool2", "k_pool", "k_true_polar")),
    ("halo", ("k_export_flows", "k_import_flows")),
]


def phase_of(name):
    for ph, keys in PHASES:
        for k in keys:
            if name == k or name.startswith(k + "<"):
                return ph
    return "prep"


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
    ap.add_argument("csv")
    ap.add_argument("--label", default="")
    ap.add_argument("--preps", type=int, default=0, help="k_prep launches per step (0: guess 8, else 1)")
    ap.add_argument("--timeline", action="store_true", help="per-stream busy fraction in 2-ms bins")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Stream_Id", ""),
                     r.get("Queue_Id", "")))
    rows.sort()
    preps = [i for i, r in enumerate(rows) if r[2] == "k_prep"]
    per = a.preps or (8 if len(preps) >= 16 else 1)
    lo = preps[len(preps) - per]
    queues = collections.defaultdict(set)  # the hardware queue(s) each stream's kernels went through
    for r in rows:
        queues[r[3]].add(r[4])
    sel = [r[:4] for r in rows[lo:] if r[2] != "k_stats"]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    span = t1 - t0
    busy = union([(s, e) for s, e, *_ in sel])
    print(f"{a.label}: last step = {per} call(s) from the {len(preps) - per + 1}-th k_prep; "
          f"span {span / 1e6:.2f} ms, any kernel running {busy / 1e6:.2f} ms, none {(span - busy) / 1e6:.2f} ms")
    by = collections.defaultdict(list)
    names = collections.defaultdict(lambda: [0, 0])
    for s, e, k, st in sel:
        by[phase_of(k)].append((s, e))
        names[k][0] += 1
        names[k][1] += e - s
    print(f"{'phase':6s} {'launches':>8s} {'sum ms':>9s} {'union ms':>9s} {'union/span':>10s}")
    for ph in ("prep", "fit", "flow", "cand", "pool", "halo"):
        iv = by.get(ph, [])
        print(f"{ph:6s} {len(iv):8d} {sum(e - s for s, e in iv) / 1e6:9.2f} {union(iv) / 1e6:9.2f} "
              f"{union(iv) / span:10.3f}")
    # per stream: busy union and the kernels it ran, then a coarse timeline
    # (fraction of each 2-ms bin during which the stream runs a kernel)
    streams = collections.defaultdict(list)
    for s, e, k, st in sel:
        streams[st].append((s, e, k))
    print("streams:")
    for st, iv in sorted(streams.items()):
        ks = collections.Counter(k for _, _, k in iv)
        print(f"  stream {st} (queue {','.join(sorted(queues[st]))}): busy {union([(s, e) for s, e, _ in iv]) / 1e6:8.2f} ms"
              f"  {dict(ks.most_common(4))}")
    if a.timeline:
        nb = int(span // 2_000_000) + 1
        print("timeline (2-ms bins, busy fraction per stream: " + " ".join(sorted(streams)) + ")")
        for b in range(nb):
            b0, b1 = t0 + b * 2_000_000, t0 + (b + 1) * 2_000_000
            fr = []
            for st in sorted(streams):
                iv = [(max(s, b0), min(e, b1)) for s, e, _ in streams[st] if e > b0 and s < b1]
                fr.append(union(iv) / 2_000_000)
            print(f"  {b * 2:5d} ms " + " ".join(f"{f:4.2f}" for f in fr))
    print("kernels:")
    for k, (n, tot) in sorted(names.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:24s} n={n:6d} sum {tot / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
