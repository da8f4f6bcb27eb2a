#!/usr/bin/env python3
"""How much of the sensor a k_chain launch touches (CPU, synthetic stream).

A k_chain launch walks one pooling super-chunk (64 chunks of 8,192 events at
C3) over every 256-cell group of the stored region.  For the review's "make
k_chain proportional to active cells" this counts, per super-chunk of the
config's stream: the groups with at least one event in it, the cells with at
least one event, and the cells whose events fall in the 500 us before it (the
candidates through a valid snapshot come from these).

usage: chain_activity.py [--config 3] [--events 5000000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
import farms  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--events", type=int, default=5_000_000)
ap.add_argument("--chunk", type=int, default=8192)
ap.add_argument("--batch", type=int, default=64)
a = ap.parse_args()
W, H = (320, 320) if a.config == 2 else (1280, 720)
ev = farms.synth_config(a.config, a.events)
x, y, t, _ = ev.relative()
lin = x.astype(np.int64) * H + y
t64 = t.astype(np.int64)
n, S = len(x), a.chunk * a.batch
ngroups = (W * H + 255) // 256
print(f"config {a.config}: {n} events over {int(t64[-1] - t64[0])} us, super-chunk {S} events, {ngroups} groups")
for s0 in range(0, n - S + 1, S):
    sl = slice(s0, s0 + S)
    g = np.unique(lin[sl] // 256).size
    cells = np.unique(lin[sl]).size
    lo = t64[sl].min() - 500
    recent = np.unique(lin[max(0, s0 - 4 * S):s0][t64[max(0, s0 - 4 * S):s0] >= lo]).size
    print(f"super-chunk {s0 // S}: groups touched {g} / {ngroups}, cells touched {cells} ({cells / (W * H):.0%}), "
          f"cells with events in the 500 us before {recent}, span {int(t64[sl].max() - t64[sl].min())} us")
