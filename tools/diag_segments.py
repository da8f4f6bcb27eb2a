#!/usr/bin/env python3
"""Diagnostic: the engine segment scenario of tests/test_segments.py step by
step, printing progress (flushed) so a failing step is identified."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import farms  # noqa: E402
import segments  # noqa: E402

cfg, n, fs, nseg = (int(v) for v in sys.argv[1:5])
W, H = (1280, 720) if cfg == 3 else (320, 320)
x, y, t, p = farms.synth_config(cfg, n).relative()
segs = segments.plan(t, nseg)
dev = torch.device("cuda", 0)
skip_seed = os.environ.get("DIAG_NO_SEED") == "1"
for r, s in enumerate(segs):
    sl = slice(s.warm, s.end)
    print("segment", r, s, "seed" if r and not skip_seed else "fresh", flush=True)
    with farms.FlowManager(H, W, fs, 5) as fm:
        if r > 0 and not skip_seed:
            sae = torch.from_numpy(segments.last_stamps_np(x[:s.warm], y[:s.warm], t[:s.warm], W, H)).to(dev)
            fm.seed_sae(sae)
            print("  seeded", flush=True)
        rec = fm.process(x[sl], y[sl], t[sl], p[sl])
        print("  processed", int((rec.r_local > 0).sum()), flush=True)
print("done", flush=True)
