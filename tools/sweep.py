#!/usr/bin/env python3
"""Chunk-size sweep on one resident stream (tuning aid; not part of the bench contract)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import farms  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--events", type=int, default=50_000_000)
ap.add_argument("--fs", type=int, default=5)
ap.add_argument("--pool", default="8192,16384,32768,65536,131072")
ap.add_argument("--fit", default="1048576")
ap.add_argument("--batch", default="8")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()

W, H = (1280, 720) if a.config >= 3 else ((320, 320) if a.config == 2 else (128, 128))
ev = farms.synth_config(a.config, a.events)
x, y, t, p = ev.relative()
dev = torch.device("cuda", 0)
dx, dy = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
dt, dp = torch.from_numpy(t.view(np.int32)).to(dev), torch.from_numpy(p).to(dev)
n = len(ev)
out = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev) for c in farms.COLUMNS[4:]}
import itertools  # noqa: E402
for fc, pc, pb in itertools.product(*[[int(v) for v in s.split(",")] for s in (a.fit, a.pool, a.batch)]):
    if True:
        fm = farms.FlowManager(H, W, a.fs, 5, fit_chunk=fc, pool_chunk=pc, pool_batch=pb)
        fm.process_device(dx, dy, dt, dp, out)  # warmup
        best = 1e9
        for _ in range(a.reps):
            fm.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fm.process_device(dx, dy, dt, dp, out)
            best = min(best, time.perf_counter() - t0)
        fm.set_profiling(True)
        fm.reset()
        fm.process_device(dx, dy, dt, dp, out)
        st = fm.stats()
        fm.close()
        print(json.dumps({"fit_chunk": fc, "pool_chunk": pc, "pool_batch": pb, "ms": round(best * 1e3, 1),
                          "Mev_s": round(n / best / 1e6, 1), "ms_fit_k": round(st["ms_fit_kernel"], 1),
                          "ms_pool_k": round(st["ms_pool_kernel"], 1), "ms_fit_sweep": round(st["ms_fit"], 1),
                          "ms_pool_sweep": round(st["ms_pool"], 1), "ms_prep": round(st["ms_prep"], 1),
                          "valid": st["n_valid"],
                          "cand_per_valid": round(st["pool_candidates"] / max(st["n_valid"], 1), 1),
                          "contrib_per_valid": round(st["pool_contributors"] / max(st["n_valid"], 1), 1)}),
              flush=True)
