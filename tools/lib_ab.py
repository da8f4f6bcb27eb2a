#!/usr/bin/env python3
"""Device-resident step time of engine builds side by side on one box (A/B of
builds across rounds: FARMS_HIP_LIB picks the library of each child process).

usage: lib_ab.py --config C --steps K LIB [LIB ...]   (paths relative to the
package directory, e.g. build/libfarms_hip.so build/libfarms_hip_r03.so)
Each build runs in its own process, twice in alternation (ABAB), on the same
synthetic stream; prints ms per step (best and mean) per run.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd")


def child(cfg, steps):
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    import farms

    W, H = (320, 320) if cfg == 2 else (1280, 720)
    fs = {2: 5, 3: 5, 4: 7, 5: 7}[cfg]
    jump = 25 if cfg == 5 else 5
    n = {4: 50_000_000, 5: 50_000_000}.get(cfg, 0) or None
    ev = farms.synth_config(cfg, n)
    x, y, t, p = ev.relative()
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in (x, y, t.view(np.int32), p)]
    o = {c: torch.empty(len(x), dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    # (FARMS_AB_POOL_BATCH / FARMS_AB_POOL_CHUNK: handle parameters for a sweep)
    kw = {k: int(os.environ[e]) for k, e in (("pool_batch", "FARMS_AB_POOL_BATCH"), ("pool_chunk", "FARMS_AB_POOL_CHUNK"))
          if os.environ.get(e)}
    fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=50, **kw)
    ts = []
    for i in range(steps + 1):
        fm.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fm.process_device(*d, o)
        torch.cuda.synchronize()
        if i:
            ts.append((time.perf_counter() - t0) * 1e3)
    h = int(torch.sum(o["scale"].to(torch.int64) * torch.arange(len(x), device=dev) % 1000003).item())
    print(json.dumps({"lib": os.environ.get("FARMS_HIP_LIB", "default"), "config": cfg, "events": len(x), **kw,
                      "ms_best": round(min(ts), 2), "ms_mean": round(sum(ts) / len(ts), 2), "scale_hash": h}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        child(a.config, a.steps)
        return
    rc = 0
    for _ in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, FARMS_HIP_LIB=lib)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--config", str(a.config),
                                "--steps", str(a.steps)], env=env, timeout=600)
            rc = rc or r.returncode
            if r.returncode:
                return r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
