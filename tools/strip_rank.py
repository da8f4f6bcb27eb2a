#!/usr/bin/env python3
"""One rank of an N-rank weak-scaling run, on one GPU (tuning aid).

Builds each requested rank's share of the N x E-event stream bench.py --gpus N
would run (the same per-rank generation and split: --split strips: x-strips
with the flow-halo exchange; strips-recompute; segments: temporal segments)
and times its step on device 0, one rank after the other.  For segments the
step is last_stamps + merge + seed + the warm-up and segment, the RCCL
all-gather itself (2 x 7.4 MB per rank) not timed; for strips it is the fit
sweep, the import of the halo flows (taken from a second handle that fits the
halo itself, so the flows are realistic) and the pooling sweep, the RCCL
send/recv itself not timed.
The N-GPU bench value is then predicted as N x E / max-over-ranks step time;
the driver's own N-GPU run is the measurement.
"""
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
import segments  # noqa: E402
import strips  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8, help="strips (simulated GPUs)")
ap.add_argument("--ranks", default="", help="comma list; default: all")
ap.add_argument("--events", type=int, default=50_000_000, help="events per GPU")
ap.add_argument("--fit", default="0")
ap.add_argument("--pool", type=int, default=0, help="pooling chunk (0: the engine's default)")
ap.add_argument("--batch", type=int, default=0, help="pooling chunks per super-chunk (0: default)")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--split", choices=("strips", "strips-recompute", "segments"), default="strips")
a = ap.parse_args()

W, H, fs, maxw, jump = 1280, 720, 5, 50, 5
sp = farms.synth_params(3)
sp.n_events = n_stream = a.events * a.n
exch = a.split == "strips"
if a.split != "segments":
    t0 = time.time()
    plan = strips.plan_hist(farms.synth_column_hist(sp), H, a.n, fs, maxw, exchange=exch)
    print(f"column histogram of {n_stream} events in {time.time() - t0:.1f} s", flush=True)
ranks = [int(r) for r in a.ranks.split(",")] if a.ranks else range(a.n)
dev = torch.device("cuda", 0)
for fc in [int(v) for v in a.fit.split(",")]:
    worst = 0.0
    for r in ranks:
        t0 = time.time()
        if a.split != "segments":
            s = plan[r]
            ev, _, tf = farms.synth_select(sp, 0, n_stream, s.reg_lo, s.reg_hi)
            x, y, t, p = ev.relative(tf)
            owned = int(strips.owned_mask(x, s).sum())
            region, own, cols = (s.reg_lo, s.reg_hi), (s.own_lo, s.own_hi), [s.own_lo, s.own_hi]
        else:
            lo, hi = segments.rank_window(n_stream, a.n, r)
            ev, _, tf = farms.synth_select(sp, lo, hi)
            x, y, t, p = ev.relative(tf)
            s, n_head = segments.plan_rank(t, lo, n_stream, a.n, r)
            x, y, t, p = (v[s.warm - lo:s.end - lo] for v in (x, y, t, p))
            owned = s.end - s.start
            region, own, cols = None, None, [s.start, s.end]
        print(f"rank {r}: {len(x)} events generated in {time.time() - t0:.1f} s", flush=True)
        dx = torch.from_numpy(x).to(dev)
        dy = torch.from_numpy(y).to(dev)
        dt = torch.from_numpy(t.view(np.int32)).to(dev)
        dp = torch.from_numpy(p).to(dev)
        n = len(dx)
        out = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
               for c in farms.COLUMNS[4:]}
        fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw, fit_chunk=fc, pool_chunk=a.pool,
                               pool_batch=a.batch, region=region, owned=own, import_halo=exch)
        if exch:  # realistic halo flows: a handle that fits the halo itself
            halo = np.flatnonzero(~strips.owned_mask(x, s)).astype(np.int32)
            hidx = torch.from_numpy(halo).to(dev)
            hflows = torch.empty((len(halo), 3), dtype=torch.float64, device=dev)
            with farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw, fit_chunk=fc,
                                   region=region) as fh:
                fh.fit_device(dx, dy, dt, dp, out)
                fh.export_flows(hidx, hflows)
                fh.pool_device()
        if a.split == "segments":  # the surfaces of the ranks before this one: stand-ins of the right shape
            mine = torch.empty((2, W * H), dtype=torch.int64, device=dev)
            rows = max(len(segments.merge_rows(r)), 1)
            stack = torch.full((rows, W * H), -1, dtype=torch.int64, device=dev)
            sae = torch.empty(W * H, dtype=torch.int64, device=dev)
            o = s.n_warm

        def run():
            if exch:
                fm.fit_device(dx, dy, dt, dp, out)
                fm.import_flows(hidx, hflows)
                fm.pool_device()
                return
            if a.split == "segments":
                fm.last_stamps(dx[o:], dy[o:], dt[o:], n_head, mine[0], mine[1])
                if r > 0:
                    fm.merge_stamps(stack, sae)
                    fm.seed_sae(sae)
            fm.process_device(dx, dy, dt, dp, out)
        run()  # warmup
        best = 1e9
        for _ in range(a.reps):
            fm.reset()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            run()
            best = min(best, time.perf_counter() - t1)
        fm.set_profiling(farms.PROF_TIMING)
        fm.reset()
        run()
        st = fm.stats()
        fm.close()
        worst = max(worst, best)
        print(json.dumps({"n": a.n, "rank": r, "fit_chunk": fc, "pool_chunk": a.pool, "batch": a.batch, "split": a.split, "range": cols, "stored": n,
                          "owned": owned, "ms": round(best * 1e3, 1), "ms_fit_sweep": round(st["ms_fit"], 1),
                          "ms_pool_sweep": round(st["ms_pool"], 1), "ms_fit_k": round(st["ms_fit_kernel"], 1),
                          "ms_pool_k": round(st["ms_pool_kernel"], 1)}), flush=True)
        del dx, dy, dt, dp, out
        torch.cuda.empty_cache()
    print(json.dumps({"n": a.n, "fit_chunk": fc, "predicted_Mev_s": round(a.n * a.events / worst / 1e6, 1),
                      "worst_ms": round(worst * 1e3, 1)}), flush=True)
