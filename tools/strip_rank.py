#!/usr/bin/env python3
"""One rank of an N-rank weak-scaling run, on one GPU (tuning aid).

Builds each requested rank's share of the N x E-event stream bench.py --gpus N
would run (multirank.make_share: the same per-rank generation and split) and
times its step on device 0, one rank after the other:
  * segments: last_stamps + merge + seed + the warm-up and segment (the RCCL
    all-gather of 2 x 7.4 MB per rank not timed);
  * strips: the pipelined step of multirank.Stepper -- sub-batch b+1's fit and
    its halo import under the pooling of b -- with the halo flows taken from a
    second handle that fits the halo itself (realistic flows; the RCCL
    send/recv itself not timed);
  * strips-recompute: one process_device over the widened region.
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
import multirank  # noqa: E402
import segments  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8, help="ranks (simulated GPUs)")
ap.add_argument("--ranks", default="", help="comma list; default: all")
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--events", type=int, default=50_000_000, help="events per GPU")
ap.add_argument("--nsub", type=int, default=8, help="strips: sub-batches of the pipelined step")
ap.add_argument("--pool", type=int, default=0, help="pooling chunk (0: the engine's default)")
ap.add_argument("--fit-chunk", type=int, default=0, help="fit chunk (0: the engine's default)")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--split", choices=multirank.SPLITS, default="strips")
ap.add_argument("--host-times", action="store_true",
                help="strips: print the host time of each call of the last timed step (where the host blocks)")
ap.add_argument("--halo-cache", default="",
                help="strips: directory of the halo flows per rank (.npy); computed and saved when absent, "
                     "loaded when present, so that a profiled run (rocprofv3 --pmc) holds only the rank's own "
                     "kernels")
a = ap.parse_args()

W, H = (320, 320) if a.config == 2 else (1280, 720)
fs = {2: 5, 3: 5, 4: 7, 5: 7}[a.config]
jump, maxw = (25, 50) if a.config == 5 else (5, 50)
sp = farms.synth_params(a.config)
sp.n_events = n_stream = a.events * a.n
hist = None
if a.split != "segments":
    t0 = time.time()
    hist = farms.synth_column_hist(sp)
    print(f"column histogram of {n_stream} events in {time.time() - t0:.1f} s", flush=True)
ranks = [int(r) for r in a.ranks.split(",")] if a.ranks else range(a.n)
dev = torch.device("cuda", 0)
worst = 0.0
for r in ranks:
    t0 = time.time()
    sh = multirank.make_share(sp, a.split, a.n, r, fs, maxw, hist)
    print(f"rank {r}: {sh.n} events generated in {time.time() - t0:.1f} s", flush=True)
    dx = torch.from_numpy(sh.x).to(dev)
    dy = torch.from_numpy(sh.y).to(dev)
    dt = torch.from_numpy(sh.t.view(np.int32)).to(dev)
    dp = torch.from_numpy(sh.p).to(dev)
    n = sh.n
    out = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
           for c in farms.COLUMNS[4:]}
    fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw, pool_chunk=a.pool,
                           fit_chunk=a.fit_chunk, **multirank.engine_args(sh))
    if sh.lists is not None:
        s = sh.strip
        # realistic halo flows: a handle that fits the whole stored region itself
        halo = np.flatnonzero(~sh.owned)
        hflows = torch.zeros((n, 3), dtype=torch.float64, device=dev)
        cache = os.path.join(a.halo_cache, f"halo_c{a.config}_n{a.n}_r{r}_{a.events}.npy") if a.halo_cache else ""
        if cache and os.path.exists(cache):
            hflows[torch.from_numpy(halo).to(dev)] = torch.from_numpy(np.load(cache)).to(dev)
        else:
            with farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw,
                                   region=(s.reg_lo, s.reg_hi)) as fh:
                fh.fit_device(dx, dy, dt, dp, out)
                hf = torch.empty((len(halo), 3), dtype=torch.float64, device=dev)
                fh.export_flows(torch.from_numpy(halo.astype(np.int32)).to(dev), hf)
                hflows[torch.from_numpy(halo).to(dev)] = hf
                fh.pool_device()
            if cache:
                os.makedirs(a.halo_cache, exist_ok=True)
                np.save(cache, hf.cpu().numpy())
        ex_buf = torch.empty((1, 3), dtype=torch.float64, device=dev)
        cuts = np.searchsorted(sh.gidx, [b * n_stream // a.nsub for b in range(a.nsub + 1)])
        cuts[-1] = n
        subs = []
        for b in range(a.nsub):
            lo, hi = int(cuts[b]), int(cuts[b + 1])
            hb = halo[(halo >= lo) & (halo < hi)]
            subs.append((lo, hi, torch.from_numpy((hb - lo).astype(np.int32)).to(dev),
                         hflows[torch.from_numpy(hb).to(dev)].contiguous()))
    seg = a.split == "segments" and sh.seg is not None  # (N = 1: the whole stream, one call)
    if seg:  # the surfaces of the ranks before this one: stand-ins of the right shape
        mine = torch.empty((2, W * H), dtype=torch.int64, device=dev)
        rows = max(len(segments.merge_rows(r)), 1)
        stack = torch.full((rows, W * H), -1, dtype=torch.int64, device=dev)
        sae = torch.empty(W * H, dtype=torch.int64, device=dev)
        o = sh.seg.n_warm

    log = []

    def timed(tag, fn, *args):
        t = time.perf_counter()
        fn(*args)
        log.append((tag, t, time.perf_counter()))

    def run():
        fm.reset()
        log.clear()
        if sh.lists is not None:
            # the order of multirank.Stepper.step: the exchange of b+1 (its gather
            # queued behind the fit) with the fit of b+2 issued before the wait,
            # then the scatter queued ahead of the pooling of b+1
            def fit(b):
                lo, hi, _, _ = subs[b]
                timed(f"fit{b}", fm.fit_device, dx[lo:hi], dy[lo:hi], dt[lo:hi], dp[lo:hi],
                      {c: v[lo:hi] for c, v in out.items()})

            def exchange(b, nxt):
                _, _, hi_idx, hf = subs[b]
                timed(f"export{b}", fm.export_flows_async, hi_idx[:1], ex_buf)
                if nxt < len(subs):
                    fit(nxt)
                timed(f"wait{b}", fm.export_wait)
                timed(f"import{b}", fm.import_flows_async, hi_idx, hf)
            fit(0)
            exchange(0, 1)
            for b in range(len(subs)):
                timed(f"pool{b}", fm.pool_device)
                if b + 1 < len(subs):
                    exchange(b + 1, b + 2)
            return
        if seg:
            timed("last_stamps", fm.last_stamps, dx[o:], dy[o:], dt[o:], sh.n_head, mine[0], mine[1])
            if r > 0:
                timed("merge", fm.merge_stamps, stack, sae)
                timed("seed", fm.seed_sae, sae)
        timed("process", fm.process_device, dx, dy, dt, dp, out)
    run()  # warmup
    best = 1e9
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t1)
    if a.host_times and log:
        z = log[0][1]
        print("host calls of the last step (ms from its start: begin, duration):", flush=True)
        for tag, t0c, t1c in log:
            print(f"  {tag:10s} {1e3 * (t0c - z):8.2f} {1e3 * (t1c - t0c):8.2f}", flush=True)
    fm.close()
    worst = max(worst, best)
    print(json.dumps({"n": a.n, "rank": r, "split": a.split, "config": a.config, "nsub": a.nsub,
                      "pool_chunk": a.pool, "stored": n, "owned": sh.n_owned, "ms": round(best * 1e3, 1)}),
          flush=True)
    del dx, dy, dt, dp, out
    torch.cuda.empty_cache()
print(json.dumps({"n": a.n, "split": a.split, "predicted_Mev_s": round(a.n * a.events / worst / 1e6, 1),
                  "worst_ms": round(worst * 1e3, 1)}), flush=True)
