#!/usr/bin/env python3
"""bench.py — FARMS_Flow batch hot path on MI355X.

Metric (BASELINE.json): Mevents/s (and % of the HBM roofline) at 1/2/4/8 GPUs.
Workload at N=1: BASELINE config 3 — synthetic 1280x720 DVS-shape stream, 50M
events, filtersize 5, inlierCheck 5 (the north_star's headline configuration).
A step = one full pass of the hot path (surfaces reset + every event through
local fit and multiscale pooling) over the whole resident stream.

Multi-GPU (torchrun, one process per GPU): weak scaling — the stream holds N x
the per-GPU event count on the same sensor; rank r owns the events of one
x-strip (event-count quantiles) and its handle stores the strip widened by the
pooling + fit halo, so its records are bitwise those of a one-GPU run.  No
data-path collective (strips.py); value = owned events of all
ranks / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

import farms  # noqa: E402
import strips  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
SENSOR = {1: (128, 128), 2: (320, 320), 3: (1280, 720), 4: (1280, 720), 5: (1280, 720)}
FILTER = {1: 3, 2: 5, 3: 5, 4: 7, 5: 7}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--events", type=int, default=0, help="override the stream length")
    ap.add_argument("--fit-chunk", type=int, default=0)
    ap.add_argument("--pool-chunk", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=1_500_000, help="events in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(ev, width, height, fs, jump, maxw, n_sample):
    """Oracle ("port": single-thread C restatement, -O2) on the first n_sample
    events of the same stream."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleFlow

    sample = ev.head(min(n_sample, len(ev)))
    x, y, t, p = sample.relative()
    of = OracleFlow(height, width, fs, 5, jump, maxw)
    t0 = time.perf_counter()
    of.process(x, y, t, p)
    dt = time.perf_counter() - t0
    return {"value": len(sample) / dt / 1e6, "unit": "Mevents/s", "cores": 1, "kind": "port",
            "sample": f"first {len(sample)} events of the same stream, oracle/farms_oracle.c -O2, 1 thread, {dt:.1f} s"}


def pmc_traffic(cfg, world, pool_launches):
    """HBM bytes per k_pool launch from the committed rocprofv3 PMC passes of the
    same workload (tools/gpu_traffic.sh -> profiles/rNN_traffic_c<cfg>.json,
    FETCH_SIZE doubled per the gfx950 correction).  None unless the profile saw
    exactly this launch count (i.e. the same stream and chunking)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_c{cfg}.json")))
    if world != 1 or not files:
        return None
    k = json.load(open(files[-1]))["kernels"].get("k_pool<11>" if cfg != 5 else "k_pool<3>")
    if not k or k["dispatches"] != pool_launches:
        return None
    return round(k["traffic_bytes_per_launch"])


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # FARMS_BENCH_DEVICE pins every rank to one device (rehearsal of N ranks on a
    # one-GPU box, with FARMS_DIST_BACKEND=gloo); the driver uses neither.
    device = int(os.environ.get("FARMS_BENCH_DEVICE", local_rank))
    backend = os.environ.get("FARMS_DIST_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        dist.init_process_group(backend)
    dev = torch.device("cuda", device)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    cfg = args.config
    W, H = SENSOR[cfg]
    fs = FILTER[cfg]
    jump, maxw = (25, 50) if cfg == 5 else (5, 50)
    sp = farms.synth_params(cfg)
    per_gpu = args.events or (int(sp.n_events) if cfg in (1, 2, 3) else 50_000_000)
    sp.n_events = per_gpu * world  # weak scaling: fixed events per GPU
    ev = farms.synth_generate(sp)  # same seed on every rank: the same stream
    x, y, t, p = ev.relative()
    strip = strips.plan(x, W, world, fs, maxw)[rank]
    if world > 1:
        m = strips.region_mask(x, strip)
        x, y, t, p = x[m], y[m], t[m], p[m]
    n = len(x)
    n_owned = int(strips.owned_mask(x, strip).sum())
    dx = torch.from_numpy(x).to(dev)
    dy = torch.from_numpy(y).to(dev)
    dt_ = torch.from_numpy(t.view(np.int32)).to(dev)
    dp = torch.from_numpy(p).to(dev)
    out = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
           for c in farms.COLUMNS[4:]}
    fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw, device=device,
                           fit_chunk=args.fit_chunk, pool_chunk=args.pool_chunk,
                           region=(strip.reg_lo, strip.reg_hi), owned=(strip.own_lo, strip.own_hi))
    torch.cuda.synchronize()

    def step():
        fm.reset()
        fm.process_device(dx, dy, dt_, dp, out)

    for _ in range(args.warmup):
        step()
    fm.set_profiling(farms.PROF_TIMING)  # HIP events around the k_pool launches only
    stats = []
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        stats.append(fm.stats())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], device=red_dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        nn = torch.tensor([n_owned], device=red_dev, dtype=torch.float64)
        dist.all_reduce(nn)
        total_events = float(nn.item())
    else:
        total_events = float(n_owned)

    ms_step = elapsed / args.steps * 1e3
    value = total_events * args.steps / elapsed / 1e6
    pool_ms = sum(s["ms_pool_kernel"] for s in stats) / len(stats)
    ts = stats[-1]  # timings of the last timed step
    pool_launches = ts["pool_launches"]
    # work counters (U_pool, candidates, contributors) from one more, untimed step
    fm.set_profiling(True)
    step()
    st = fm.stats()
    alg_bytes = 20.0 * st["pool_cells"]  # 20 B per pooled cell of a valid event
    achieved = alg_bytes / (pool_ms / 1e3) / 1e9 if pool_ms > 0 else 0.0
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(cfg, world, pool_launches),
                "traffic_unit": "HBM bytes per launch (PMC)",
                "algorithmic_bytes_per_launch": round(alg_bytes / max(pool_launches, 1)),
                "kernel": "k_pool", "launches_per_step": pool_launches,
                "avg_launch_us": round(pool_ms * 1e3 / max(pool_launches, 1), 2)}
    line = {
        "metric": "Mevents/s (and % HBM roofline) at 1/2/4/8 GPUs; max |dtheta| vs CPU ref",
        "value": round(value, 3), "unit": "Mevents/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"BASELINE config {cfg}: {W}x{H} synthetic moving-bars stream, "
                               f"{per_gpu} events/GPU, filtersize {fs}, inlierCheck 5, scales 0..{maxw} step {jump}",
                   "events_per_gpu": per_gpu, "width": W, "height": H, "filtersize": fs,
                   "parallelism": (f"{world} x-strips, halo {strips.halo(fs, maxw)} columns recomputed, "
                                   "no data-path collective") if world > 1 else "1 GPU"},
        "roofline": roofline,
        "detail": {"valid_frac": round(st["n_valid"] / max(st["n_events"], 1), 4),
                   "ms_prep": round(ts["ms_prep"], 3), "ms_fit_sweep": round(ts["ms_fit"], 3),
                   "ms_pool_sweep": round(ts["ms_pool"], 3), "ms_pool_kernel": round(pool_ms, 3),
                   "ms_fit_kernel": round(ts["ms_fit_kernel"], 3),
                   "dense_equiv_bytes_per_event": round(alg_bytes / max(n, 1), 1),
                   "cand_per_valid": round(st["pool_candidates"] / max(st["n_valid"], 1), 1),
                   "contrib_per_valid": round(st["pool_contributors"] / max(st["n_valid"], 1), 1)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(ev, W, H, fs, jump, maxw, args.cpu_sample)
    if world > 1:
        line["detail"]["rank0_stored_events"] = n
        line["detail"]["rank0_owned_events"] = n_owned
    fm.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
