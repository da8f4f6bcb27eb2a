#!/usr/bin/env python3
"""bench.py — FARMS_Flow batch hot path on MI355X.

Metric (BASELINE.json): Mevents/s (and % of the HBM roofline) at 1/2/4/8 GPUs.
Workload at N=1: BASELINE config 3 — synthetic 1280x720 DVS-shape stream, 50M
events, filtersize 5, inlierCheck 5 (the north_star's headline configuration).
A step = one full pass of the hot path (surfaces reset + every event through
local fit and multiscale pooling) over the whole resident stream.

Multi-GPU (torchrun, one process per GPU): weak scaling — the stream holds N x
the per-GPU event count on the same sensor.  On a time-ordered stream (the
synthetic one is) rank r owns the r-th temporal segment: every step the ranks
compute their per-pixel last-stamp surfaces on the GPU, all-gather them over
RCCL, and each rank starts from the merged SAE plus a re-fitted 500 us warm-up
(segments.py).  --split strips (or an unordered stream) uses
x-strips with recomputed halos instead (strips.py).  Either way the owned
records are bitwise those of a one-GPU run; value = owned events of all ranks
/ max-over-ranks time.

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
import segments  # noqa: E402
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
    ap.add_argument("--split", choices=("segments", "strips"), default="segments",
                    help="N > 1: temporal segments (time-ordered streams) or x-strips")
    return ap.parse_args()


def cpu_baseline(sample, width, height, fs, jump, maxw):
    """Oracle ("port": single-thread C restatement, -O2) on a head sample of the
    same stream."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleFlow

    x, y, t, p = sample.relative()
    of = OracleFlow(height, width, fs, 5, jump, maxw)
    t0 = time.perf_counter()
    ref = of.process(x, y, t, p)
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu)
    except OSError:
        pass
    return ref, {"value": len(sample) / dt / 1e6, "unit": "Mevents/s", "cores": 1, "kind": "port",
                 "sample": f"first {len(sample)} events of the same stream, oracle/farms_oracle.c -O2, 1 thread, "
                           f"{dt:.1f} s",
                 "cpu_model": cpu, "host_threads": os.cpu_count()}


def parity_vs_cpu(ref, out, k):
    """The metric's "max |dtheta| vs CPU ref": the GPU records of the timed run's
    first k events against the oracle's records of the same k events (the path
    is causal, so the prefix of a full run equals a run of the prefix).  Bar as
    in tests/parity.py: validity bit-exact, r within 1e-4 relative, theta within
    1e-4 rad."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from parity import compare

    gpu = {c: ref[c] for c in farms.COLUMNS[:4]}  # x/y/t/p are inputs, not outputs of process_device
    gpu.update({c: out[c][:k].cpu().numpy() for c in farms.COLUMNS[4:]})
    rep = compare(gpu, ref)
    return {"events_compared": k, "valid_events": rep["valid_ref"], "valid_mismatch": rep["valid_mismatch"],
            "max_dtheta_true_rad": rep["theta_true_max_abs"], "max_dtheta_local_rad": rep["theta_local_max_abs"],
            "max_rel_r_true": rep["r_true_max_rel"], "max_rel_r_local": rep["r_local_max_rel"],
            "scale_mismatch": rep["scale_mismatch"], "ok": rep["ok"]}


def pmc_traffic(cfg, world, pool_launches):
    """HBM bytes per k_pool launch from the committed rocprofv3 PMC passes of the
    same workload (tools/gpu_traffic.sh -> profiles/rNN_traffic_c<cfg>.json,
    FETCH_SIZE doubled per the gfx950 correction).  None unless the profile saw
    whole steps of this launch count (i.e. the same stream and chunking)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_c{cfg}.json")))
    if world != 1 or not files:
        return None
    k = json.load(open(files[-1]))["kernels"].get("k_pool<11>" if cfg != 5 else "k_pool<3>")
    if not k or k["dispatches"] % pool_launches:  # the profiled run made whole steps of this workload
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
    cpu_sample = ev.head(min(args.cpu_sample, len(ev))) if world == 1 and not args.no_cpu_baseline else None
    del ev
    # N > 1: temporal segments on a time-ordered stream, x-strips
    # otherwise (or with --split strips)
    split = "none" if world == 1 else args.split
    if split == "segments" and not segments.is_time_ordered(t):
        split = "strips"
    region, owned, seg = None, None, None
    if split == "segments":
        segs = segments.plan(t, world)
        seg = segs[rank]
        n_head = segments.head_length(segs, rank)
        sl = slice(seg.warm, seg.end)
        x, y, t, p = x[sl], y[sl], t[sl], p[sl]
        n_owned = seg.end - seg.start
        label = (f"{world} temporal segments of the time-ordered stream: per step the ranks' last-stamp "
                 f"surfaces are all-gathered over {backend.upper()} and each rank starts from the merged SAE "
                 f"plus a re-fitted 500 us warm-up ({seg.n_warm} events on rank {rank})")
    elif split == "strips":
        strip = strips.plan(x, W, world, fs, maxw)[rank]
        m = strips.region_mask(x, strip)
        x, y, t, p = x[m], y[m], t[m], p[m]
        region, owned = (strip.reg_lo, strip.reg_hi), (strip.own_lo, strip.own_hi)
        n_owned = int(strips.owned_mask(x, strip).sum())
        label = f"{world} x-strips, halo {strips.halo(fs, maxw)} columns recomputed, no data-path collective"
    else:
        n_owned = len(x)
        label = "1 GPU"
    n = len(x)
    dx = torch.from_numpy(x).to(dev)
    dy = torch.from_numpy(y).to(dev)
    dt_ = torch.from_numpy(t.view(np.int32)).to(dev)
    dp = torch.from_numpy(p).to(dev)
    out = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
           for c in farms.COLUMNS[4:]}
    fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw, device=device,
                           fit_chunk=args.fit_chunk, pool_chunk=args.pool_chunk, region=region, owned=owned)
    if seg is not None:  # stamp surfaces: this rank's [head, full], everyone's, the merged SAE
        WHs = W * H
        mine = torch.empty((2, WHs), dtype=torch.int64, device=dev)
        gath = torch.empty((2 * world, WHs), dtype=torch.int64, device=red_dev)
        rows = torch.tensor(segments.merge_rows(rank), dtype=torch.int64, device=dev)
        sel = torch.empty((len(segments.merge_rows(rank)), WHs), dtype=torch.int64, device=dev)
        sae = torch.empty(WHs, dtype=torch.int64, device=dev)
        o = seg.n_warm  # the segment's own events start after the warm-up
    torch.cuda.synchronize()

    def step():
        fm.reset()
        if seg is not None:
            fm.last_stamps(dx[o:], dy[o:], dt_[o:], n_head, mine[0], mine[1])
            dist.all_gather_into_tensor(gath, mine if red_dev == dev else mine.cpu())
            if rank > 0:
                torch.index_select(gath.to(dev, non_blocking=False), 0, rows, out=sel)
                torch.cuda.synchronize()
                fm.merge_stamps(sel, sae)
                fm.seed_sae(sae)
        fm.process_device(dx, dy, dt_, dp, out)

    # HIP events around the k_pool launches (and phases) only; set before the
    # warmup so that the timed steps replay the launch graph the warmup captured
    fm.set_profiling(farms.PROF_POOL)
    for _ in range(args.warmup):
        step()
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
                   "parallelism": label},
        "roofline": roofline,
        "detail": {"valid_frac": round(st["n_valid"] / max(st["n_events"], 1), 4),
                   "ms_prep": round(ts["ms_prep"], 3), "ms_fit_sweep": round(ts["ms_fit"], 3),
                   "ms_pool_sweep": round(ts["ms_pool"], 3), "ms_pool_kernel": round(pool_ms, 3),
                   "ms_fit_kernel_untimed_step": round(st["ms_fit_kernel"], 3),
                   "dense_equiv_bytes_per_event": round(alg_bytes / max(n, 1), 1),
                   "cand_per_valid": round(st["pool_candidates"] / max(st["n_valid"], 1), 1),
                   "contrib_per_valid": round(st["pool_contributors"] / max(st["n_valid"], 1), 1)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ref, line["cpu_baseline"] = cpu_baseline(cpu_sample, W, H, fs, jump, maxw)
        line["parity"] = parity_vs_cpu(ref, out, len(cpu_sample))
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
