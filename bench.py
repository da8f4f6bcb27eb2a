#!/usr/bin/env python3
"""bench.py — FARMS_Flow batch hot path on MI355X.

Metric (BASELINE.json): Mevents/s (and % of the HBM roofline) at 1/2/4/8 GPUs.
Workload at N=1: BASELINE config 3 — synthetic 1280x720 DVS-shape stream, 50M
events, filtersize 5, inlierCheck 5 (the north_star's headline configuration).
A step = one full pass of the hot path (surfaces reset + every event through
local fit and multiscale pooling) over the whole stream, resident in HBM when
the timed region starts (the contract); the host-to-host rate of the C ABI
(farms_process: H2D, kernels, D2H — SURVEY §8d's timed region) is reported
beside it as `host_path`.

Multi-GPU (one process per GPU over RCCL; multirank.py): weak
scaling — the stream holds N x the per-GPU event count on the same sensor.
--split segments (default): rank r owns the r-th temporal segment, started
every step from the SAE all-gathered over RCCL plus a re-fitted 500 us
warm-up; --split strips: rank r owns an x-strip, fits its columns and
exchanges the local flows of its halo events with one grouped send/recv per
step.  Either way the owned records are bitwise those of a one-GPU run (the
line's parity block checks that across every rank boundary on a short
stream); value = owned events of all ranks / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd")
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

import farms  # noqa: E402
import multirank  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
SENSOR = {1: (128, 128), 2: (320, 320), 3: (1280, 720), 4: (1280, 720), 5: (1280, 720)}
FILTER = {1: 3, 2: 5, 3: 5, 4: 7, 5: 7}
# events per GPU, the weak-scaling unit: BASELINE.json config 4 is 200M events
# on 4 GPUs, config 5 1G events on 8 GPUs; configs 1-3 run their own streams
PER_GPU = {4: 50_000_000, 5: 125_000_000}
METRIC = "Mevents/s (and % HBM roofline) at 1/2/4/8 GPUs; max |dtheta| vs CPU ref"


def scales(cfg: int) -> tuple[int, int]:
    """(windowJump, maxWindow): config 5 pools 3 scales {0, 25, 50}."""
    return (25, 50) if cfg == 5 else (5, 50)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--events", type=int, default=0, help="override the per-GPU stream length")
    ap.add_argument("--fit-chunk", type=int, default=0)
    ap.add_argument("--pool-chunk", type=int, default=0)
    ap.add_argument("--pool-batch", type=int, default=0, help="pooling chunks per k_pool launch (0 = engine default)")
    ap.add_argument("--cpu-sample", type=int, default=1_500_000, help="events in the CPU-baseline sample")
    ap.add_argument("--parity-per-rank", type=int, default=60_000,
                    help="N > 1: events per rank of the short stream whose merged records are checked against "
                         "the oracle before the timed steps (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split", choices=multirank.SPLITS, default=None,
                    help="N > 1: temporal segments (time-ordered streams), x-strips with an RCCL exchange of "
                         "halo flows, or x-strips that recompute their halos.  Default: x-strips for configs 4 "
                         "and 5 (BASELINE's 4- / 8-tile spatial partition with a border halo), segments otherwise")
    ap.add_argument("--host-steps", type=int, default=2,
                    help="N=1: steps of the host-array path (farms_process: H2D + kernels + D2H) timed after "
                         "the device-resident ones (0 = skip)")
    ap.add_argument("--prof", choices=("timing", "pool"), default="timing",
                    help="HIP-event brackets in the profiled steps: around every fit and pooling launch (timing), "
                         "or the pooling launches only (pool)")
    ap.add_argument("--prof-steps", type=int, default=2,
                    help="steps after the timed ones with HIP-event brackets (the kernel timings of the roofline); "
                         "the timed steps run without them")
    ap.add_argument("--plan-only", action="store_true",
                    help="launch, rendezvous, per-rank stream shares and partition only; no GPU, no timing "
                         "(CPU test of the multi-rank plumbing; value is null)")
    a = ap.parse_args()
    if a.split is None:
        a.split = default_split(a.config)
    return a


def default_split(cfg: int) -> str:
    """BASELINE configs 4 and 5 state a spatial partition ("4-tile spatial
    partition with RCCL border halo", "8-tile partition"): their multi-GPU lines
    run the x-strips with the halo-flow exchange.  The other configs state one
    GPU; their N > 1 lines run temporal segments (the better-scaling split,
    DESIGN.md §6), named as such in config.workload."""
    return "strips" if cfg in (4, 5) else "segments"


def split_name(split: str, world: int) -> str:
    """The partition a line measured, as config.workload names it."""
    if world == 1:
        return "1 GPU"
    return {"strips": f"{world}-tile spatial partition (x-strips) with RCCL halo-flow exchange",
            "strips-recompute": f"{world}-tile spatial partition (x-strips), halos recomputed, no collective",
            "segments": f"{world} temporal segments (not a spatial partition), RCCL all-gather of SAE surfaces"}[split]


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return int(so.getsockname()[1])


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start the N ranks as a
    child torchrun on this node (one process per GPU), before anything touches
    the GPU, and return its exit code.  Its rank 0 prints the JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            return next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "unknown")
    except OSError:
        return "unknown"


def cpu_baseline(x, y, t, p, k, width, height, fs, jump, maxw):
    """Oracle ("port": single-thread C restatement, -O2) on the first k events
    of the same stream."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleFlow

    of = OracleFlow(height, width, fs, 5, jump, maxw)
    t0 = time.perf_counter()
    ref = of.process(x[:k], y[:k], t[:k], p[:k])
    dt = time.perf_counter() - t0
    return ref, {"value": k / dt / 1e6, "unit": "Mevents/s", "cores": 1, "kind": "port",
                 "sample": f"first {k} events of the same stream, oracle/farms_oracle.c -O2, 1 thread, {dt:.1f} s",
                 "cpu_model": cpu_model(), "host_threads": os.cpu_count()}


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


def profile_split(split: str, world: int) -> str:
    """The split whose committed PMC summaries a line's roofline reads: one GPU
    runs the whole-sensor call whatever the config's split for N > 1 (round 6:
    C4/C5 default to strips, and their N=1 lines read none of the strip
    summaries)."""
    return split if world > 1 else "none"


def committed_profile(kind: str, cfg: int, split: str, kernel: str):
    """Per-kernel PMC figures of the newest committed rocprofv3 summary of the
    same per-GPU workload: profiles/rNN_<kind>_c<cfg>.json (tools/gpu_traffic.sh /
    tools/gpu_sq.sh on `bench.py --config cfg --steps 1 --warmup 0`; a temporal
    segment runs exactly that call) or, for x-strips,
    profiles/rNN_<kind>_c<cfg>_strips.json (one rank-simulated strip step,
    tools/strip_rank.py).  Per-launch figures: a launch covers a fixed number of
    events (fit chunk / pooling super-chunk), whatever the stream length."""
    import glob

    suffix = "_strips" if split.startswith("strips") else ""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{kind}_c{cfg}{suffix}.json")))
    if not files:
        return None
    k = json.load(open(files[-1]))["kernels"].get(kernel)
    if not k:
        return None
    return dict(k, source=os.path.relpath(files[-1], ROOT))


def kernel_roofline(cfg: int, split: str, kernel: str, kname: str, launches: int, avg_us: float,
                    algo_bytes_per_launch: float | None, binds: str) -> dict:
    """Roofline of one hot kernel.

    achieved = HBM bytes per launch measured by the PMC counters (2 x
    FETCH_SIZE + WRITE_SIZE, the gfx950 correction) / the launch's average
    duration, timed live with HIP events on the stream that runs it inside the
    timed steps; frac = achieved / 8 TB/s.  Neither hot kernel is HBM-bound
    (their working sets stay in L2): `binds` names what binds, and `issue`
    gives the SQ counters of the same workload (VALU issue utilisation, wait
    fractions).  `algorithmic_*` is SURVEY §8d's per-event figure over the
    launch's events; for k_pool it counts the dense 101 x 101 window of every
    valid event (20 B per cell), which the kernel never reads, so that
    quotient is no physical rate and is never `frac`."""
    tr = committed_profile("traffic", cfg, split, kname)
    sq = committed_profile("sq", cfg, split, kname)
    traffic = round(tr["traffic_bytes_per_launch"]) if tr else None
    achieved = traffic / (avg_us * 1e-6) / 1e9 if traffic and avg_us > 0 else None
    r = {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None, "traffic": traffic,
         "traffic_unit": "HBM bytes per launch (PMC: 2*FETCH_SIZE + WRITE_SIZE)",
         "traffic_source": tr["source"] if tr else None,
         "kernel": kernel, "launches_per_step": launches, "avg_launch_us": round(avg_us, 2), "binds": binds}
    if algo_bytes_per_launch is not None:
        r["algorithmic_bytes_per_launch"] = round(algo_bytes_per_launch)
        r["algorithmic_GBps"] = round(algo_bytes_per_launch / (avg_us * 1e-6) / 1e9, 1) if avg_us > 0 else None
    if sq and avg_us > 0:
        waves = max(sq["SQ_WAVES"], 1.0)
        wave_cyc = max(sq["SQ_WAVE_CYCLES"], 1.0)
        # SIMD-cycles the launch had: 1,024 SIMDs x 2.4 GHz x duration; one wave's
        # stream of independent wave64 VALU instructions issues one per 4 cycles
        # on its SIMD (v_add_f32 / v_fma_f32, /opt/skills/guides/MI355X_MICROARCH.md
        # per-instruction table), so this is the fraction of the launch's SIMD
        # cycles its VALU instructions occupy (the PMC pass runs kernels alone;
        # the duration is the concurrent one, so it reads low)
        simd_cycles = 1024 * 2.4e9 * avg_us * 1e-6
        r["issue"] = {"valu_insts_per_wave": round(sq["SQ_INSTS_VALU"] / waves, 1),
                      "valu_issue_util": round(4.0 * sq["SQ_INSTS_VALU"] / simd_cycles, 4),
                      "wait_any_frac": round(sq["SQ_WAIT_ANY"] / wave_cyc, 4),
                      "wait_inst_frac": round(sq["SQ_WAIT_INST_ANY"] / wave_cyc, 4),
                      "active_inst_frac": round(sq["SQ_ACTIVE_INST_ANY"] / wave_cyc, 4),
                      "source": sq["source"]}
        r["issue_frac"] = r["issue"]["valu_issue_util"]
    return r


def rooflines(cfg: int, split: str, ts: dict, cs: dict, ki: dict) -> dict:
    """Both hot kernels' rooflines from the timed steps' stats `ts` (HIP-event
    launch brackets) and the counted step's `cs`, keyed "k_fit" / "k_pool";
    "dominant" names the one with more kernel time per step (the pooling at
    filtersize 5, the fit at filtersize 7).  `ki` names the kernels the engine
    ran (farms_kernel_info), as the PMC summaries key them."""
    fs = FILTER[cfg]
    jump, maxw = scales(cfg)
    nf, npl = max(ts["fit_launches"], 1), max(ts["pool_launches"], 1)
    owned = max(cs["n_owned"], 1)
    # SURVEY §8d per event: the fit reads 4 B per SAE cell of the clipped union
    # (U_loc) and the 16-B event, and writes the plane (16 B) and its flag (1 B);
    # pooling reads 20 B per dense window cell of a valid event (U_pool) and
    # writes the 52-B record
    fit_algo = (4.0 * cs["sae_cells"] + 33.0 * cs["n_events"]) / nf
    pool_algo = (20.0 * cs["pool_cells"] + 52.0 * owned) / npl
    fit_k = ki.get("fit", f"k_fit_quad<{fs // 2}>")
    pool_k = ki.get("pool", f"k_pool<{maxw // jump + 1}>")
    # a launch's duration is its share of the kernel's busy wall time (the
    # union of its launch brackets on the device timeline, farms_stats
    # ms_*_busy): with two fit streams (fs 7) two fit launches run side by
    # side and the sum of the brackets counts the overlap twice (round 4:
    # 93.7 ms of fit brackets in a 61.4 ms C4 step).  So launches x
    # avg_launch_us never exceeds the step; the bracket sum is kept beside it.
    busy = {"k_fit": ts.get("ms_fit_busy") or ts["ms_fit_kernel"],
            "k_pool": ts.get("ms_pool_busy") or ts["ms_pool_kernel"]}
    out = {
        "k_fit": kernel_roofline(cfg, split, fit_k.split("<")[0], fit_k, ts["fit_launches"],
                                 busy["k_fit"] * 1e3 / nf, fit_algo,
                                 "latency (dependent L2 loads of the SAE union window), not HBM: see issue"),
        "k_pool": kernel_roofline(cfg, split, pool_k.split("<")[0], pool_k, ts["pool_launches"],
                                  busy["k_pool"] * 1e3 / npl, pool_algo,
                                  "latency (dependent L2 loads and the fp64 fold chain), not HBM: see issue"),
    }
    for k, kern in (("k_fit", "ms_fit_kernel"), ("k_pool", "ms_pool_kernel")):
        out[k]["timing"] = "busy wall time (union of the launch brackets) / launches"
        out[k]["ms_busy_per_step"] = round(busy[k], 3)
        out[k]["ms_bracket_sum_per_step"] = round(ts[kern], 3)
    out["kernels"] = ki
    out["dominant"] = "k_fit" if busy["k_fit"] > busy["k_pool"] else "k_pool"
    return out


def host_path(fm, x, y, t, p, steps: int) -> dict:
    """The boundary as the CLI uses it (vFlow.cpp:214-416, SURVEY §8d's timed
    region): host arrays in, host records out through farms_process, a
    pipeline of sub-batches (upload of sub-batch b+1 under the kernels of b,
    downloads of finished pooling super-chunks under later ones).  Timed apart
    from `value`, which keeps inputs resident in HBM (the contract).  Two legs:
    the arrays in pinned host memory (farms_host_alloc; DMAed in place: how
    the CLI holds its loop arrays) and in pageable numpy memory (staged through
    pinned buffers by host threads, the copy-out too)."""
    n = len(x)
    fm.set_profiling(0)

    def leg(ins, rec):
        fm.reset()
        fm.process(*ins, out=rec)  # warm-up: staging, output pages
        best, tot = 1e30, 0.0
        for _ in range(steps):
            fm.reset()
            t0 = time.perf_counter()
            fm.process(*ins, out=rec)
            dt = time.perf_counter() - t0
            best, tot = min(best, dt), tot + dt
        return {"value": round(n * steps / tot / 1e6, 3), "ms_per_step": round(tot / steps * 1e3, 3),
                "ms_best": round(best * 1e3, 3)}

    owners = [farms.pinned(a) for a in (x, y, t, p)]
    r = leg([a for a, _ in owners], farms.Records(n, pinned=True))
    del owners
    r.update({"unit": "Mevents/s", "steps": steps, "pageable": leg([x, y, t, p], farms.Records(n)),
              "what": "farms_process host-to-host, pinned host arrays (DMA in place: H2D 16 B/event, D2H 68 B/event "
                      "incl. the x/y/t/p echo); `pageable`: numpy arrays staged by FARMS_HOST_THREADS host threads"})
    return r


def stream_params(cfg: int, per_gpu: int, world: int):
    sp = farms.synth_params(cfg)
    sp.n_events = per_gpu * world
    return sp


def parity_multi(args, cfg, world, rank, dist, device, xdev, fm_kw) -> dict | None:
    """N > 1: the same split and exchange as the timed steps, on a short stream
    of N x parity_per_rank events of the same configuration (a share per rank),
    run once; every rank's owned records are merged by stream index and rank 0
    checks them against the oracle over the whole short stream — the bar of
    tests/parity.py against the glibc oracle, every column bitwise against the
    oracle with the GPU's correctly rounded libm — overall and per rank
    boundary (multirank.boundary_events: each segment's first 500 us, each
    strip border's pooling reach).  Returns rank 0's block (None elsewhere)."""
    W, H = SENSOR[cfg]
    jump, maxw = scales(cfg)
    sp = stream_params(cfg, args.parity_per_rank, world)
    hist = multirank.column_hist(sp, dist, rank, xdev) if args.split != "segments" else None
    sh = multirank.make_share(sp, args.split, world, rank, FILTER[cfg], maxw, hist)
    with farms.FlowManager(H, W, FILTER[cfg], 5, window_jump=jump, max_window=maxw, device=device.index,
                           **fm_kw, **multirank.engine_args(sh)) as fm:
        st = multirank.Stepper(fm, sh, dist, device, xdev)
        dist.barrier()
        st.step()
        rec = st.owned_records()
    merged = multirank.gather_owned(dist, rec, sh.n_stream)
    if rank != 0:
        return None
    if merged is None:
        return {"ok": False, "what": "the ranks' owned events do not partition the stream"}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import OracleFlow
    from parity import multi_report

    ev = farms.synth_generate(sp)
    x, y, t, p = ev.relative()
    refs = {}

    def run(libm):  # the two oracles in parallel threads (ctypes releases the GIL)
        refs[libm] = OracleFlow(H, W, FILTER[cfg], 5, jump, maxw, libm=libm).process(x, y, t, p)

    th = [threading.Thread(target=run, args=(m,)) for m in ("glibc", "cr")]
    for a in th:
        a.start()
    for a in th:
        a.join()
    bnd = multirank.boundary_events(multirank.plan_info(sh), x, t, maxw, W, H)
    rep = multi_report(merged, refs["glibc"], refs["cr"], bnd, maxw)
    rep["what"] = (f"{world} ranks, split {args.split}, on a {sh.n_stream}-event stream of config {cfg}: every "
                   f"rank's owned records vs the oracle over the whole stream (glibc: the tolerance bar; the "
                   f"correctly rounded libm: bitwise), and per rank boundary")
    return rep


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    import torch

    # FARMS_BENCH_DEVICE pins every rank to one device (rehearsal of N ranks on a
    # one-GPU box, with FARMS_DIST_BACKEND=gloo); the driver uses neither.
    dev_idx = int(os.environ.get("FARMS_BENCH_DEVICE", local_rank))
    backend = os.environ.get("FARMS_DIST_BACKEND", "gloo" if args.plan_only else "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist

        if not args.plan_only:
            torch.cuda.set_device(dev_idx)
        dist.init_process_group(backend)
    device = torch.device("cuda", dev_idx)
    xdev = device if backend == "nccl" else torch.device("cpu")  # where collectives run

    cfg = args.config
    W, H = SENSOR[cfg]
    fs = FILTER[cfg]
    jump, maxw = scales(cfg)
    sp0 = farms.synth_params(cfg)
    per_gpu = args.events or PER_GPU.get(cfg, int(sp0.n_events))
    sp = stream_params(cfg, per_gpu, world)
    hist = multirank.column_hist(sp, dist, rank, xdev if not args.plan_only else None) \
        if world > 1 and args.split != "segments" else None
    sh = multirank.make_share(sp, args.split, world, rank, fs, maxw, hist)
    n, n_owned = sh.n, sh.n_owned
    if args.plan_only:
        total = n_owned
        if dist:
            tt = torch.tensor([n_owned], dtype=torch.int64)
            dist.all_reduce(tt)
            total = int(tt.item())
        line = {"metric": METRIC, "value": None, "unit": "Mevents/s", "n_gpus": world, "plan_only": True,
                "config": {"workload": f"BASELINE config {cfg}; {split_name(args.split, world)}",
                           "split": args.split, "events_per_gpu": per_gpu, "parallelism": sh.label},
                "detail": {"owned_events_all_ranks": total, "stream_events": sh.n_stream,
                           "rank0_stored_events": n, "rank0_owned_events": n_owned}}
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    fm_kw = {"fit_chunk": args.fit_chunk, "pool_chunk": args.pool_chunk, "pool_batch": args.pool_batch}
    parity = None
    if world > 1 and args.parity_per_rank > 0:
        parity = parity_multi(args, cfg, world, rank, dist, device, xdev, fm_kw)
    fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=maxw, device=dev_idx, **fm_kw,
                           **multirank.engine_args(sh))
    st = multirank.Stepper(fm, sh, dist, device, xdev)
    torch.cuda.synchronize()

    # the timed steps run uninstrumented (HIP-event brackets around every fit
    # launch cost 4-6 ms per step); the kernel timings come from prof_steps
    # more steps with HIP events around the phases and every fit and pooling
    # launch, on the streams that run them (farms_stats sums them over a
    # step's calls)
    fm.set_profiling(0)
    if dist:
        dist.barrier()  # communicators up on every rank before the first exchange
    for _ in range(args.warmup):
        st.step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st.step()
    torch.cuda.synchronize()
    elapsed_rank = time.perf_counter() - t0  # this rank's own steps, before waiting for the others
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fm.set_profiling(farms.PROF_TIMING if args.prof == "timing" else farms.PROF_POOL)
    stats = []
    for _ in range(max(args.prof_steps, 1)):
        st.step()
        stats.append(fm.stats())
    if dist:
        dist.barrier()
    if dist:
        tt = torch.tensor([elapsed], device=xdev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        nn = torch.tensor([n_owned], device=xdev, dtype=torch.float64)
        dist.all_reduce(nn)
        total_events = float(nn.item())
    else:
        total_events = float(n_owned)

    ms_step = elapsed / args.steps * 1e3
    value = total_events * args.steps / elapsed / 1e6
    mean = {k: sum(s_[k] for s_ in stats) / len(stats)
            for k in ("ms_fit_kernel", "ms_pool_kernel", "ms_fit_busy", "ms_pool_busy")}
    ts = dict(stats[-1], **mean)  # launch counts of a step, kernel times averaged over the profiled steps
    # work counters (U_loc, U_pool, candidates, contributors) from one more, untimed step
    fm.set_profiling(True)
    st.step()
    cs = fm.stats()
    rl = rooflines(cfg, profile_split(args.split, world), ts, cs, fm.kernel_info())
    dom = rl["dominant"]
    mine = {"rank": rank, "ms_step_rank": round(elapsed_rank / args.steps * 1e3, 3),
            "stored_events": n, "owned_events": n_owned,
            "valid_frac": round(cs["n_valid"] / max(cs["n_owned"], 1), 4),
            "dominant": dom, "avg_launch_us": {k: rl[k]["avg_launch_us"] for k in ("k_fit", "k_pool")},
            "frac": {k: rl[k]["frac"] for k in ("k_fit", "k_pool")},
            "ms_fit_kernel": round(ts["ms_fit_kernel"], 3), "ms_pool_kernel": round(ts["ms_pool_kernel"], 3)}
    per_rank = [mine]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    # the line's roofline: rank 0's dominant kernel, with every rank's figures
    # (per_rank) and the slowest rank named
    roofline = dict(rl[dom])
    # the launches of the named kernel fit inside the step (busy-time accounting)
    roofline["launches_x_avg_ms"] = round(roofline["launches_per_step"] * roofline["avg_launch_us"] / 1e3, 3)
    roofline["fits_in_step"] = roofline["launches_x_avg_ms"] <= ms_step
    if world > 1:
        roofline["rank"] = rank
        roofline["critical_rank"] = max(per_rank, key=lambda r: r["ms_step_rank"])["rank"]
        roofline["per_rank"] = per_rank
    roofline["other"] = {k: {f: rl[k].get(f) for f in ("kernel", "frac", "achieved", "avg_launch_us",
                                                        "launches_per_step", "traffic_source")}
                         for k in ("k_fit", "k_pool") if k != dom}
    roofline["engine_kernels"] = rl["kernels"]
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mevents/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"BASELINE config {cfg}: {W}x{H} synthetic moving-bars stream, "
                               f"{per_gpu} events/GPU, filtersize {fs}, inlierCheck 5, scales 0..{maxw} step {jump}; "
                               f"{split_name(args.split, world)}",
                   "split": args.split if world > 1 else "none",
                   "events_per_gpu": per_gpu, "width": W, "height": H, "filtersize": fs,
                   "parallelism": sh.label},
        "roofline": roofline,
        "detail": {"valid_frac": round(cs["n_valid"] / max(cs["n_owned"], 1), 4),
                   "ms_prep": round(ts["ms_prep"], 3), "ms_fit_sweep": round(ts["ms_fit"], 3),
                   "ms_pool_sweep": round(ts["ms_pool"], 3), "ms_fit_kernel": round(ts["ms_fit_kernel"], 3),
                   "ms_pool_kernel": round(ts["ms_pool_kernel"], 3),
                   "fit_launches": ts["fit_launches"], "pool_launches": ts["pool_launches"],
                   "profiling": f"{args.prof}, {max(args.prof_steps, 1)} steps after the timed ones",
                   "dense_equiv_bytes_per_event": round(20.0 * cs["pool_cells"] / max(n_owned, 1), 1),
                   "cand_per_valid": round(cs["pool_candidates"] / max(cs["n_valid"], 1), 1),
                   "contrib_per_valid": round(cs["pool_contributors"] / max(cs["n_valid"], 1), 1),
                   "cand_max": cs.get("pool_scan_max", 0),
                   "cand_over_1k_frac": round(cs.get("pool_scan_over_1k", 0) / max(cs["n_valid"], 1), 6)},
    }
    if world == 1 and args.host_steps > 0:
        line["host_path"] = host_path(fm, sh.x, sh.y, sh.t, sh.p, args.host_steps)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        k = min(args.cpu_sample, n)
        ref, line["cpu_baseline"] = cpu_baseline(sh.x, sh.y, sh.t, sh.p, k, W, H, fs, jump, maxw)
        line["parity"] = parity_vs_cpu(ref, st.out, k)
    if parity is not None:
        line["parity"] = parity
    if world > 1:
        line["detail"]["rank0_stored_events"] = n
        line["detail"]["rank0_owned_events"] = n_owned
        if sh.lists is not None:
            line["detail"]["rank0_halo_flows_received"] = st.n_halo_flows
    fm.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
