"""One rank of a multi-GPU run: its share of the stream and one step of the
hot path on it.

bench.py runs this with the HIP engine (farms.FlowManager) over RCCL; the CPU
tests run the same code with the oracle as the engine over gloo, so the share
planning, the exchanges and the merge of the owned records are one code path.

A rank owns a set of stream events and reports exactly those records; the
owned records of all ranks partition the stream and are bitwise those of one
whole-stream run.  Splits:

  * "segments" (time-ordered streams, segments.py): rank r owns the r-th run of
    the stream, processed from the SAE as of its start (the in-order merge of
    every earlier segment's last-stamp surface: one all-gather per step) plus a
    re-fitted 500 us warm-up;
  * "strips" (x-strips with a flow-halo exchange, strips.py): rank r owns a
    column range, stores it widened by the pooling halo, fits its owned
    events and receives the local flows of its halo events from their owners
    (one grouped send/recv per step);
  * "strips-recompute": x-strips that re-fit their halos (no collective).

The engine interface (duck-typed; farms.FlowManager has it): reset,
process_device, fit_device, export_flows, import_flows, pool_device,
last_stamps, merge_stamps, seed_sae.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

import farms
import segments
import strips

SPLITS = ("segments", "strips", "strips-recompute")


@dataclass
class Share:
    split: str                      # "none" or one of SPLITS
    world: int
    rank: int
    n_stream: int                   # events of the whole stream
    x: np.ndarray                   # stored events (relative stamps, clamped polarity)
    y: np.ndarray
    t: np.ndarray
    p: np.ndarray
    gidx: np.ndarray                # stream index of every stored event
    owned: np.ndarray               # bool: stored events this rank reports
    width: int = 0
    height: int = 0
    seg: segments.Segment | None = None
    n_head: int = 0
    plan: list = field(default_factory=list)   # strips: every rank's Strip
    lists: dict | None = None       # strips: exchange lists per peer
    label: str = ""

    @property
    def n(self) -> int:
        return int(self.x.shape[0])

    @property
    def n_owned(self) -> int:
        return int(self.owned.sum())

    @property
    def strip(self):
        return self.plan[self.rank] if self.plan else None


def column_hist(sp, dist=None, rank: int = 0, device=None) -> np.ndarray:
    """Events per column of the whole stream: computed on rank 0 and broadcast
    (each rank would otherwise re-plan the whole stream for it)."""
    if dist is None:
        return farms.synth_column_hist(sp)
    import torch

    dev = device if device is not None else torch.device("cpu")
    h = torch.zeros(int(sp.width), dtype=torch.int64, device=dev)
    if rank == 0:
        h.copy_(torch.from_numpy(farms.synth_column_hist(sp)))
    dist.broadcast(h, 0)
    return h.cpu().numpy()


def make_share(sp, split: str, world: int, rank: int, fs: int, max_window: int, hist=None) -> Share:
    """This rank's events of the synthetic stream `sp` (sp.n_events = the whole
    stream), generated without materialising the rest (farms.synth_select):
    stamps relative to the stream's first one, clamped polarity."""
    W, H = int(sp.width), int(sp.height)
    n = int(sp.n_events)
    if world == 1:
        ev = farms.synth_generate(sp)
        x, y, t, p = ev.relative()
        return Share("none", 1, 0, n, x, y, t, p, np.arange(n, dtype=np.int64), np.ones(n, bool), W, H, label="1 GPU")
    if split == "segments":
        lo, hi = segments.rank_window(n, world, rank)
        ev, _, t_first = farms.synth_select(sp, lo, hi)
        x, y, t, p = ev.relative(t_first)
        seg, n_head = segments.plan_rank(t, lo, n, world, rank)  # raises on an unordered stream
        sl = slice(seg.warm - lo, seg.end - lo)
        owned = np.zeros(seg.end - seg.warm, bool)
        owned[seg.n_warm:] = True
        return Share("segments", world, rank, n, x[sl], y[sl], t[sl], p[sl],
                     np.arange(seg.warm, seg.end, dtype=np.int64), owned, W, H, seg=seg, n_head=n_head,
                     label=(f"{world} temporal segments of the time-ordered stream: per step the ranks' last-stamp "
                            f"surfaces are all-gathered and each rank starts from the merged SAE plus a re-fitted "
                            f"500 us warm-up ({seg.n_warm} events on rank {rank})"))
    if split not in ("strips", "strips-recompute"):
        raise ValueError(f"unknown split {split}")
    exch = split == "strips"
    if hist is None:
        hist = farms.synth_column_hist(sp)
    plan = strips.plan_hist(hist, H, world, fs, max_window, exchange=exch)
    s = plan[rank]
    ev, gidx, t_first = farms.synth_select(sp, 0, n, s.reg_lo, s.reg_hi, count=int(hist[s.reg_lo:s.reg_hi].sum()))
    x, y, t, p = ev.relative(t_first)
    sh = Share(split, world, rank, n, x, y, t, p, gidx, strips.owned_mask(x, s), W, H, plan=plan)
    hl, hr = strips.halo(fs, max_window, W, H, exchange=exch)
    if exch:
        sh.lists = strips.exchange_lists(x, plan, rank)
        sh.label = (f"{world} x-strips: each rank fits its owned columns and sends the local flows of its events in "
                    f"other ranks' halos ({hl} / {hr} columns) with one grouped send/recv per sub-batch, the fit and "
                    f"exchange of sub-batch b+1 under the pooling of b")
    else:
        sh.label = f"{world} x-strips, halos of {hl} / {hr} columns recomputed, no data-path collective"
    return sh


def engine_args(sh: Share) -> dict:
    """FlowManager keyword arguments for this share (stored / owned columns)."""
    s = sh.strip
    if s is None:
        return {}
    return {"region": (s.reg_lo, s.reg_hi), "owned": (s.own_lo, s.own_hi), "import_halo": sh.split == "strips"}


class Stepper:
    """One step of the hot path on a rank: the per-event loop over the share,
    with the split's exchange.  Tensors live on `device` (the GPU for the HIP
    engine, the CPU for the oracle); `xdev` is where collectives run (the GPU
    under RCCL, the CPU under gloo).

    x-strips with the flow exchange run the step as a pipeline of `nsub`
    sub-batches cut at the same stream indices on every rank (so the per-
    sub-batch exchange lists pair up): the fit of sub-batch b+1 and its
    exchange run while the pooling of b does, and the fit of b+2 is issued
    before that exchange is waited for (farms_fit_device / farms_pool_device
    pipeline, the asynchronous exchange calls); consecutive sub-batches are
    bitwise one call."""

    def __init__(self, eng, sh: Share, dist, device, xdev, nsub: int = 8):
        import torch

        self.eng, self.sh, self.dist = eng, sh, dist
        self.dev, self.xdev = device, xdev
        self.dx = torch.from_numpy(sh.x).to(device)
        self.dy = torch.from_numpy(sh.y).to(device)
        self.dt = torch.from_numpy(sh.t.view(np.int32)).to(device)
        self.dp = torch.from_numpy(sh.p).to(device)
        n = sh.n
        self.out = {c: torch.zeros(n, dtype=torch.int32 if c == "scale" else torch.float64, device=device)
                    for c in farms.COLUMNS[4:]}
        if sh.lists is not None:  # flow-halo exchange buffers, per peer
            L = sh.lists
            self.send_idx = {q: torch.from_numpy(a).to(device) for q, (a, _) in L.items()}
            self.recv_idx = {q: torch.from_numpy(b).to(device) for q, (_, b) in L.items()}
            self.send_buf = {q: torch.empty((len(a), 3), dtype=torch.float64, device=device) for q, (a, _) in L.items()}
            self.recv_buf = {q: torch.empty((len(b), 3), dtype=torch.float64, device=device) for q, (_, b) in L.items()}
            same = xdev == device
            self.send_x = self.send_buf if same else {q: v.to(xdev) for q, v in self.send_buf.items()}
            self.recv_x = self.recv_buf if same else {q: v.to(xdev) for q, v in self.recv_buf.items()}
            # sub-batches [lo, hi) of the stored events, cut at stream indices
            # G_b = b * n_stream / nsub; per sub-batch and peer the slices of
            # the exchange lists and buffers, indices local to the sub-batch.
            # nsub depends on nothing rank-local: every rank runs the same
            # number of exchanges (a rank with fewer stored events than nsub
            # gets empty sub-batches, which the engines accept), so the grouped
            # send/recv pairs up on every rank.
            nsub = max(1, int(nsub))
            cuts = np.searchsorted(sh.gidx, [b * sh.n_stream // nsub for b in range(nsub + 1)])
            cuts[-1] = sh.n
            self.sub = []
            for b in range(nsub):
                lo, hi = int(cuts[b]), int(cuts[b + 1])
                parts = {}
                for q, (a, r) in L.items():
                    s0, s1 = np.searchsorted(a, [lo, hi])
                    r0, r1 = np.searchsorted(r, [lo, hi])
                    parts[q] = (torch.from_numpy(a[s0:s1] - lo).to(device), torch.from_numpy(r[r0:r1] - lo).to(device),
                                slice(int(s0), int(s1)), slice(int(r0), int(r1)))
                self.sub.append((lo, hi, parts))
        if sh.seg is not None:  # stamp surfaces: this rank's [head, full], everyone's, the merged SAE
            WH = sh.width * sh.height
            self.mine = torch.empty((2, WH), dtype=torch.int64, device=device)
            self.gath = torch.empty((2 * sh.world, WH), dtype=torch.int64, device=xdev)
            rows = segments.merge_rows(sh.rank)
            self.rows = torch.tensor(rows, dtype=torch.int64, device=device)
            self.sel = torch.empty((len(rows), WH), dtype=torch.int64, device=device)
            self.sae = torch.empty(WH, dtype=torch.int64, device=device)

    @property
    def n_halo_flows(self) -> int:
        return sum(len(b) for _, b in self.sh.lists.values()) if self.sh.lists else 0

    def _sync(self):
        import torch

        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def _sync_current(self):
        """Wait for the work issued on torch's current stream of the device (the
        collectives and copies), not for the engine's streams."""
        import torch

        if self.dev.type == "cuda":
            torch.cuda.current_stream(self.dev).synchronize()

    def step(self) -> None:
        import torch

        eng, sh, d = self.eng, self.sh, self.dist
        eng.reset()
        if sh.lists is not None:
            def fit(b):
                lo, hi, _ = self.sub[b]
                eng.fit_device(self.dx[lo:hi], self.dy[lo:hi], self.dt[lo:hi], self.dp[lo:hi],
                               {c: v[lo:hi] for c, v in self.out.items()})

            def exchange(b, fit_next=None):
                # the gathers of sub-batch b queued behind its fit; the fit of
                # b + 1 (fit_next) issued before they are waited for, so that
                # stream F is never idle across the exchange; the scatters queued
                # ahead of b's pooling (each sub-batch its own buffer slices)
                _, _, parts = self.sub[b]
                sx, rx = {}, {}
                for q, (si, ri, ss, rs) in parts.items():
                    eng.export_flows_async(si, self.send_buf[q][ss])
                if fit_next is not None:
                    fit_next()
                eng.export_wait()
                for q, (si, ri, ss, rs) in parts.items():
                    if self.send_x[q] is not self.send_buf[q]:
                        self.send_x[q][ss].copy_(self.send_buf[q][ss])
                    sx[q], rx[q] = self.send_x[q][ss], self.recv_x[q][rs]
                strips.exchange(d, sh.lists, sx, rx)
                for q, (si, ri, ss, rs) in parts.items():
                    if self.recv_x[q] is not self.recv_buf[q]:
                        self.recv_buf[q][rs].copy_(self.recv_x[q][rs])
                self._sync_current()  # the received flows in place (the current stream only)
                for q, (si, ri, ss, rs) in parts.items():
                    eng.import_flows_async(ri, self.recv_buf[q][rs])

            # fit(b + 1) under the pooling of b; fit(b + 2) issued inside the
            # exchange of b + 1 (at most two fits pending: farms_hip.h)
            nsub = len(self.sub)
            fit(0)
            exchange(0, (lambda: fit(1)) if nsub > 1 else None)
            for b in range(nsub):
                eng.pool_device()
                if b + 1 < nsub:
                    exchange(b + 1, (lambda b2=b + 2: fit(b2)) if b + 2 < nsub else None)
            return
        if sh.seg is not None:
            o = sh.seg.n_warm  # the segment's own events start after the warm-up
            eng.last_stamps(self.dx[o:], self.dy[o:], self.dt[o:], sh.n_head, self.mine[0], self.mine[1])
            d.all_gather_into_tensor(self.gath, self.mine if self.xdev == self.dev else self.mine.to(self.xdev))
            if sh.rank > 0:
                torch.index_select(self.gath.to(self.dev), 0, self.rows, out=self.sel)
                self._sync()
                eng.merge_stamps(self.sel, self.sae)
                eng.seed_sae(self.sae)
        eng.process_device(self.dx, self.dy, self.dt, self.dp, self.out)

    def owned_records(self) -> dict:
        """This rank's owned records (host arrays) with their stream indices."""
        sh = self.sh
        m = sh.owned
        rec = {"gidx": sh.gidx[m], "x": sh.x[m], "y": sh.y[m], "t": sh.t[m].view(np.int32), "p": sh.p[m]}
        rec.update({c: self.out[c].cpu().numpy()[m] for c in farms.COLUMNS[4:]})
        return rec


def gather_owned(dist, rec: dict, n_stream: int):
    """Every rank's owned records merged by stream index, on every rank (None
    if some stream event is owned by no rank or by two)."""
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, rec)
    merged = {c: np.zeros(n_stream, dtype=np.int32 if c in farms.INT_COLUMNS else np.float64) for c in farms.COLUMNS}
    seen = np.zeros(n_stream, np.int32)
    for part in parts:
        g = part["gidx"]
        seen[g] += 1
        for c in farms.COLUMNS:
            merged[c][g] = part[c]
    return merged if bool((seen == 1).all()) else None


def boundary_events(plan_info: dict, x: np.ndarray, t: np.ndarray, max_window: int, width: int,
                    height: int) -> list[tuple[str, np.ndarray]]:
    """Per rank boundary of a split, the stream events whose records depend on
    what crosses it (for the N > 1 parity block):
      * segments, boundary r-1 | r: rank r's events of the first 500 us of its
        segment -- their fits read the merged SAE, their pooling the warm-up's
        flows (vFlow.cpp:961, 1002);
      * strips, boundary at column c: owned events whose pooling window crosses
        it, x in [c - M - a, c + M) (a: the W-1 clip's alias columns,
        vFlow.cpp:1000/1113) -- they read the neighbour's flows.
    plan_info: {"split": ..., "starts": [segment starts]} or {"split": ...,
    "cuts": [strip borders]}."""
    out = []
    if plan_info["split"] == "segments":
        tt = t.astype(np.int64)
        for r, s in enumerate(plan_info["starts"][1:], start=1):
            e = np.arange(s, len(tt))
            out.append((f"segment {r - 1}|{r} at event {s}", e[tt[s:] < tt[s] + segments.KILL_US]))
    elif plan_info["split"] in ("strips", "strips-recompute"):
        hl, hr = strips.pool_halo(max_window, width, height)
        for c in plan_info["cuts"]:
            out.append((f"strip border at column {c}", np.flatnonzero((x >= c - hr) & (x < c + hl))))
    return out


def plan_info(sh: Share) -> dict:
    if sh.split == "segments":
        return {"split": "segments", "starts": segments.cuts(sh.n_stream, sh.world)[:-1]}
    if sh.plan:
        return {"split": sh.split, "cuts": [s.own_hi for s in sh.plan[:-1]]}
    return {"split": sh.split}
