"""bench.py's multi-rank plumbing (multirank.py) on the CPU: gloo ranks with the
oracle as the engine, through the very share planning, exchanges and merge of
the owned records that bench.py runs over RCCL with the HIP engine.

For every split (temporal segments, x-strips with the flow-halo exchange,
x-strips that recompute their halos) the merged owned records of all ranks
are bitwise those of one whole-stream oracle run, and the N > 1 parity block
(tests/parity.multi_report) sees events at every rank boundary and passes.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import farms
import multirank
import segments
from oracle import OracleFlow
from parity import bitwise_equal, gate, multi_report

COLS = farms.COLUMNS


class OracleEngine:
    """The engine interface of multirank.Stepper over the CPU oracle, on CPU
    tensors.  Exchange payload: (L, theta, valid) per flow."""

    def __init__(self, H, W, fs, inl=5, jump=5, maxw=50, region=None, owned=None, import_halo=False):
        self.args = (H, W, fs, inl, jump, maxw)
        self.W, self.H = W, H
        self.owned, self.import_halo = owned, import_halo
        self.reset()

    def reset(self):
        self.sae = None
        self.fitter = OracleFlow(*self.args)   # SAE state across the sub-batches of a step
        self.pooler = OracleFlow(*self.args)   # flow state across them
        self.pending = []                      # fits not yet pooled, oldest first

    def _oracle(self):
        if self.sae is not None:
            self.fitter.seed_sae(self.sae)
            self.sae = None
        return self.fitter

    @staticmethod
    def _np(x, y, t, p):
        return x.numpy(), y.numpy(), t.numpy().view(np.uint32), p.numpy()

    def seed_sae(self, sae):
        self.sae = sae.numpy().copy()

    def last_stamps(self, x, y, t, n_head, head, full):
        xs, ys, ts = x.numpy(), y.numpy(), t.numpy().view(np.uint32)
        if n_head > 0:
            head.copy_(torch.from_numpy(segments.last_stamps_np(xs[:n_head], ys[:n_head], ts[:n_head], self.W, self.H)))
        full.copy_(torch.from_numpy(segments.last_stamps_np(xs, ys, ts, self.W, self.H)))

    def merge_stamps(self, stack, out):
        out.copy_(torch.from_numpy(segments.merge_np(list(stack.numpy()))))

    def process_device(self, x, y, t, p, out):
        r = self._oracle().process(*self._np(x, y, t, p))  # (one call per step)
        for c in COLS[4:]:
            out[c].copy_(torch.from_numpy(r[c]))

    def fit_device(self, x, y, t, p, out):
        ev = self._np(x, y, t, p)
        fit = self._oracle().process(*ev)  # halo events' flows are replaced by imports
        xs = ev[0]
        own = (xs >= self.owned[0]) & (xs < self.owned[1]) if self.import_halo else np.ones(len(xs), bool)
        self.pending.append({"ev": ev, "out": out, "fit": fit, "L": np.where(own, fit["r_local"], 0.0),
                             "th": np.where(own, fit["theta_local"], 0.0), "valid": own & gate(fit["vx"], fit["vy"])})

    # the exchange acts on the oldest fit not yet pooled (farms_hip.h)
    def export_flows(self, idx, buf):
        f, i = self.pending[0], idx.numpy()
        buf.copy_(torch.from_numpy(np.stack([f["L"][i], f["th"][i], f["valid"][i].astype(np.float64)], axis=1)))

    def import_flows(self, idx, buf):
        f, i, b = self.pending[0], idx.numpy(), buf.numpy()
        f["L"][i], f["th"][i], f["valid"][i] = b[:, 0], b[:, 1], b[:, 2] > 0

    export_flows_async = export_flows
    import_flows_async = import_flows

    def export_wait(self):
        pass

    def pool_device(self):
        f = self.pending.pop(0)
        x, y, t, _ = f["ev"]
        r = self.pooler.pool_given(x, y, t, f["valid"], f["L"], f["th"])
        for c in ("vx", "vy", "r_local", "theta_local"):
            f["out"][c].copy_(torch.from_numpy(f["fit"][c]))
        for c in ("r_true", "theta_true", "scale"):
            f["out"][c].copy_(torch.from_numpy(r[c]))


def _free_port():
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        return sock.getsockname()[1]


def _rank_main(rank, world, port, cfg, per_rank, split, q, engine="oracle"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fs, maxw = 5, 50
    sp = farms.synth_params(cfg)
    sp.n_events = per_rank * world
    hist = multirank.column_hist(sp, dist, rank) if split != "segments" else None
    sh = multirank.make_share(sp, split, world, rank, fs, maxw, hist)
    W, H = int(sp.width), int(sp.height)
    cpu = torch.device("cpu")
    if engine == "hip":  # every rank on device 0, collectives over gloo on the CPU
        eng = farms.FlowManager(H, W, fs, 5, max_window=maxw, device=0, **multirank.engine_args(sh))
        st = multirank.Stepper(eng, sh, dist, torch.device("cuda", 0), cpu)
    else:
        eng = OracleEngine(H, W, fs, maxw=maxw, **multirank.engine_args(sh))
        st = multirank.Stepper(eng, sh, dist, cpu, cpu)
    st.step()
    merged = multirank.gather_owned(dist, st.owned_records(), sh.n_stream)
    if rank == 0:
        q.put((merged, multirank.plan_info(sh), sh.label))
    dist.destroy_process_group()


@pytest.mark.parametrize("split,world,cfg,per_rank", [("segments", 3, 2, 20_000), ("strips", 3, 2, 20_000),
                                                      ("strips", 2, 3, 25_000), ("strips-recompute", 2, 3, 25_000),
                                                      # strips storing fewer events than the 8 sub-batches of a step:
                                                      # every rank still runs 8 exchanges (empty sub-batches)
                                                      ("strips", 3, 2, 3)])
def test_gloo_ranks_with_the_oracle_engine_reproduce_the_whole_run(split, world, cfg, per_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, cfg, per_rank, split, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    merged, info, label = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert merged is not None, "owned events do not partition the stream"
    sp = farms.synth_params(cfg)
    sp.n_events = per_rank * world
    W, H = int(sp.width), int(sp.height)
    x, y, t, p = farms.synth_generate(sp).relative()
    whole = OracleFlow(H, W, 5, 5).process(x, y, t, p)
    assert bitwise_equal(merged, whole)
    bnd = multirank.boundary_events(info, x, t, 50, W, H)
    assert len(bnd) == world - 1
    rep = multi_report(merged, whole, whole, bnd)
    print(label, rep)
    assert rep["ok"], rep
    if per_rank < 100:  # the tiny stream: too few events for valid flows at every border
        return
    for b in rep["boundaries"]:
        assert b["events"] > 0 and b["valid_events"] > 0 and b["bitwise_vs_cr_oracle"]


@pytest.mark.gpu
@pytest.mark.parametrize("split,world", [("strips", 2), ("segments", 3), ("strips", 3), ("strips-recompute", 2)])
def test_gloo_ranks_with_the_hip_engine_reproduce_the_whole_run(split, world):
    """The same plumbing with the HIP engine, every rank on device 0: the merged
    owned records equal one whole-stream engine run bitwise (the x-strip step is
    the pipelined one: fit and exchange of sub-batch b+1 under the pooling of b)."""
    cfg, per_rank = 3, 120_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, cfg, per_rank, split, q, "hip"))
             for r in range(world)]
    for pr in procs:
        pr.start()
    merged, info, label = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert merged is not None
    sp = farms.synth_params(cfg)
    sp.n_events = per_rank * world
    x, y, t, p = farms.synth_generate(sp).relative()
    with farms.FlowManager(720, 1280, 5, 5) as fm:
        whole = fm.process(x, y, t, p)
    assert bitwise_equal(merged, whole)


def test_boundary_events_of_a_strip_border_reach_both_ways():
    x = np.array([0, 40, 49, 50, 99, 100, 150, 200], np.int32)
    t = np.zeros(8, np.uint32)
    (name, idx), = multirank.boundary_events({"split": "strips", "cuts": [100]}, x, t, 50, 320, 320)
    assert idx.tolist() == [3, 4, 5]  # x in [100 - 50, 100 + 50): the windows that cross column 100
    (name, idx), = multirank.boundary_events({"split": "segments", "starts": [0, 3]}, x,
                                             np.array([0, 1, 2, 3, 100, 502, 503, 900], np.uint32), 50, 320, 320)
    assert idx.tolist() == [3, 4, 5]  # rank 1's events within 500 us of its start (t = 3)
