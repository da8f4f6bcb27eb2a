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
        self.ev = None

    def _oracle(self):
        o = OracleFlow(*self.args)
        if self.sae is not None:
            o.seed_sae(self.sae)
        return o

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
        r = self._oracle().process(*self._np(x, y, t, p))
        for c in COLS[4:]:
            out[c].copy_(torch.from_numpy(r[c]))

    def fit_device(self, x, y, t, p, out):
        self.ev, self.out = self._np(x, y, t, p), out
        self.fit = self._oracle().process(*self.ev)  # halo events' flows are replaced by imports
        xs = self.ev[0]
        own = (xs >= self.owned[0]) & (xs < self.owned[1]) if self.import_halo else np.ones(len(xs), bool)
        self.L = np.where(own, self.fit["r_local"], 0.0)
        self.th = np.where(own, self.fit["theta_local"], 0.0)
        self.valid = own & gate(self.fit["vx"], self.fit["vy"])

    def export_flows(self, idx, buf):
        i = idx.numpy()
        buf.copy_(torch.from_numpy(np.stack([self.L[i], self.th[i], self.valid[i].astype(np.float64)], axis=1)))

    def import_flows(self, idx, buf):
        i, b = idx.numpy(), buf.numpy()
        self.L[i], self.th[i], self.valid[i] = b[:, 0], b[:, 1], b[:, 2] > 0

    def pool_device(self):
        x, y, t, _ = self.ev
        r = self._oracle().pool_given(x, y, t, self.valid, self.L, self.th)
        for c in ("vx", "vy", "r_local", "theta_local"):
            self.out[c].copy_(torch.from_numpy(self.fit[c]))
        for c in ("r_true", "theta_true", "scale"):
            self.out[c].copy_(torch.from_numpy(r[c]))


def _free_port():
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        return sock.getsockname()[1]


def _rank_main(rank, world, port, cfg, per_rank, split, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fs, maxw = 5, 50
    sp = farms.synth_params(cfg)
    sp.n_events = per_rank * world
    hist = multirank.column_hist(sp, dist, rank) if split != "segments" else None
    sh = multirank.make_share(sp, split, world, rank, fs, maxw, hist)
    W, H = int(sp.width), int(sp.height)
    eng = OracleEngine(H, W, fs, maxw=maxw, **multirank.engine_args(sh))
    cpu = torch.device("cpu")
    st = multirank.Stepper(eng, sh, dist, cpu, cpu)
    st.step()
    merged = multirank.gather_owned(dist, st.owned_records(), sh.n_stream)
    if rank == 0:
        q.put((merged, multirank.plan_info(sh), sh.label))
    dist.destroy_process_group()


@pytest.mark.parametrize("split,world,cfg,per_rank", [("segments", 3, 2, 20_000), ("strips", 3, 2, 20_000),
                                                      ("strips", 2, 3, 25_000), ("strips-recompute", 2, 3, 25_000)])
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
    for b in rep["boundaries"]:
        assert b["events"] > 0 and b["valid_events"] > 0 and b["bitwise_vs_cr_oracle"]


def test_boundary_events_of_a_strip_border_reach_both_ways():
    x = np.array([0, 40, 49, 50, 99, 100, 150, 200], np.int32)
    t = np.zeros(8, np.uint32)
    (name, idx), = multirank.boundary_events({"split": "strips", "cuts": [100]}, x, t, 50, 320, 320)
    assert idx.tolist() == [3, 4, 5]  # x in [100 - 50, 100 + 50): the windows that cross column 100
    (name, idx), = multirank.boundary_events({"split": "segments", "starts": [0, 3]}, x,
                                             np.array([0, 1, 2, 3, 100, 502, 503, 900], np.uint32), 50, 320, 320)
    assert idx.tolist() == [3, 4, 5]  # rank 1's events within 500 us of its start (t = 3)
