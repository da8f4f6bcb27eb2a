"""Past-the-count reads, made deterministic (FARMS_POISON=1).

A kernel that reads a workspace word its call has not written finds zeros in a
fresh allocation and an earlier call's data in recycled memory, so such a bug
shows only when memory happens to be reused (round 5: k_pool2's idle half read
the descriptor past its chunk's count and faulted only after another call or
handle had used the memory; fixed in 10d81af).  FARMS_POISON=1 fills, before
every call, the per-event workspace the call must write before reading it
(descriptors, links, planes, flows, accepted flags, the overflow list) and,
before each super-chunk's candidate build, the ring buffers it fills, with
0x7F bytes: event ids and slot indices near 2^31.  A read of any such word
then goes far out of range (the pre-10d81af engine's idle half takes event
0x7F7F7F7F and loads its flow ~68 GB past the array) instead of passing on
zeros.  Under it the pairs, one-event-per-wave pooling, the host path's
sub-batches, the two-phase strip steps and the sparse short-sensor band
split must give bitwise the records of the unpoisoned runs (and of the
oracle where one is checked).
"""
import numpy as np
import pytest
import torch

import farms
from parity import bitwise_equal, compare
from test_gpu_parity import test_short_wide_sensor_sparse_band_split_vs_oracle as sparse_band_case
from test_strips import engine_strips

pytestmark = pytest.mark.gpu


def _calls(x, y, t, p, splits, **kw):
    with farms.FlowManager(720, 1280, kw.pop("fs", 5), 5, **kw) as fm:
        parts = [fm.process(x[a:b], y[a:b], t[a:b], p[a:b]) for a, b in splits]
    return {c: np.concatenate([getattr(q, c) for q in parts]) for c in farms.COLUMNS}


@pytest.mark.parametrize("pairs,fs", [("1", 5), ("0", 5), ("1", 7)])
def test_poisoned_split_calls_are_bitwise(pairs, fs, monkeypatch):
    """Several calls on one handle with odd pooled counts per chunk (an idle
    last half in many pairs), small pooling chunks: poisoned == clean."""
    ev = farms.synth_config(4 if fs == 7 else 3, 150_001)
    x, y, t, p = ev.relative()
    splits = [(0, 1), (1, 50_001), (50_001, 50_004), (50_004, 150_001)]
    monkeypatch.setenv("FARMS_POOL_PAIRS", pairs)
    clean = _calls(x, y, t, p, splits, fs=fs, pool_chunk=2048, pool_batch=4)
    monkeypatch.setenv("FARMS_POISON", "1")
    dirty = _calls(x, y, t, p, splits, fs=fs, pool_chunk=2048, pool_batch=4)
    assert bitwise_equal(clean, dirty), compare(clean, dirty)
    assert int((clean["r_true"] != 0).sum()) > 10_000


def test_poisoned_host_path_is_bitwise(monkeypatch):
    """farms_process in pipelined sub-batches on two workspace sets (pinned
    inputs and records): poisoned == clean."""
    ev = farms.synth_config(3, 2_000_000)
    x, y, t, p = ev.relative()
    keep = []
    ins = [x, y, t, p]
    for i in range(4):
        ins[i], own = farms.pinned(ins[i])
        keep.append(own)
    outs = []
    for poison in ("0", "1"):
        monkeypatch.setenv("FARMS_POISON", poison)
        with farms.FlowManager(720, 1280, 5, 5, pool_chunk=1024, pool_batch=8) as fm:
            outs.append(fm.process(*ins, out=farms.Records(len(x), pinned=True)))
    assert bitwise_equal(outs[0], outs[1]), compare(outs[0], outs[1])


@pytest.mark.parametrize("n_strips,fs", [(3, 5), (4, 7)])
def test_poisoned_strip_steps_are_bitwise(n_strips, fs, monkeypatch):
    """x-strip handles (the fit, the halo exchange, the pooling as separate
    calls; several handles in one process, as in the round-5 fault) under
    poison: bitwise the whole-sensor run."""
    ev = farms.synth_config(3, 200_000)
    x, y, t, p = ev.relative()
    with farms.FlowManager(720, 1280, fs, 5) as fm:
        whole = fm.process(x, y, t, p)
    monkeypatch.setenv("FARMS_POISON", "1")
    got = engine_strips(x, y, t, p, 1280, 720, fs, n_strips, True)
    assert bitwise_equal(got, whole), compare(whole, got)


@pytest.mark.parametrize("pairs", ["1", "0"])
def test_poisoned_sparse_band_split_vs_oracle(pairs, monkeypatch):
    """The short wide sensor's band split (rows crossing a column band two
    x-rows past their start) with the ring poisoned: a row read past its band's
    candidates would pool 0x7F records."""
    monkeypatch.setenv("FARMS_POISON", "1")
    sparse_band_case(pairs, monkeypatch)


def test_poisoned_two_phase_pipeline_is_bitwise(monkeypatch):
    """The x-strip stepper's order on one handle (the fit of b+1 issued before
    the pooling of b, three workspace sets in rotation) under poison."""
    ev = farms.synth_config(3, 200_000)
    x, y, t, p = ev.relative()
    with farms.FlowManager(720, 1280, 5, 5) as fm:
        ref = fm.process(x, y, t, p)
    monkeypatch.setenv("FARMS_POISON", "1")
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x, y, t.view(np.int32), p)]
    n = len(x)
    o = {c: torch.zeros(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    splits = [(0, 60_001), (60_001, 60_002), (60_002, 130_000), (130_000, n)]
    with farms.FlowManager(720, 1280, 5, 5, fit_chunk=8192) as fm:
        pending = 0
        for a, b in splits:
            fm.fit_device(*[v[a:b] for v in d], {c: v[a:b] for c, v in o.items()})
            pending += 1
            if pending == 2:
                fm.pool_device()
                pending -= 1
        for _ in range(pending):
            fm.pool_device()
        torch.cuda.synchronize()
    g = {c: v for c, v in zip(farms.COLUMNS[:4], (x, y, t.astype(np.int32), p))}
    g.update({c: o[c].cpu().numpy() for c in farms.COLUMNS[4:]})
    assert bitwise_equal(ref, g), compare(ref, g)
