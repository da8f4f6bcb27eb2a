"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Oracle status: "parity unpinned" (no reference fixtures exist; the reference
cannot be built here — see DESIGN.md §4).  Every stream is checked three ways:
  * against the oracle with glibc's libm (the reference): the bar of
    tests/parity.py (indices / polarity / validity bit-exact, r and theta
    within 1e-4); the libm residual is counted;
  * against the oracle with the HIP path's correctly rounded atan2 / sin / cos
    (farms_oracle_set_libm): every column bit for bit — the fit, the gate and
    the pooling arithmetic of the GPU are the reference's;
  * pooling_check: the reference pooling over the GPU's own local flows gives
    the identical scale column.
"""
import numpy as np
import torch  # noqa: F401  (its HIP runtime loads before libfarms_hip.so: farms.load_hip_library)
import pytest

import farms
from oracle import OracleFlow
from parity import bitwise_equal, compare, pooling_check

pytestmark = pytest.mark.gpu

SENSOR = {1: (128, 128), 2: (320, 320), 3: (1280, 720)}


def oracles(x, y, t, p, height, width, fs, inl=5, jump=5, maxw=50):
    """Records of the reference restatement (glibc libm) and of the same
    restatement with the HIP path's correctly rounded libm."""
    import threading

    refs = {}

    def run(libm):  # in parallel threads (ctypes releases the GIL)
        refs[libm] = OracleFlow(height, width, fs, inl, jump, maxw, libm=libm).process(x, y, t, p)

    th = [threading.Thread(target=run, args=(m,)) for m in ("glibc", "cr")]
    for a in th:
        a.start()
    for a in th:
        a.join()
    return refs["glibc"], refs["cr"]


def run_pair(ev, width, height, fs, inl=5, jump=5, maxw=50, **kw):
    x, y, t, p = ev.relative()
    with farms.FlowManager(height, width, fs, inl, window_jump=jump, max_window=maxw, **kw) as fm:
        g = fm.process(x, y, t, p)
    return (g,) + oracles(x, y, t, p, height, width, fs, inl, jump, maxw)


def assert_parity(g, r, height, width, jump=5, maxw=50, rc=None):
    """The bar of tests/parity.py against the reference restatement, the scale
    column pinned exactly by pooling_check, and (rc) every column bitwise equal
    to the restatement run with the GPU's correctly rounded libm."""
    rep = compare(g, r)
    pc = pooling_check(g, height, width, jump, maxw)
    print(rep, pc)
    assert rep["ok"], rep
    assert pc["ok"], pc
    assert pc["scale_mismatch"] == 0, pc
    if rc is not None:
        assert bitwise_equal(g, rc), compare(g, rc)
    return rep


@pytest.mark.parametrize("cfg,n,fs", [(1, 100_000, 3), (2, 300_000, 5), (3, 250_000, 5), (3, 120_000, 7)])
def test_configs_vs_oracle(cfg, n, fs):
    W, H = SENSOR[cfg]
    ev = farms.synth_config(cfg, n)
    g, r, rc = run_pair(ev, W, H, fs)
    rep = assert_parity(g, r, H, W, rc=rc)
    assert rep["valid_ref"] > n // 20  # the stream really exercises pooling


@pytest.mark.timeout(600)  # three CPU oracle passes over 2M events: past 120 s on a busy host
def test_config2_full_stream_vs_oracle():
    """BASELINE config 2 at its full size (2M events, 320 x 320, fs 5): every
    record against the oracle (both libms, run in parallel threads: ~40 s
    each)."""
    import threading

    ev = farms.synth_config(2)
    assert len(ev) == 2_000_000
    x, y, t, p = ev.relative()
    with farms.FlowManager(320, 320, 5, 5) as fm:
        g = fm.process(x, y, t, p)
    refs = {}

    def run(libm):
        refs[libm] = OracleFlow(320, 320, 5, 5, libm=libm).process(x, y, t, p)

    th = [threading.Thread(target=run, args=(m,)) for m in ("glibc", "cr")]
    for a in th:
        a.start()
    for a in th:
        a.join()
    rep = assert_parity(g, refs["glibc"], 320, 320, rc=refs["cr"])
    assert rep["valid_ref"] > 2_000_000 // 5


def test_config4_stream_vs_oracle():
    """BASELINE config 4's own stream (seed 0x5EED0004, fs 7, 11 scales): a
    500k-event head (the oracle takes ~12 s per libm)."""
    ev = farms.synth_config(4, 500_000)
    g, r, rc = run_pair(ev, 1280, 720, 7)
    rep = assert_parity(g, r, 720, 1280, rc=rc)
    assert rep["valid_ref"] > 500_000 // 20


def test_short_wide_sensor_double_visits():
    """W > H with 2*maxWindow >= H: the W-1 clip (vFlow.cpp:1000/1113) makes a
    window row run through several columns, so cells are visited twice by one
    scale and cells past the last column are cut (W*H bound).  The pooling
    order then differs from ascending cell order; the scale column must still
    match the reference's pooling exactly."""
    W, H = 160, 24
    n = 40_000
    ev = farms.synth_config(1, n)  # 128 x 128 bars, folded onto the short sensor
    x = (ev.x.astype(np.int64) % W).astype(np.int32)
    y = (ev.y.astype(np.int64) % H).astype(np.int32)
    t = (ev.t - ev.t[0]).astype(np.uint32)
    p = np.maximum(ev.p, 0).astype(np.int32)
    x[:50] = W - 1  # last column: the window runs past the end of the surfaces
    with farms.FlowManager(H, W, 3, 3) as fm:
        g = fm.process(x, y, t, p)
    r, rc = oracles(x, y, t, p, H, W, 3, 3)
    rep = assert_parity(g, r, H, W, rc=rc)
    assert rep["valid_ref"] > 1000


@pytest.mark.parametrize("pairs", ["1", "0"])
def test_short_wide_sensor_sparse_band_split_vs_oracle(pairs, monkeypatch):
    """k_cand's band-contiguous slots on a short wide sensor (160 x 24, M = 50
    > H): the W-1 clip carries every window row over three x-rows, so a row
    can cross a column band (32 columns here) two x-rows past its start, not
    only at the next one.  The row must split there: the slots between band
    b's last candidate and band b+1's first are not band b's.  The stream is
    sparse per pooling chunk (256-event chunks, ~10-30 % of the cells are
    candidates) and its stamps are compressed 64x, so that the ring of three
    candidate buffers (pool_batch 1) still holds contributors of a chunk three
    back in those slots: a row read past its band's count pools them.  Both
    pooling kernels (k_pool2 pairs, k_pool one event per wave) against the
    oracle."""
    W, H = 160, 24
    n = 40_000
    ev = farms.synth_config(1, n)
    x = (ev.x.astype(np.int64) % W).astype(np.int32)
    y = (ev.y.astype(np.int64) % H).astype(np.int32)
    t = ((ev.t - ev.t[0]) // 64).astype(np.uint32)
    p = np.maximum(ev.p, 0).astype(np.int32)
    monkeypatch.setenv("FARMS_CAND", "events")
    monkeypatch.setenv("FARMS_POOL_PAIRS", pairs)
    with farms.FlowManager(H, W, 3, 3, pool_chunk=256, pool_batch=1) as fm:
        g = fm.process(x, y, t, p)
        info = fm.kernel_info()
    assert info["cand_last"] == "k_cand", info
    assert info["pool"].startswith("k_pool2<" if pairs == "1" else "k_pool<"), info
    r, rc = oracles(x, y, t, p, H, W, 3, 3)
    rep = assert_parity(g, r, H, W, rc=rc)
    assert rep["valid_ref"] > 1000


def test_three_scales_vs_oracle():
    """BASELINE config 5 shape: fs=7 with scales {0,25,50}, a 500k-event head."""
    ev = farms.synth_config(5, 500_000)
    g, r, rc = run_pair(ev, 1280, 720, 7, jump=25, maxw=50)
    assert_parity(g, r, 720, 1280, 25, 50, rc=rc)
    assert set(np.unique(g.scale)) <= {0, 25, 50}


def test_chunking_is_bitwise_invariant():
    ev = farms.synth_config(3, 200_000)
    x, y, t, p = ev.relative()
    outs = []
    for fc, pc in [(0, 0), (777, 313), (50_000, 4096), (1 << 22, 1 << 20)]:
        with farms.FlowManager(720, 1280, 5, 5, fit_chunk=fc, pool_chunk=pc) as fm:
            outs.append(fm.process(x, y, t, p))
    for o in outs[1:]:
        assert bitwise_equal(outs[0], o)


def test_pool_variants_are_bitwise_invariant(monkeypatch):
    """k_pool is built twice (7- and 6-wave VGPR floors, pool_for picks by
    filter size): both builds give the same bits."""
    ev = farms.synth_config(3, 120_000)
    x, y, t, p = ev.relative()
    outs = []
    for cap in ("7", "6"):
        monkeypatch.setenv("FARMS_POOL_CAP", cap)
        with farms.FlowManager(720, 1280, 5, 5) as fm:
            outs.append(fm.process(x, y, t, p))
    assert bitwise_equal(outs[0], outs[1])


def test_streaming_split_equals_one_call():
    ev = farms.synth_config(2, 150_000)
    x, y, t, p = ev.relative()
    with farms.FlowManager(320, 320, 5, 5) as fm:
        whole = fm.process(x, y, t, p)
    with farms.FlowManager(320, 320, 5, 5) as fm:
        parts = [fm.process(x[a:b], y[a:b], t[a:b], p[a:b]) for a, b in [(0, 1), (1, 40_000), (40_000, 40_001),
                                                                       (40_001, 150_000)]]
    cat = {c: np.concatenate([getattr(q, c) for q in parts]) for c in farms.COLUMNS}
    assert bitwise_equal(whole, cat)


def test_reset_restarts_the_stream():
    ev = farms.synth_config(1, 20_000)
    x, y, t, p = ev.relative()
    with farms.FlowManager(128, 128, 3, 5) as fm:
        a = fm.process(x, y, t, p)
        fm.reset()
        b = fm.process(x, y, t, p)
    assert bitwise_equal(a, b)


def test_unsorted_timestamps_vs_oracle():
    """The reference never assumes time order: wrapped / out-of-order stamps,
    future stamps (MAXSTAMP branch, vFlow.cpp:897-902 and 1229-1230)."""
    rng = np.random.default_rng(7)
    ev = farms.synth_config(2, 60_000)
    x, y, t, p = ev.relative()
    t = t.astype(np.int64)
    swap = rng.random(t.shape[0]) < 0.05
    t[swap] = rng.integers(0, int(t.max()) + 1, swap.sum())
    t = t.astype(np.uint32)
    with farms.FlowManager(320, 320, 5, 5) as fm:
        g = fm.process(x, y, t, p)
    r, rc = oracles(x, y, t, p, 320, 320, 5, 5)
    assert_parity(g, r, 320, 320, rc=rc)


def test_edges_hot_pixel_and_filter_sizes():
    rng = np.random.default_rng(11)
    W, H = 64, 48
    n = 30_000
    x = rng.integers(0, W, n).astype(np.int32)
    y = rng.integers(0, H, n).astype(np.int32)
    # corners, borders and one hot pixel firing a long burst
    x[:400] = rng.choice([0, W - 1], 400)
    y[400:800] = rng.choice([0, H - 1], 400)
    x[5000:9000] = 17
    y[5000:9000] = 9
    t = np.sort(rng.integers(0, 2_000_000, n)).astype(np.uint32)
    t[6000:6100] = t[6000]  # equal stamps
    p = rng.integers(0, 2, n).astype(np.int32)
    for fs, inl in [(1, 5), (2, 3), (4, 5), (5, 0), (6, 7), (7, 4), (9, 10)]:
        with farms.FlowManager(H, W, fs, inl) as fm:
            g = fm.process(x, y, t, p)
        r, rc = oracles(x, y, t, p, H, W, fs, inl)
        assert_parity(g, r, H, W, rc=rc)


def test_tall_sensor_and_tiny_sensor():
    rng = np.random.default_rng(3)
    for W, H in [(40, 200), (5, 5), (3, 7)]:
        n = 8000
        x = rng.integers(0, W, n).astype(np.int32)
        y = rng.integers(0, H, n).astype(np.int32)
        t = np.sort(rng.integers(0, 400_000, n)).astype(np.uint32)
        p = np.ones(n, np.int32)
        with farms.FlowManager(H, W, 3, 3) as fm:
            g = fm.process(x, y, t, p)
        r, rc = oracles(x, y, t, p, H, W, 3, 3)
        assert_parity(g, r, H, W, rc=rc)


def test_empty_and_single_event():
    with farms.FlowManager(320, 320, 3, 5) as fm:
        e = fm.process(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.uint32), np.zeros(0, np.int32))
        assert e.n == 0
        one = fm.process(np.array([5], np.int32), np.array([6], np.int32), np.array([0], np.uint32),
                         np.array([1], np.int32))
    assert one.x[0] == 5 and one.y[0] == 6 and one.r_local[0] == 0 and one.scale[0] == 0


def test_out_of_sensor_event_is_rejected():
    with farms.FlowManager(32, 32, 3, 5) as fm:
        with pytest.raises(farms.FarmsError) as ei:
            fm.process(np.array([1, 32], np.int32), np.array([1, 1], np.int32), np.array([0, 1], np.uint32),
                       np.array([1, 1], np.int32))
        assert ei.value.code == farms.FARMS_EINVAL
        # the handle stays usable
        ok = fm.process(np.array([1], np.int32), np.array([1], np.int32), np.array([0], np.uint32),
                        np.array([1], np.int32))
        assert ok.n == 1


@pytest.mark.parametrize("fs", [3, 5, 7])
def test_fit_variants_are_bitwise_identical(fs, monkeypatch):
    """The quad-lane fits (FARMS_FIT_MODE 0: re-gathered winning window, 1:
    union tile by columns, 2: union tile by rows) and the one-thread fit
    evaluate the same arithmetic in the same order: bitwise-equal records.
    The sweep on one fit stream or two (FARMS_FIT_STREAMS, even / odd chunks;
    small fit chunks so that there are many of each) gives the same bits."""
    ev = farms.synth_config(3, 150_000)
    x, y, t, p = ev.relative()
    outs = []
    for quad, mode, streams, fc in [("1", "1", "2", 0), ("1", "0", "2", 0), ("1", "2", "2", 0), ("0", "1", "2", 0),
                                    ("1", "1", "1", 0), ("1", "1", "1", 8192), ("1", "1", "2", 8192)]:
        monkeypatch.setenv("FARMS_FIT_QUAD", quad)
        monkeypatch.setenv("FARMS_FIT_MODE", mode)
        monkeypatch.setenv("FARMS_FIT_STREAMS", streams)
        with farms.FlowManager(720, 1280, fs, 5, fit_chunk=fc) as fm:
            outs.append(fm.process(x, y, t, p))
    for o in outs[1:]:
        assert bitwise_equal(outs[0], o)


def test_full_size_stream_properties():
    """BASELINE config 3 at full size (50M events, 1280x720, fs 5): the run is
    bitwise invariant to chunking, and its first 100k records equal the
    oracle's run of those 100k events (the path is causal)."""
    import torch

    ev = farms.synth_config(3)
    x, y, t, p = ev.relative()
    n = len(x)
    assert n == 50_000_000
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in (x, y, t.view(np.int32), p)]
    outs = []
    for fc, pc in [(0, 0), (262_144, 16_384)]:
        o = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
             for c in farms.COLUMNS[4:]}
        with farms.FlowManager(720, 1280, 5, 5, fit_chunk=fc, pool_chunk=pc) as fm:
            fm.process_device(*d, o)
        outs.append(o)
    for c in farms.COLUMNS[4:]:
        a, b = outs[0][c], outs[1][c]
        if a.dtype == torch.float64:
            a, b = a.view(torch.int64), b.view(torch.int64)
        assert torch.equal(a, b), c
    k = 100_000
    g = {c: v for c, v in zip(farms.COLUMNS[:4], (x[:k], y[:k], t[:k].astype(np.int32), p[:k]))}
    g.update({c: outs[0][c][:k].cpu().numpy() for c in farms.COLUMNS[4:]})
    r, rc = oracles(x[:k], y[:k], t[:k], p[:k], 720, 1280, 5, 5)
    assert_parity(g, r, 720, 1280, rc=rc)
    assert int((outs[0]["r_local"] > 0).sum()) > n // 4  # most of the stream is pooled


def test_host_path_plan_on_a_stream_that_jumps_back(monkeypatch):
    """The host-array path decides each sub-batch's candidate build (k_cand or
    k_chain) from its own copy of the stamps (host_plan_reach) instead of
    waiting for the device's plan.  A stream whose second half comes first --
    its stamps jump back by about half the span at the seam, so the chunks past
    the seam reach back to the first chunk (k_chain) while the others stay
    time-ordered (k_cand) -- gives bitwise the device path's records, with
    FARMS_PLAN_CHECK=1 comparing the two plans of every sub-batch."""
    import torch

    monkeypatch.setenv("FARMS_PLAN_CHECK", "1")
    ev = farms.synth_config(3, 2_000_000)
    x, y, t, p = ev.relative()
    h = len(x) // 2 + 12_345  # the seam inside a sub-batch, not on a chunk boundary
    x, y, t, p = (np.ascontiguousarray(np.concatenate([a[h:], a[:h]])) for a in (x, y, t, p))
    n = len(x)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in (x, y, t.view(np.int32), p)]
    o = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    with farms.FlowManager(720, 1280, 5, 5, pool_chunk=1024, pool_batch=8) as fm:
        fm.process_device(*d, o)
        fm.reset()
        g = fm.process(x, y, t, p)
    dd = {c: v for c, v in zip(farms.COLUMNS[:4], (x, y, t.astype(np.int32), p))}
    dd.update({c: o[c].cpu().numpy() for c in farms.COLUMNS[4:]})
    assert bitwise_equal(g, dd)
    assert int((dd["r_local"] > 0).sum()) > n // 4


@pytest.mark.parametrize("threads,pool_chunk,pin", [("1", 1024, "none"), ("3", 2048, "all"), ("8", 0, "mixed"),
                                                    ("8", 1024, "all")])
def test_host_path_equals_device_path(threads, pool_chunk, pin, monkeypatch):
    """farms_process (pipelined sub-batches -- several here: the stream is 3M
    events, a sub-batch at least 4 super-chunks of pool_chunk x pool_batch --,
    record downloads overlapped per pooling super-chunk, pinned arrays DMAed
    in place and pageable ones staged) gives bitwise the records of
    farms_process_device on the same stream, for any thread count and mix of
    pinned and pageable arrays."""
    import torch

    monkeypatch.setenv("FARMS_HOST_THREADS", threads)
    monkeypatch.setenv("FARMS_PLAN_CHECK", "1")  # each sub-batch's host-side plan against the device's
    ev = farms.synth_config(3, 3_000_000)
    x, y, t, p = ev.relative()
    n = len(x)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(a).to(dev) for a in (x, y, t.view(np.int32), p)]
    o = {c: torch.empty(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    keep = []
    ins = [x, y, t, p]
    if pin != "none":
        for i in ((0, 1, 2, 3) if pin == "all" else (1, 2)):
            ins[i], own = farms.pinned(ins[i])
            keep.append(own)
    rec = farms.Records(n, pinned=pin == "all")
    if pin == "mixed":  # a pinned record column and a pinned echo column among pageable ones
        for c in ("vx", "t"):
            a, own = farms.pinned(getattr(rec, c))
            setattr(rec, c, a)
            keep.append(own)
    with farms.FlowManager(720, 1280, 5, 5, pool_chunk=pool_chunk, pool_batch=8 if pool_chunk else 0) as fm:
        fm.process_device(*d, o)
        fm.reset()
        g = fm.process(*ins, out=rec)
        fm.reset()
        g1 = fm.process(x[:777], y[:777], t[:777], p[:777])  # one sub-batch
    dd = {c: v for c, v in zip(farms.COLUMNS[:4], (x, y, t.astype(np.int32), p))}
    dd.update({c: o[c].cpu().numpy() for c in farms.COLUMNS[4:]})
    assert bitwise_equal(g, dd)
    assert g1.n == 777 and np.array_equal(g1.scale, dd["scale"][:777])


@pytest.mark.parametrize("subs,echo", [("1", "1"), ("3", "0"), ("16", "1")])
def test_host_path_pipeline_knobs_are_bitwise_invariant(subs, echo, monkeypatch):
    """The host path's pipeline knobs change only how the work is cut and
    moved: FARMS_SUBBATCHES (one call, or n/k events per sub-batch) and
    FARMS_ECHO_DMA (1: the x/y/t/p echo into pinned record columns by D2H from
    the device copies; 0, the default since round 5: by host copies from the
    inputs) give bitwise the default's records."""
    ev = farms.synth_config(3, 2_000_000)
    x, y, t, p = ev.relative()
    keep = []
    ins = [x, y, t, p]
    for i in range(4):
        ins[i], own = farms.pinned(ins[i])
        keep.append(own)
    with farms.FlowManager(720, 1280, 5, 5, pool_chunk=1024, pool_batch=8) as fm:
        ref = fm.process(*ins, out=farms.Records(len(x), pinned=True))
    monkeypatch.setenv("FARMS_SUBBATCHES", subs)
    monkeypatch.setenv("FARMS_ECHO_DMA", echo)
    with farms.FlowManager(720, 1280, 5, 5, pool_chunk=1024, pool_batch=8) as fm:
        g = fm.process(*ins, out=farms.Records(len(x), pinned=True))
    assert bitwise_equal(ref, g)
    assert np.array_equal(g.x, x) and np.array_equal(g.t.view(np.uint32), t)


@pytest.mark.parametrize("pin", [False, True])
def test_host_path_out_of_sensor_in_a_later_sub_batch(pin):
    """An event outside the sensor stops a pipelined call before its sub-batch
    (pinned or pageable inputs); after a reset the handle processes the stream
    as if fresh."""
    ev = farms.synth_config(3, 2_000_000)
    x, y, t, p = ev.relative()
    xb = x.copy()
    xb[-5] = 1280
    keep = []
    ins = [xb, y, t, p]
    if pin:
        for i in range(4):
            ins[i], own = farms.pinned(ins[i])
            keep.append(own)
    with farms.FlowManager(720, 1280, 5, 5, pool_chunk=1024, pool_batch=8) as fm:
        with pytest.raises(farms.FarmsError) as ei:
            fm.process(*ins)
        assert ei.value.code == farms.FARMS_EINVAL
        fm.reset()
        a = fm.process(x, y, t, p)
    with farms.FlowManager(720, 1280, 5, 5, pool_chunk=1024, pool_batch=8) as fm:
        b = fm.process(x, y, t, p)
    assert bitwise_equal(a, b)


def serial_inputs(ev):
    """vFlowManager::run's view of a file (vFlow.cpp:520-580): the first line
    only stamps lastEventTime with its absolute time; the loop's events carry
    t - t0 (t0 = the first line's stamp) and clamped polarity."""
    first = (int(ev.x[0]), int(ev.y[0]), int(ev.t[0]))
    x, y = ev.x[1:].astype(np.int32), ev.y[1:].astype(np.int32)
    t = (ev.t[1:].astype(np.uint32) - np.uint32(ev.t[0])).astype(np.uint32)
    p = np.maximum(ev.p[1:], 0).astype(np.int32)
    return first, x, y, t, p


def run_serial(first, x, y, t, p, H, W, fs, inl=5, jump=5, maxw=50, splits=None, **kw):
    with farms.FlowManager(H, W, fs, inl, window_jump=jump, max_window=maxw, serial=True, **kw) as fm:
        fm.serial_first(*first)
        if splits is None:
            g = fm.process(x, y, t, p)
        else:
            parts = [fm.process(x[a:b], y[a:b], t[a:b], p[a:b]) for a, b in splits]
            g = {c: np.concatenate([getattr(q, c) for q in parts]) for c in farms.COLUMNS}
    outs = []
    for libm in ("glibc", "cr"):
        o = OracleFlow(H, W, fs, inl, jump, maxw, serial=True, libm=libm)
        o.serial_first(*first)
        outs.append(o.process(x, y, t, p))
    return g, outs[0], outs[1]


def assert_serial_parity(g, r, rc, H, W, first, jump=5, maxw=50):
    rep = compare(g, r)
    pc = pooling_check(g, H, W, jump, maxw, serial=True, first=first)
    print(rep, pc)
    assert rep["ok"], rep
    assert pc["ok"] and pc["scale_mismatch"] == 0, pc
    assert bitwise_equal(g, rc), compare(g, rc)
    return rep


@pytest.mark.parametrize("cfg,n,fs", [(1, 100_000, 3), (2, 200_000, 5), (3, 150_000, 5), (4, 100_000, 7)])
def test_serial_mode_vs_oracle(cfg, n, fs):
    """--SERIAL 1 (vFlowManager::run, the reference CLI's default): own cell
    pooled with the previous stamp at its pixel, fallback to the own flow when
    nothing contributes (vFlow.cpp:790, 1085-1094)."""
    W, H = {1: (128, 128), 2: (320, 320), 3: (1280, 720), 4: (1280, 720)}[cfg]
    first, x, y, t, p = serial_inputs(farms.synth_config(cfg, n + 1))
    g, r, rc = run_serial(first, x, y, t, p, H, W, fs)
    rep = assert_serial_parity(g, r, rc, H, W, first)
    assert rep["valid_ref"] > n // 20


def test_serial_first_line_stamp_and_streaming():
    """The first line's absolute stamp sits in lastEventTime of its pixel: with a
    small t0 an early event there pools its own cell against it.  Serial mode
    is also bitwise invariant to splitting the stream across calls and to the
    chunk sizes."""
    ev = farms.synth_config(1, 60_001)
    t = (ev.t - ev.t[0] + 300).astype(np.uint32)  # t0 = 300
    ev = farms.Events(ev.x.copy(), ev.y.copy(), t, ev.p.copy())
    # events 1..40 at the first line's pixel, 10 us apart (relative 0..400)
    ev.x[1:41], ev.y[1:41] = ev.x[0], ev.y[0]
    ev.t[1:41] = 300 + 10 * np.arange(40, dtype=np.uint32)
    order = np.argsort(ev.t, kind="stable")
    ev = farms.Events(ev.x[order], ev.y[order], ev.t[order], ev.p[order])
    first, x, y, t, p = serial_inputs(ev)
    g, r, rc = run_serial(first, x, y, t, p, 128, 128, 3)
    assert_serial_parity(g, r, rc, 128, 128, first)
    g2, _, _ = run_serial(first, x, y, t, p, 128, 128, 3, splits=[(0, 7), (7, 20_000), (20_000, len(x))],
                          fit_chunk=1000, pool_chunk=256)
    assert bitwise_equal(g, g2)


def test_serial_first_only_on_a_fresh_handle():
    """farms_serial_first after events would overwrite the previous-stamp source
    of the serial pooling: refused until a reset.  The first line's stamp shows
    in lastEventTime until an event fires at its pixel (vFlow.cpp:556)."""
    with farms.FlowManager(32, 32, 3, 5, serial=True) as fm:
        fm.serial_first(3, 4, 777)
        lt = np.zeros(32 * 32)
        fm._lib.farms_get_last_event_time(fm._h, lt.ctypes.data_as(__import__("ctypes").c_void_p))
        assert lt[3 * 32 + 4] == 777
        fm.process(np.array([1], np.int32), np.array([1], np.int32), np.array([5], np.uint32), np.array([1], np.int32))
        with pytest.raises(farms.FarmsError) as ei:
            fm.serial_first(3, 4, 777)
        assert ei.value.code == farms.FARMS_EINVAL
        fm.process(np.array([3], np.int32), np.array([4], np.int32), np.array([0], np.uint32), np.array([1], np.int32))
        fm._lib.farms_get_last_event_time(fm._h, lt.ctypes.data_as(__import__("ctypes").c_void_p))
        assert lt[3 * 32 + 4] == 0 and lt[1 * 32 + 1] == 5  # the event's own (relative) stamp 0 now
        fm.reset()
        fm.serial_first(3, 4, 777)


def _process(x, y, t, p, H, W, fs, splits=None, serial_first=None, **kw):
    with farms.FlowManager(H, W, fs, 5, serial=serial_first is not None, **kw) as fm:
        if serial_first is not None:
            fm.serial_first(*serial_first)
        if splits is None:
            g = fm.process(x, y, t, p)
            g = {c: getattr(g, c) for c in farms.COLUMNS}
        else:
            parts = [fm.process(x[a:b], y[a:b], t[a:b], p[a:b]) for a, b in splits]
            g = {c: np.concatenate([getattr(q, c) for q in parts]) for c in farms.COLUMNS}
        return g, fm.kernel_info()["cand_last"]


def test_candidate_builds_are_bitwise_identical(monkeypatch):
    """The pooling candidate lists come from k_cand (event-driven, chunks
    independent) on time-local streams and from k_chain (the per-cell chain)
    otherwise; FARMS_CAND forces either.  Both give the same bits on every
    stream shape: time-ordered (C3, with many small pooling chunks too, and C4's
    fs 7), split across calls, serial mode, and out-of-order stamps."""
    ev3 = farms.synth_config(3, 200_000)
    x3, y3, t3, p3 = ev3.relative()
    ev2 = farms.synth_config(2, 120_000)
    x2, y2, t2, p2 = ev2.relative()
    rng = np.random.default_rng(11)
    tu = t2.astype(np.int64)
    swap = rng.random(tu.shape[0]) < 0.05
    tu[swap] = rng.integers(0, int(tu.max()) + 1, swap.sum())
    tu = tu.astype(np.uint32)
    ev4 = farms.synth_config(4, 150_000)
    x4, y4, t4, p4 = ev4.relative()
    first, xs, ys, ts, ps = serial_inputs(farms.synth_config(1, 60_001))
    cases = [
        ("c3", (x3, y3, t3, p3, 720, 1280, 5), {}, "k_cand"),
        ("c3_small_chunks", (x3, y3, t3, p3, 720, 1280, 5), {"pool_chunk": 1024, "pool_batch": 16}, "k_cand"),
        ("c4", (x4, y4, t4, p4, 720, 1280, 7), {}, "k_cand"),
        ("c2_split", (x2, y2, t2, p2, 320, 320, 5), {"splits": [(0, 1), (1, 40_000), (40_000, 40_001),
                                                              (40_001, 120_000)]}, "k_cand"),
        ("c1_serial", (xs, ys, ts, ps, 128, 128, 3), {"serial_first": first, "splits": [(0, 7), (7, 30_000),
                                                                                      (30_000, len(xs))]}, "k_cand"),
        # (235 chunks: the random stamps reach back further than kCandMaxBack)
        ("c2_unsorted", (x2, y2, tu, p2, 320, 320, 5), {"pool_chunk": 512}, "k_chain"),
    ]
    for name, args, kw, default in cases:
        outs = {}
        for mode in ("", "events", "chain"):
            if mode:
                monkeypatch.setenv("FARMS_CAND", mode)
            else:
                monkeypatch.delenv("FARMS_CAND", raising=False)
            outs[mode], used = _process(*args, **kw)
            want = {"": default, "events": "k_cand", "chain": "k_chain"}[mode]
            assert used == want, (name, mode, used)
        for mode in ("events", "chain"):
            assert bitwise_equal(outs[""], outs[mode]), (name, mode, compare(outs[""], outs[mode]))


def test_work_order_builds_are_bitwise_identical(monkeypatch):
    """The work order (tile-sorted events of each pooling chunk), the fit
    descriptors, the column-band starts and the chunk spans come from one
    workgroup per chunk (k_chunk_order, pooling chunks of 2,048 / 4,096 / 8,192
    events) or from the device-wide sort (FARMS_ORDER=sort; any other chunk
    size, e.g. fs 7's 16,384): the same bits for every chunk size either way."""
    ev = farms.synth_config(3, 150_000)
    x, y, t, p = ev.relative()
    outs = []
    for pc in (2048, 4096, 8192, 16384):
        for order in ("", "sort"):
            if order:
                monkeypatch.setenv("FARMS_ORDER", order)
            else:
                monkeypatch.delenv("FARMS_ORDER", raising=False)
            with farms.FlowManager(720, 1280, 5, 5, pool_chunk=pc) as fm:
                outs.append(fm.process(x, y, t, p))
    for o in outs[1:]:
        assert bitwise_equal(outs[0], o)


@pytest.mark.parametrize("shift", ["2", "4"])
def test_work_order_tile_sizes_are_bitwise_identical(shift, monkeypatch):
    """FARMS_TILE_SHIFT (log2 of the work-order tile's edge: 4x4 and 16x16
    tiles against the default 8x8) changes the order in which the fit and the
    pooling visit a chunk's events, the column bands of k_cand and the block
    placement, never the records (both order paths: k_chunk_order and the
    device-wide sort)."""
    ev = farms.synth_config(3, 150_000)
    x, y, t, p = ev.relative()
    monkeypatch.delenv("FARMS_TILE_SHIFT", raising=False)
    with farms.FlowManager(720, 1280, 5, 5) as fm:
        ref = fm.process(x, y, t, p)
    monkeypatch.setenv("FARMS_TILE_SHIFT", shift)
    for order in ("", "sort"):
        if order:
            monkeypatch.setenv("FARMS_ORDER", order)
        else:
            monkeypatch.delenv("FARMS_ORDER", raising=False)
        with farms.FlowManager(720, 1280, 5, 5) as fm:
            assert bitwise_equal(ref, fm.process(x, y, t, p)), (shift, order)


def _device_run(fm, x, y, t, p, splits, two_phase):
    """Records of one device-resident run: process_device per split, or the
    two-phase calls with the fit of split b+1 issued before the pooling of b
    (two fits pending, as multirank.Stepper runs the x-strips)."""
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x, y, t.view(np.int32), p)]
    n = len(x)
    o = {c: torch.zeros(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}

    def sl(a, b):
        return [v[a:b] for v in d], {c: v[a:b] for c, v in o.items()}

    if not two_phase:
        for a, b in splits:
            ins, out = sl(a, b)
            fm.process_device(*ins, out)
    else:
        pending = 0
        for a, b in splits:
            ins, out = sl(a, b)
            fm.fit_device(*ins, out)
            pending += 1
            if pending == 2:
                fm.pool_device()
                pending -= 1
        for _ in range(pending):
            fm.pool_device()
    torch.cuda.synchronize()
    g = {c: v for c, v in zip(farms.COLUMNS[:4], (x, y, t.astype(np.int32), p))}
    g.update({c: o[c].cpu().numpy() for c in farms.COLUMNS[4:]})
    return g


@pytest.mark.parametrize("fs", [5, 7])
def test_fit_streams_on_device_paths_are_bitwise_identical(fs, monkeypatch):
    """The fit sweep on one stream or two (FARMS_FIT_STREAMS; even / odd fit
    chunks, the fs-7 default of the device calls): independent even / odd SAE
    preps, final commits waiting across streams and a k_flow waiting on the
    other stream's last fit.  Run where the two streams are used -- device
    calls (farms_process_device, split in several calls) and the two-phase
    calls with two fits pending (farms_fit_device / farms_pool_device, the
    x-strips' pipelined step) -- with small fit chunks (many of each parity):
    bitwise the host path's one-stream run (farms_process)."""
    ev = farms.synth_config(4 if fs == 7 else 3, 200_000)
    x, y, t, p = ev.relative()
    with farms.FlowManager(720, 1280, fs, 5) as fm:
        ref = fm.process(x, y, t, p)
    splits = [(0, 70_001), (70_001, 70_002), (70_002, 140_000), (140_000, len(x))]
    for streams in ("1", "2"):
        monkeypatch.setenv("FARMS_FIT_STREAMS", streams)
        for two_phase in (False, True):
            with farms.FlowManager(720, 1280, fs, 5, fit_chunk=8192) as fm:
                g = _device_run(fm, x, y, t, p, splits, two_phase)
            assert bitwise_equal(ref, g), (streams, two_phase, compare(ref, g))


def test_paired_pooling_overflow_past_the_pair_bitmap_is_bitwise(monkeypatch):
    """An event whose window holds more than kPairBitPos (1,024) candidates
    leaves the pair's bitmap: k_pool2 lists it and k_pool_ovf pools it one
    event per wave with the full bitmap, right after the launch.  A C2 stream
    with its stamps compressed 16x (dense windows) through both pooling kernels
    gives the same bits, and the scan-width tail shows the path ran."""
    ev = farms.synth_config(2, 200_001)
    x, y, t, p = ev.relative()
    t = (t // 16).astype(t.dtype)
    outs, tail = {}, {}
    for pairs in ("1", "0"):
        monkeypatch.setenv("FARMS_POOL_PAIRS", pairs)
        with farms.FlowManager(320, 320, 5, 5) as fm:
            fm.set_profiling(True)
            outs[pairs] = fm.process(x, y, t, p)
            tail[pairs] = fm.stats()["pool_scan_max"]
    assert tail["1"] > 1024, tail
    assert bitwise_equal(outs["1"], outs["0"]), compare(outs["0"], outs["1"])
    assert int((outs["1"].r_true != 0).sum()) > 1000


@pytest.mark.parametrize("jump,maxw,pc", [(50, 50, 0), (25, 50, 0), (10, 50, 2048), (5, 50, 0), (4, 50, 0), (5, 20, 1024)])
def test_paired_pooling_is_bitwise_one_event_per_wave(jump, maxw, pc, monkeypatch):
    """k_pool2 pools two events per wave (K <= 11 scales: 3 (K - 1) lanes per
    event, counts from a histogram, scale 0 from the own entry) and k_pool one
    (FARMS_POOL_PAIRS=0, and every K > 11 or odd pooling chunk): the same bits,
    for 2 to 13 scales, an odd-sized last pair and partial last chunks."""
    ev = farms.synth_config(3, 150_001)
    x, y, t, p = ev.relative()
    K = maxw // jump + 1
    outs = {}
    for pairs in ("1", "0"):
        monkeypatch.setenv("FARMS_POOL_PAIRS", pairs)
        with farms.FlowManager(720, 1280, 5, 5, window_jump=jump, max_window=maxw, pool_chunk=pc) as fm:
            outs[pairs] = fm.process(x, y, t, p)
            kern = fm.kernel_info()["pool"]
        want = "k_pool2<" if pairs == "1" and 2 <= K <= 11 else "k_pool<"
        assert kern.startswith(want), (kern, K)
    assert bitwise_equal(outs["1"], outs["0"]), compare(outs["0"], outs["1"])
    assert int((outs["1"].r_true != 0).sum()) > 1000


@pytest.mark.parametrize("fs", [5, 7])
def test_async_exchange_order_is_bitwise(fs):
    """The x-strip stepper's order (multirank.Stepper.step): the gather of
    sub-batch b queued behind its fit, the fit of b+1 issued before the host
    waits for it (two fits pending, three workspace sets in rotation), the
    scatter queued on the chain stream ahead of b's pooling.  Records bitwise
    farms_process; the exported flows bitwise those of one fit at a time with
    the synchronous farms_export_flows (the exchange calls act on the oldest
    fit not yet pooled).  A second pass re-imports a subset of each sub-batch's
    exported flows, every third with L = 0 (the event then counts as invalid),
    through both orders: the scatter on the chain stream ahead of the pooling
    takes effect (records differ from the plain run) and the two orders agree
    bit for bit."""
    ev = farms.synth_config(4 if fs == 7 else 3, 200_000)
    x, y, t, p = ev.relative()
    with farms.FlowManager(720, 1280, fs, 5) as fm:
        ref = fm.process(x, y, t, p)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x, y, t.view(np.int32), p)]
    n = len(x)
    splits = [(0, 50_000), (50_000, 50_001), (50_001, 120_000), (120_000, 160_000), (160_000, n)]
    none = torch.zeros(0, dtype=torch.int32, device=dev)

    def imports(b, idx, bufs, reimport, keep):
        """(indices, flows) to import after sub-batch b's export: none, or
        every other exported slot with every third of those zeroed (kept
        alive until the end: the engine reads them when the pooling runs)."""
        if not reimport:
            return none, bufs[b]
        sel = torch.arange(0, len(idx[b]), 2, device=dev)
        ii = idx[b][sel].contiguous()
        fl = bufs[b][sel].clone()
        fl[::3, 0] = 0.0
        torch.cuda.current_stream().synchronize()  # both made on torch's stream: complete before the engine reads them
        keep += [ii, fl]
        return ii, fl

    def run(async_order, reimport=False):
        o = {c: torch.zeros(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
             for c in farms.COLUMNS[4:]}
        idx = [torch.arange(0, b - a, 5, dtype=torch.int32, device=dev) for a, b in splits]
        bufs = [torch.full((len(i), 3), -1.0, dtype=torch.float64, device=dev) for i in idx]
        keep = []
        with farms.FlowManager(720, 1280, fs, 5, fit_chunk=8192) as fm:
            def fit(b):
                a, e = splits[b]
                fm.fit_device(*[v[a:e] for v in d], {c: v[a:e] for c, v in o.items()})

            if async_order:
                def exchange(b, nxt):
                    fm.export_flows_async(idx[b], bufs[b])
                    if nxt < len(splits):
                        fit(nxt)
                    fm.export_wait()
                    fm.import_flows_async(*imports(b, idx, bufs, reimport, keep))
                fit(0)
                exchange(0, 1)
                for b in range(len(splits)):
                    fm.pool_device()
                    if b + 1 < len(splits):
                        exchange(b + 1, b + 2)
            else:
                for b in range(len(splits)):
                    fit(b)
                    fm.export_flows(idx[b], bufs[b])
                    fm.import_flows(*imports(b, idx, bufs, reimport, keep))
                    fm.pool_device()
            torch.cuda.synchronize()
        g = {c: v for c, v in zip(farms.COLUMNS[:4], (x, y, t.astype(np.int32), p))}
        g.update({c: o[c].cpu().numpy() for c in farms.COLUMNS[4:]})
        return g, [b.cpu().numpy() for b in bufs]

    g_async, f_async = run(True)
    g_sync, f_sync = run(False)
    assert bitwise_equal(ref, g_async), compare(ref, g_async)
    assert bitwise_equal(ref, g_sync), compare(ref, g_sync)
    for a, b in zip(f_async, f_sync):
        assert a.tobytes() == b.tobytes()
        assert (a[:, 0] >= 0).all()  # every slot written
    r_async, _ = run(True, reimport=True)
    r_sync, _ = run(False, reimport=True)
    assert bitwise_equal(r_async, r_sync), compare(r_sync, r_async)
    assert not bitwise_equal(ref, r_sync)  # the zeroed flows took effect


def test_exchange_index_outside_the_fit_is_refused():
    """farms_export_flows / farms_import_flows with an index outside the fit's
    events: nothing is read or written through it (no device fault) and the
    synchronous calls return FARMS_EINVAL; the handle then pools as usual."""
    ev = farms.synth_config(2, 20_000)
    x, y, t, p = ev.relative()
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x, y, t.view(np.int32), p)]
    n = len(x)
    o = {c: torch.zeros(n, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    with farms.FlowManager(320, 320, 5, 5) as fm:
        ref = fm.process(x, y, t, p)
        fm.reset()
        fm.fit_device(*d, o)
        bad = torch.tensor([0, n, -1, 1 << 30], dtype=torch.int32, device=dev)
        buf = torch.full((4, 3), -7.0, dtype=torch.float64, device=dev)
        torch.cuda.current_stream().synchronize()  # (made on torch's stream)
        for call in (lambda: fm.export_flows(bad, buf), lambda: fm.import_flows(bad[1:], buf[1:])):
            with pytest.raises(farms.FarmsError) as ei:
                call()
            assert ei.value.code == farms.FARMS_EINVAL
        assert (buf[1:] == -7.0).all() and (buf[0] >= 0).all()  # only the valid slot written
        fm.pool_device()
    g = {c: v for c, v in zip(farms.COLUMNS[:4], (x, y, t.astype(np.int32), p))}
    g.update({c: o[c].cpu().numpy() for c in farms.COLUMNS[4:]})
    assert bitwise_equal(ref, g), compare(ref, g)
