"""Known-answer tests pinning the CPU oracle (oracle/farms_oracle.c).

The reference ships no tests or fixtures and cannot be built here (SURVEY.md
§4, §8c), so the oracle is pinned by cases whose answer follows from the
reference's formulas by hand (vFlow.cpp line numbers cited per case).  Overall
parity status: "parity unpinned" (DESIGN.md §4).
"""
import math

import numpy as np
import pytest

from oracle import OracleFlow


def ramp(W, H, a, b, t0=0):
    """All pixels fire once, in time order, with t = (a*x + b*y)*1e6 us (a, b in
    s/px): a plane of slopes dt/dx = a, dt/dy = b."""
    xs, ys = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")
    x, y = xs.ravel(), ys.ravel()
    t = np.rint((a * x + b * y) * 1e6).astype(np.int64) + t0
    order = np.lexsort((y, x, t))
    return (x[order].astype(np.int32), y[order].astype(np.int32), t[order].astype(np.uint32),
            np.ones(x.size, np.int32))


@pytest.mark.parametrize("fs", [3, 5, 7])
def test_planar_ramp_recovers_the_plane(fs):
    """computeGrads fits t = a x + b y + c (vFlow.cpp:1307-1341); the flow is
    speed * (cos, sin)(atan2(a, b)) with speed = 1/sqrt(a^2+b^2)
    (vFlow.cpp:1373-1377), i.e. Vx = b/(a^2+b^2), Vy = a/(a^2+b^2)."""
    a, b = 2e-3, 1e-3
    x, y, t, p = ramp(40, 30, a, b)
    out = OracleFlow(30, 40, fs, 5).process(x, y, t, p)
    vx_ref, vy_ref = b / (a * a + b * b), a / (a * a + b * b)
    fr = fs // 2
    inner = (x >= 3 * fr) & (x < 40 - 3 * fr) & (y >= 3 * fr) & (y < 30 - 3 * fr) & (t > 0)
    assert inner.sum() > 100
    assert np.all(out["r_local"][inner] > 0)
    np.testing.assert_allclose(out["vx"][inner], vx_ref, rtol=2e-3)
    np.testing.assert_allclose(out["vy"][inner], vy_ref, rtol=2e-3)
    # local theta = atan2(Vy, Vx) (vFlow.cpp:325)
    np.testing.assert_allclose(out["theta_local"][inner], math.atan2(vy_ref, vx_ref), atol=2e-3)


def test_first_event_is_invalid():
    """A lone event: every window holds unvisited cells stored as Event(0,0,0,0)
    (vFlow.cpp:80-93), AtA is rank 2, DET < 1 (vFlow.cpp:1323) -> no flow."""
    out = OracleFlow(32, 32, 3, 5).process(np.array([10], np.int32), np.array([12], np.int32),
                                           np.array([0], np.uint32), np.array([1], np.int32))
    assert out["vx"][0] == 0 and out["vy"][0] == 0 and out["r_local"][0] == 0
    assert out["r_true"][0] == 0 and out["scale"][0] == 0
    assert out["x"][0] == 10 and out["y"][0] == 12 and out["t"][0] == 0 and out["p"][0] == 1


def test_clipped_windows_give_no_flow():
    """Windows crossing the border are skipped (vFlow.cpp:889); on a 3x3 sensor
    with fs=5 every window is clipped -> best score stays MAXSTAMP+1 -> (0,0)."""
    x, y, t, p = ramp(3, 3, 1e-3, 2e-3)
    out = OracleFlow(3, 3, 5, 1).process(x, y, t, p)
    assert np.all(out["vx"] == 0) and np.all(out["vy"] == 0)


def test_inlier_threshold_gates_the_flow():
    """inliers >= minEvtsOnPlane (vFlow.cpp:934): a 3x3 plane has at most 8
    inliers with Y > 0, so minEvtsOnPlane 9 kills every flow."""
    x, y, t, p = ramp(20, 20, 2e-3, 1e-3, t0=1000)
    ok = OracleFlow(20, 20, 3, 8).process(x, y, t, p)
    none = OracleFlow(20, 20, 3, 10).process(x, y, t, p)
    assert (ok["r_local"] > 0).sum() > 50
    assert (none["r_local"] > 0).sum() == 0


def test_pooling_single_flow_is_scale_zero():
    """One valid flow and nothing else recent: every scale's mean is the event's
    own flow, the first strict max is scale 0 (vFlow.cpp:1159-1166) and the
    global flow equals the local one (vFlow.cpp:1072-1075, 365-366)."""
    a, b = 2e-3, 1e-3
    x, y, t, p = ramp(40, 30, a, b)
    out = OracleFlow(30, 40, 3, 5).process(x, y, t, p)
    v = np.flatnonzero(out["r_local"] > 0)
    first = v[0]
    # the first valid event has no recent valid neighbour
    assert out["scale"][first] == 0
    assert out["r_true"][first] == pytest.approx(out["r_local"][first], rel=1e-12)
    assert out["theta_true"][first] == pytest.approx(out["theta_local"][first], abs=1e-12)


def test_kill_time_excludes_old_flows():
    """Only cells with |t_e - lastEventTime| < 500 us pool (vFlow.cpp:1002).  On a
    12 x 12 ramp with dt = 700 * (13 dx + dy) us every pair of pixels is >= 700 us
    apart, so no neighbour is ever recent: scale 0 always wins and RTrue == RLocal."""
    x, y, t, p = ramp(12, 12, 9.1e-3, 7e-4)
    out = OracleFlow(12, 12, 3, 5).process(x, y, t, p)
    v = out["r_local"] > 0
    assert v.sum() > 40
    np.testing.assert_allclose(out["r_true"][v], out["r_local"][v], rtol=1e-12)
    assert np.all(out["scale"][v] == 0)


def test_recent_neighbours_pool_and_pick_the_largest_mean():
    """A fast ramp (100 us per pixel): neighbours within 500 us pool; the scale
    with the largest mean length wins and the global vector is that scale's mean
    of L*(cos, sin)(theta) (vFlow.cpp:1005-1008, 1023-1075)."""
    x, y, t, p = ramp(60, 60, 1e-4, 6e-5)
    out = OracleFlow(60, 60, 3, 5).process(x, y, t, p)
    v = out["r_local"] > 0
    assert v.sum() > 1000
    assert np.any(out["scale"][v] > 0)
    # on a near-perfect plane all local flows agree, so the pooled flow does too
    inner = v & (x > 10) & (x < 50) & (y > 10) & (y < 50)
    np.testing.assert_allclose(out["r_true"][inner], out["r_local"][inner], rtol=2e-2)


def test_polarity_is_only_echoed():
    """Polarity never enters the computation."""
    x, y, t, p = ramp(25, 25, 1e-3, 1.5e-3)
    a = OracleFlow(25, 25, 3, 5).process(x, y, t, p)
    b = OracleFlow(25, 25, 3, 5).process(x, y, t, np.zeros_like(p))
    for c in ("r_true", "theta_true", "vx", "vy", "r_local", "theta_local", "scale"):
        np.testing.assert_array_equal(a[c], b[c])
    assert np.all(b["p"] == 0)


def test_parameter_normalisation():
    """filterSize < 5 -> 3, even -> odd - 1 (vFlow.cpp:32-33); more scales than
    maxWindow is rejected (spatialPool.at() would throw, vFlow.cpp:966,1025)."""
    x, y, t, p = ramp(30, 30, 2e-3, 1e-3)
    f4 = OracleFlow(30, 30, 4, 5).process(x, y, t, p)
    f3 = OracleFlow(30, 30, 3, 5).process(x, y, t, p)
    f6 = OracleFlow(30, 30, 6, 5).process(x, y, t, p)
    f5 = OracleFlow(30, 30, 5, 5).process(x, y, t, p)
    np.testing.assert_array_equal(f4["vx"], f3["vx"])
    np.testing.assert_array_equal(f6["vx"], f5["vx"])
    with pytest.raises(ValueError):
        OracleFlow(30, 30, 3, 5, window_jump=1, max_window=50)


def test_out_of_sensor_event_rejected():
    with pytest.raises(ValueError):
        OracleFlow(10, 10, 3, 5).process(np.array([10], np.int32), np.array([0], np.int32),
                                         np.array([0], np.uint32), np.array([1], np.int32))


def _bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def test_pool_given_reproduces_the_oracle_pooling():
    """farms_oracle_pool_given (the GPU pooling checker) fed the oracle's own
    local flows reproduces the oracle's RTrue / ThetaTrue / scale bit for bit:
    it is the same pooling (vFlow.cpp:952-1210), only the fit is skipped."""
    import farms
    from parity import gate

    ev = farms.synth_config(2, 30_000)
    x, y, t, p = ev.relative()
    ref = OracleFlow(320, 320, 5, 5).process(x, y, t, p)
    got = OracleFlow(320, 320, 5, 5).pool_given(x, y, t, gate(ref["vx"], ref["vy"]), ref["r_local"],
                                                ref["theta_local"])
    assert (ref["r_local"] > 0).sum() > 3000
    for c in ("r_true", "theta_true"):
        assert np.array_equal(_bits(got[c]), _bits(ref[c])), c
    assert np.array_equal(got["scale"], ref["scale"])


def test_serial_mode_semantics():
    """vFlowManager::run (vFlow.cpp:465-826): lastEventTime is written after the
    pooling (:790), so the pooled event's own cell is tested against the
    previous event at its pixel; the first line only stamps lastEventTime
    (:531-556).  A pixel that fires twice 100 us apart: in batch mode the own
    cell always contributes (|dt| = 0); in serial mode only the second event's
    own cell does (its previous stamp is 100 us old), the first event's own cell
    carries the t = 0 'never visited' stamp, 5000 us away."""
    a, b = 2e-3, 1e-3
    x, y, t, p = ramp(24, 24, a, b, t0=5000)
    i = int(np.flatnonzero((x == 12) & (y == 12))[0])
    # the same pixel again, 100 us later, appended at the end of the stream
    x2 = np.append(x, x[i]).astype(np.int32)
    y2 = np.append(y, y[i]).astype(np.int32)
    t2 = np.append(t, t.max() + 100).astype(np.uint32)
    p2 = np.ones(x2.size, np.int32)
    batch = OracleFlow(24, 24, 3, 3).process(x2, y2, t2, p2)
    ser = OracleFlow(24, 24, 3, 3, serial=True)
    s = ser.process(x2, y2, t2, p2)
    # the fit reads cSurf, written before the fit in both modes: identical local flows
    assert np.array_equal(_bits(batch["vx"]), _bits(s["vx"]))
    assert np.array_equal(_bits(batch["vy"]), _bits(s["vy"]))
    # an isolated event (no neighbour within 500 us) pools only itself in batch
    # mode and nothing in serial mode: scale 0 either way, global = its own flow
    # (vFlow.cpp:1085-1094) — so compare the events whose pooling differs
    diff = np.flatnonzero(_bits(batch["r_true"]) != _bits(s["r_true"]))
    assert diff.size > 0  # the own-cell stamp changes some poolings
    # first line of a serial run: lastEventTime[x][y] = absolute t, no SAE entry
    o = OracleFlow(24, 24, 3, 3, serial=True)
    o.serial_first(3, 4, 123456)
    one = o.process(np.array([3], np.int32), np.array([4], np.int32), np.array([0], np.uint32),
                    np.array([1], np.int32))
    assert one["r_local"][0] == 0  # a lone event: DET < 1


def test_eigen33_gemv_order_moves_bits_not_records():
    """The oracle's Eigen switch (farms_oracle_set_eigen): 3.3's GEMV adds each
    block of four columns of (A2*At)*Y as res + ((p0 + p3) + (p2 + p1)) on the
    rows of a and b, 3.4 sums sequentially (vFlow.cpp:1338).  Filtersize 3 takes
    Eigen's lazy product in both (n + 4 < 20): bitwise equal.  At filtersize 5
    the last ulp of many local flows moves, while validity, scale and the 1e-4
    bar hold (the full-size measurement: profiles/r05_eigen_sensitivity.log)."""
    import farms
    from parity import compare

    for fs, cfg in ((3, 1), (5, 2)):
        W, H = (128, 128) if cfg == 1 else (320, 320)
        x, y, t, p = farms.synth_config(cfg, 40_000).relative()
        a = OracleFlow(H, W, fs, 5, eigen=34).process(x, y, t, p)
        b = OracleFlow(H, W, fs, 5, eigen=33).process(x, y, t, p)
        same = np.array_equal(a["vx"].view(np.int64), b["vx"].view(np.int64))
        if fs == 3:
            assert same
        else:
            assert not same
            rep = compare(b, a)
            assert rep["ok"] and rep["valid_mismatch"] == 0 and rep["scale_mismatch"] == 0, rep
    with pytest.raises(ValueError):
        OracleFlow(320, 320, 5, 5, eigen=32)
