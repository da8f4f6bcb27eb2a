"""Record comparison used by the parity tests.

Bar (north_star): x/y/t/p and the validity flag bit-exact;
RTrue/RLocal relative error <= 1e-4; ThetaTrue/ThetaLocal wrap-aware
|dtheta| <= 1e-4 rad.

The scale column is an argmax over per-scale mean lengths, so an ulp anywhere
in the summed lengths can flip it on a near tie.  Two checks pin it:
  * pooling_check(): the oracle's pooling run on the GPU's own local flows
    (oracle/farms_oracle.h, farms_oracle_pool_given).  Same inputs, same
    summation order (vFlow.cpp:998-1021) -> the scale column must be identical.
  * compare(): against the full oracle.  The only remaining difference is the
    local flow itself, whose atan2/cos/sin are correctly rounded on the GPU
    and come from glibc in the oracle (glibc misrounds a small fraction of
    arguments); `local_ulp_events` counts the events whose Vx/Vy differ
    bitwise, and a scale mismatch is accepted only for an event whose pooling
    window can hold such an event: an earlier (or the same) event within the
    kill time (vFlow.cpp:1002) and within the window's columns, x - M to
    x + M + 2 (the W-1 clip's alias column, vFlow.cpp:1000).  Every other scale
    mismatch fails the bar.
"""
from __future__ import annotations

import numpy as np

REL_TOL = 1e-4
ANG_TOL = 1e-4


def _get(rec, name):
    return rec[name] if isinstance(rec, dict) else getattr(rec, name)


def wrap_diff(a, b):
    d = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)) % (2 * np.pi)
    return np.minimum(d, 2 * np.pi - d)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.maximum(np.abs(b), 1e-300)
    err = np.abs(a - b) / den
    both_zero = (a == 0) & (b == 0)
    both_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    both_nan = np.isnan(a) & np.isnan(b)
    err[both_zero | both_inf | both_nan] = 0.0
    return err


KILL_US = 500  # vFlow.cpp:961


def _scale_unexplained(gpu, ref, both, local_diff, max_window) -> int:
    """Scale mismatches with no bitwise-different local flow that the event's
    pooling can read: none earlier (or itself) within KILL_US and columns
    [x - M, x + M + 2]."""
    sg, sr = np.asarray(_get(gpu, "scale")), np.asarray(_get(ref, "scale"))
    bad = np.flatnonzero(both & (sg != sr))
    if bad.size == 0:
        return 0
    x = np.asarray(_get(ref, "x"), np.int64)
    t = np.asarray(_get(ref, "t")).astype(np.uint32).astype(np.int64)
    dif = np.flatnonzero(local_diff)
    n_bad = 0
    for e in bad:
        d = dif[dif <= e]
        near = (np.abs(t[d] - t[e]) < KILL_US) & (x[d] >= x[e] - max_window) & (x[d] <= x[e] + max_window + 2)
        n_bad += int(not near.any())
    return n_bad


def compare(gpu, ref, max_window: int = 50) -> dict:
    """Return a report dict; report['ok'] is the pass/fail of the bar."""
    rep = {}
    n = len(_get(ref, "x"))
    rep["n"] = n
    for c in ("x", "y", "t", "p"):
        rep[f"{c}_mismatch"] = int(np.count_nonzero(_get(gpu, c) != _get(ref, c)))
    vg = _get(gpu, "r_local") > 0
    vr = _get(ref, "r_local") > 0
    rep["valid_ref"] = int(vr.sum())
    rep["valid_mismatch"] = int(np.count_nonzero(vg != vr))
    both = vg & vr
    for c in ("r_true", "r_local"):
        e = rel_err(_get(gpu, c)[both], _get(ref, c)[both])
        rep[f"{c}_max_rel"] = float(e.max()) if e.size else 0.0
    for c in ("theta_true", "theta_local"):
        e = wrap_diff(_get(gpu, c)[both], _get(ref, c)[both])
        e[np.isnan(_get(gpu, c)[both]) & np.isnan(_get(ref, c)[both])] = 0
        rep[f"{c}_max_abs"] = float(np.nanmax(e)) if e.size else 0.0
    # raw local flow vector, printed for invalid events too (vFlow.cpp:394-395).
    # Error relative to |v|: near theta = +-pi/2 one component is speed*cos(~pi/2)
    # ~ 1e-16*speed, where a 1-ulp change of the angle is a 100% change of that
    # component but 1e-16 of the vector.
    gx, gy = np.asarray(_get(gpu, "vx"), np.float64), np.asarray(_get(gpu, "vy"), np.float64)
    rx, ry = np.asarray(_get(ref, "vx"), np.float64), np.asarray(_get(ref, "vy"), np.float64)
    fin = np.isfinite(rx) & np.isfinite(ry)
    same_nonfinite = (~fin) & (((gx == rx) | (np.isnan(gx) & np.isnan(rx))) & ((gy == ry) | (np.isnan(gy) & np.isnan(ry))))
    with np.errstate(invalid="ignore", over="ignore"):
        norm = np.hypot(rx, ry)
        err = np.where(norm > 0, np.hypot(gx - rx, gy - ry) / np.where(norm > 0, norm, 1.0), np.hypot(gx, gy))
    err = np.where(fin, err, np.where(same_nonfinite, 0.0, np.inf))
    rep["v_max_rel"] = float(err.max()) if err.size else 0.0
    rep["scale_mismatch"] = int(np.count_nonzero(_get(gpu, "scale")[both] != _get(ref, "scale")[both]))
    # events whose local flow differs bitwise (libm ulps: correctly rounded vs glibc atan2/cos/sin)
    local_diff = (gx.view(np.int64) != rx.view(np.int64)) | (gy.view(np.int64) != ry.view(np.int64))
    rep["local_ulp_events"] = int(np.count_nonzero(local_diff))
    rep["scale_mismatch_unexplained"] = _scale_unexplained(gpu, ref, both, local_diff, max_window)
    ok = all(rep[f"{c}_mismatch"] == 0 for c in ("x", "y", "t", "p")) and rep["valid_mismatch"] == 0
    ok = ok and rep["r_true_max_rel"] <= REL_TOL and rep["r_local_max_rel"] <= REL_TOL
    ok = ok and rep["theta_true_max_abs"] <= ANG_TOL and rep["theta_local_max_abs"] <= ANG_TOL
    ok = ok and rep["v_max_rel"] <= REL_TOL
    ok = ok and rep["scale_mismatch_unexplained"] == 0
    rep["ok"] = bool(ok)
    return rep


def gate(vx, vy):
    """Validity gate of vFlow.cpp:315 on the raw local flow."""
    vx = np.asarray(vx, np.float64)
    vy = np.asarray(vy, np.float64)
    return ~np.isnan(vx) & ~np.isnan(vy) & (vx != 0) & (vy != 0)


def pooling_check(gpu, height, width, window_jump=5, max_window=50, serial=False, first=None) -> dict:
    """Run the oracle's pooling (vFlow.cpp:952-1210) on the GPU's own local flows
    and compare: the scale column must match exactly, RTrue / ThetaTrue within
    ocml-vs-glibc cos/sin ulps.  `first` = (x, y, t_abs) of a serial run's first
    line (vFlow.cpp:531-556)."""
    from oracle import OracleFlow

    o = OracleFlow(height, width, 3, 5, window_jump, max_window, serial=serial)
    if first is not None:
        o.serial_first(*first)
    valid = gate(_get(gpu, "vx"), _get(gpu, "vy"))
    r = o.pool_given(_get(gpu, "x"), _get(gpu, "y"), np.asarray(_get(gpu, "t")).view(np.uint32), valid,
                     _get(gpu, "r_local"), _get(gpu, "theta_local"))
    o.close()
    rep = {"pooled": int(valid.sum())}
    rep["scale_mismatch"] = int(np.count_nonzero(np.asarray(_get(gpu, "scale"))[valid] != r["scale"][valid]))
    e = rel_err(np.asarray(_get(gpu, "r_true"))[valid], r["r_true"][valid])
    rep["r_true_max_rel"] = float(e.max()) if e.size else 0.0
    d = wrap_diff(np.asarray(_get(gpu, "theta_true"))[valid], r["theta_true"][valid])
    rep["theta_true_max_abs"] = float(np.nanmax(d)) if d.size else 0.0
    rep["ok"] = bool(rep["scale_mismatch"] == 0 and rep["r_true_max_rel"] <= REL_TOL and
                     rep["theta_true_max_abs"] <= ANG_TOL)
    return rep


def multi_report(merged, ref, ref_cr, boundaries, max_window: int = 50) -> dict:
    """N > 1 parity block: the owned records of every rank, merged by stream
    index, against the oracle run on the whole parity stream (glibc: the bar
    of compare(); the correctly rounded libm: every column bitwise), and the
    same per rank boundary (multirank.boundary_events: the events whose
    records read what crosses it)."""
    rep = compare(merged, ref, max_window)
    out = {"events_compared": rep["n"], "valid_events": rep["valid_ref"], "valid_mismatch": rep["valid_mismatch"],
           "scale_mismatch": rep["scale_mismatch"], "max_dtheta_true_rad": rep["theta_true_max_abs"],
           "max_rel_r_true": rep["r_true_max_rel"], "bitwise_vs_cr_oracle": bitwise_equal(merged, ref_cr)}
    per = []
    for name, idx in boundaries:
        sub = lambda d: {c: np.asarray(_get(d, c))[idx] for c in _COLS}  # noqa: E731
        g, r = sub(merged), sub(ref)
        vg, vr = np.asarray(g["r_local"]) > 0, np.asarray(r["r_local"]) > 0
        both = vg & vr
        per.append({"boundary": name, "events": int(len(idx)), "valid_events": int(vr.sum()),
                    "valid_mismatch": int(np.count_nonzero(vg != vr)),
                    "scale_mismatch": int(np.count_nonzero(np.asarray(g["scale"])[both] != np.asarray(r["scale"])[both])),
                    "bitwise_vs_cr_oracle": bitwise_equal(g, sub(ref_cr))})
    out["boundaries"] = per
    out["ok"] = bool(rep["ok"] and out["bitwise_vs_cr_oracle"] and all(b["events"] > 0 for b in per))
    return out


_COLS = ("x", "y", "t", "p", "r_true", "theta_true", "vx", "vy", "r_local", "theta_local", "scale")


def bitwise_equal(a, b) -> bool:
    cols = ("x", "y", "t", "p", "r_true", "theta_true", "vx", "vy", "r_local", "theta_local", "scale")
    for c in cols:
        u, v = np.asarray(_get(a, c)), np.asarray(_get(b, c))
        if u.dtype.kind == "f":
            if not np.array_equal(u.view(np.int64), v.view(np.int64)):
                return False
        elif not np.array_equal(u, v):
            return False
    return True
