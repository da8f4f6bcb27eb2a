#!/usr/bin/env python3
"""How much the Eigen version alone moves the reference's records (CPU only).

The reference pins no Eigen version (CMakeLists.txt:19 `find_package(Eigen3
REQUIRED)`, README.md:19 `apt-get install libeigen3-dev`): Ubuntu 18.04 / 20.04
ship 3.3.x, 22.04 ships 3.4.0.  The only Eigen call on the path whose result
depends on the version is temp = A2*At*Y (vFlow.cpp:1338): 3.4 sums every row
of the GEMV sequentially, 3.3 adds blocks of four columns as a packet tree on
the rows of a and b (oracle/farms_oracle.c, eigen33_gemv_packet_row).  This
runs the oracle in both modes (glibc libm, the reference's) on BASELINE config
2 in full and on the first 1.5M events of config 3 (plus config 4's fs 7 and
config 1's fs 3 heads) and reports, per stream, the events whose local flow
differs bitwise, the validity and scale mismatches and the largest angle and
radius differences — the flip rate the Eigen version alone causes.

usage: python tools/eigen_sensitivity.py [--c3-events N] [--quick]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import farms  # noqa: E402
from oracle import OracleFlow  # noqa: E402
from parity import compare, wrap_diff, rel_err  # noqa: E402

SENSOR = {1: (128, 128), 2: (320, 320), 3: (1280, 720), 4: (1280, 720)}
FS = {1: 3, 2: 5, 3: 5, 4: 7}


def run_both(cfg, n):
    W, H = SENSOR[cfg]
    ev = farms.synth_config(cfg, n)
    x, y, t, p = ev.relative()
    out = {}

    def run(ver):
        out[ver] = OracleFlow(H, W, FS[cfg], 5, 5, 50, eigen=ver).process(x, y, t, p)

    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(v,)) for v in (34, 33)]
    for a in th:
        a.start()
    for a in th:
        a.join()
    dt = time.perf_counter() - t0
    a, b = out[34], out[33]
    va, vb = a["r_local"] > 0, b["r_local"] > 0
    local_bits = (a["vx"].view(np.int64) != b["vx"].view(np.int64)) | (a["vy"].view(np.int64) != b["vy"].view(np.int64))
    both = va & vb
    rep = compare(b, a)
    res = {
        "config": cfg, "events": int(len(x)), "filtersize": FS[cfg], "sensor": f"{W}x{H}", "seconds": round(dt, 1),
        "valid_eigen34": int(va.sum()),
        "local_flow_bitwise_diff_events": int(local_bits.sum()),
        "local_flow_bitwise_diff_rate": float(local_bits.mean()) if len(x) else 0.0,
        "valid_mismatch": int((va != vb).sum()),
        "scale_mismatch": int((both & (a["scale"] != b["scale"])).sum()),
        "max_dtheta_local_rad": float(wrap_diff(a["theta_local"][both], b["theta_local"][both]).max(initial=0.0)),
        "max_dtheta_true_rad": float(wrap_diff(a["theta_true"][both], b["theta_true"][both]).max(initial=0.0)),
        "max_rel_r_local": float(rel_err(b["r_local"][both], a["r_local"][both]).max(initial=0.0)),
        "max_rel_r_true": float(rel_err(b["r_true"][both], a["r_true"][both]).max(initial=0.0)),
        "records_bitwise_equal": bool(not local_bits.any() and all(
            np.array_equal(a[c].view(np.int64) if a[c].dtype == np.float64 else a[c],
                           b[c].view(np.int64) if b[c].dtype == np.float64 else b[c]) for c in a)),
        "tolerance_bar_ok": bool(rep["ok"]),
    }
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c3-events", type=int, default=1_500_000)
    ap.add_argument("--quick", action="store_true", help="short heads only (a smoke run)")
    a = ap.parse_args()
    runs = [(2, 100_000), (3, 100_000)] if a.quick else [(1, None), (2, None), (3, a.c3_events), (4, 500_000)]
    for cfg, n in runs:
        print(json.dumps(run_both(cfg, n)), flush=True)


if __name__ == "__main__":
    main()
