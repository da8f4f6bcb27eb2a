"""CPU-baseline legs BASELINE.md §2 plans beside bench.py's own (C3, first 1.5M
events, -O2): the oracle (single-thread C restatement of vFlow.cpp:223-414) over
the full C1 and C2 streams at -O2, and the C3 head at -O0 (the reference's CMake
default: no build type).  Timed region = the oracle's process call only (the
reference's vFlow.cpp:214 -> :416).  One JSON line per leg, flushed as it ends.

Each leg runs in a child process so that the -O0 build is the one loaded
(FARMS_ORACLE_LIB).  Usage: python tools/cpu_baseline_configs.py [--c3-o0 N]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SENSOR = {1: (128, 128), 2: (320, 320), 3: (1280, 720), 4: (1280, 720), 5: (1280, 720)}
FILTER = {1: 3, 2: 5, 3: 5, 4: 7, 5: 7}


def leg(cfg: int, n: int | None, opt: str) -> dict:
    sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import farms
    from oracle import OracleFlow

    W, H = SENSOR[cfg]
    jump, maxw = (25, 50) if cfg == 5 else (5, 50)
    ev = farms.synth_config(cfg, n)
    x, y, t, p = ev.relative()
    of = OracleFlow(H, W, FILTER[cfg], 5, jump, maxw)
    t0 = time.perf_counter()
    ref = of.process(x, y, t, p)
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), cpu)
    except OSError:
        pass
    return {"config": cfg, "events": len(x), "stream": "full" if n is None else f"first {n}", "opt": opt,
            "seconds": round(dt, 3), "Mevents_per_s": len(x) / dt / 1e6, "cores": 1,
            "kind": "port", "cpu_model": cpu}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", nargs=3, metavar=("CFG", "N", "OPT"))
    ap.add_argument("--c3-o0", type=int, default=500_000, help="C3 head events of the -O0 leg")
    a = ap.parse_args()
    if a.leg:
        cfg, n, opt = int(a.leg[0]), int(a.leg[1]), a.leg[2]
        print(json.dumps(leg(cfg, n if n > 0 else None, opt)), flush=True)
        return 0
    o0 = os.path.join(ROOT, "oracle", "build", "libfarms_oracle_O0.so")
    for cfg, n, opt in ((1, 0, "O2"), (2, 0, "O2"), (3, a.c3_o0, "O0"), (3, a.c3_o0, "O2")):
        env = dict(os.environ)
        if opt == "O0":
            env["FARMS_ORACLE_LIB"] = o0
        rc = subprocess.run([sys.executable, "-u", __file__, "--leg", str(cfg), str(n), opt], env=env).returncode
        if rc:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
