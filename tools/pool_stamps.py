#!/usr/bin/env python3
"""Where a valid event's k_pool wave spends its cycles (diagnostic build).

Runs one device-resident step of a BASELINE config on the stamps build
(`make -C aperture-robust-multiscale-optical-flow_amd variant NAME=stamps
DEFS=-DFARMS_POOL_STAMPS`), then prints the shader-clock cycles per valid event
of each k_pool phase: prologue (descriptor), row setup, the candidate pass
(fold included) and the fold alone, the finish; plus steps and fold groups per
valid event.  FARMS_SERIALIZE=1 in the environment gives the kernel alone.

usage: pool_stamps.py [--config 3] [--lib build/libfarms_hip_stamps.so]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--lib", default="build/libfarms_hip_stamps.so")
    ap.add_argument("--events", type=int, default=0)
    a = ap.parse_args()
    os.environ["FARMS_HIP_LIB"] = a.lib
    sys.path.insert(0, PKG)
    import numpy as np
    import torch
    import farms

    cfg = a.config
    W, H = (320, 320) if cfg == 2 else (1280, 720)
    fs = {2: 5, 3: 5, 4: 7, 5: 7}[cfg]
    jump = 25 if cfg == 5 else 5
    n = a.events or {4: 50_000_000, 5: 50_000_000}.get(cfg, 0) or None
    ev = farms.synth_config(cfg, n)
    x, y, t, p = ev.relative()
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(v).to(dev) for v in (x, y, t.view(np.int32), p)]
    o = {c: torch.empty(len(x), dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    lib = farms.load_hip_library()
    fn = lib.farms_debug_pool_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 8)()
    fm = farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=50)
    for i in range(2):
        fm.reset()
        fn(buf)  # clear
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fm.process_device(*d, o)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
    fn(buf)
    v = list(buf)
    nv = max(v[5], 1)
    names = ["prologue", "row_setup", "cand_pass_incl_fold", "fold", "finish"]
    rep = {"config": cfg, "events": len(x), "ms_step": round(ms, 2), "valid_events": v[5],
           "serialized": os.environ.get("FARMS_SERIALIZE", "0") == "1",
           "cycles_per_valid_event": {k: round(v[i] / nv, 1) for i, k in enumerate(names)},
           "steps_per_valid_event": round(v[6] / nv, 2), "fold_groups_per_valid_event": round(v[7] / nv, 2)}
    c = rep["cycles_per_valid_event"]
    rep["cycles_per_valid_event"]["total"] = round(c["prologue"] + c["row_setup"] + c["cand_pass_incl_fold"]
                                                   + c["finish"], 1)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
