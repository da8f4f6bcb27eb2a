#!/usr/bin/env python3
"""The smallest failing case of round 5's paired-pooling fault (diagnostic
aid): a whole-sensor C2 stream through farms_fit_device + farms_pool_device
(the two-phase calls) against one farms_process_device call.  On a
FARMS_POOL2_DEBUG build it prints the recorded anomaly counters.

usage: pool_phase2_repro.py [--events 60000] [--pairs 1]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=60_000)
    ap.add_argument("--order", default="whole-first", choices=["whole-first", "phase-first"])
    ap.add_argument("--strip-first", action="store_true",
                    help="first run tests/test_strips.py's import_halo guard sequence on a middle-strip handle "
                         "(a time-reversed stream, then the stream), as the failing pytest order did")
    a = ap.parse_args()
    import numpy as np
    import torch
    import farms
    if a.strip_first:
        sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
        import strips
        W, H = 1280, 720
        ev3 = farms.synth_config(3, 200_000)
        x3, y3, t3, p3 = ev3.relative()
        s = strips.plan(x3, W, H, 3, 5, 50)[1]
        m = strips.region_mask(x3, s)
        dev = torch.device("cuda", 0)
        d3 = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (x3[m], y3[m], t3[m].view(np.int32), p3[m])]
        with farms.FlowManager(H, W, 5, 5, region=(s.reg_lo, s.reg_hi), owned=(s.own_lo, s.own_hi),
                               import_halo=True) as fm:
            for garbage in (False, True):
                if garbage:
                    fm.reset()
                    g = [torch.flip(v, [0]).contiguous() for v in d3]
                    fm.fit_device(*g, {c: torch.zeros(len(g[0]), dtype=torch.int32 if c == "scale" else torch.float64,
                                                      device=dev) for c in farms.COLUMNS[4:]})
                    fm.pool_device()
                fm.reset()
                o3 = {c: torch.zeros(int(m.sum()), dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
                      for c in farms.COLUMNS[4:]}
                fm.fit_device(*d3, o3)
                fm.pool_device()
            torch.cuda.synchronize()
        print("strip guard sequence done", flush=True)

    ev = farms.synth_config(2, a.events)
    x, y, t, p = ev.relative()
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (x, y, t.view(np.int32), p)]

    def outs():
        return {c: torch.zeros(len(x), dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
                for c in farms.COLUMNS[4:]}
    with farms.FlowManager(320, 320, 5, 5) as fm:
        dbgf = getattr(fm._lib, "farms_debug_pool2", None)
        whole, o = outs(), outs()
        if a.order == "whole-first":
            fm.process_device(*d, whole)
            fm.reset()
        fm.fit_device(*d, o)
        print("fit_device enqueued", flush=True)
        fm.pool_device()
        torch.cuda.synchronize()
        print("pool_device done", flush=True)
        if dbgf is not None:
            buf = (ctypes.c_ulonglong * 32)()
            dbgf(buf)
            print("pool2 debug:", [int(buf[i]) for i in range(32)], flush=True)
        if a.order == "phase-first":
            fm.reset()
            fm.process_device(*d, whole)
    same = all(np.array_equal(whole[c].cpu().numpy(), o[c].cpu().numpy()) for c in farms.COLUMNS[4:])
    print("bitwise", same, flush=True)
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
