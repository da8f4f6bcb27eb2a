#!/usr/bin/env python3
"""Host-array path (farms_process, pinned host arrays) against the device path
on one configuration (diagnostic).

usage: host_probe.py --config C [--steps K] [--trace]
Prints the device-resident step and the host path's step (best / mean, ms);
--trace runs one more host call with FARMS_HOST_TRACE=1 (the engine's host
timestamps on stderr).  Env knobs of the engine (FARMS_SUBBATCHES,
FARMS_SUB_HEAD, ...) apply to every host call."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--host-only", action="store_true", help="skip the device-resident timing (profiler runs)")
    ap.add_argument("--dma-load", type=int, default=0, metavar="DIR",
                    help="device path under background copies on a torch stream: 1 D2H, 2 H2D, 3 both")
    a = ap.parse_args()
    import numpy as np
    import torch
    import farms

    cfg = a.config
    W, H = (320, 320) if cfg == 2 else (1280, 720)
    fs = {2: 5, 3: 5, 4: 7, 5: 7}[cfg]
    jump = 25 if cfg == 5 else 5
    n = {4: 50_000_000, 5: 50_000_000}.get(cfg, 0) or None
    ev = farms.synth_config(cfg, n)
    x, y, t, p = ev.relative()
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(v).to(dev) for v in (x, y, t.view(np.int32), p)]
    o = {c: torch.empty(len(x), dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
         for c in farms.COLUMNS[4:]}
    own = [farms.pinned(v) for v in (x, y, t, p)]
    rec = farms.Records(len(x), pinned=True)
    res = {"config": cfg, "events": len(x), "env": {k: v for k, v in os.environ.items() if k.startswith("FARMS_")}}
    # (FARMS_AB_POOL_BATCH / FARMS_AB_POOL_CHUNK: handle parameters, as tools/lib_ab.py)
    kw = {k: int(os.environ[e]) for k, e in (("pool_batch", "FARMS_AB_POOL_BATCH"), ("pool_chunk", "FARMS_AB_POOL_CHUNK"))
          if os.environ.get(e)}
    with farms.FlowManager(H, W, fs, 5, window_jump=jump, max_window=50, **kw) as fm:
        def timed(fn):
            ts = []
            for i in range(a.steps + 1):
                fm.reset()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                if i:
                    ts.append((time.perf_counter() - t0) * 1e3)
            return {"ms_best": round(min(ts), 3), "ms_mean": round(sum(ts) / len(ts), 3)}

        if a.dma_load:  # the device path with PCIe traffic beside it (interference probe)
            import threading
            stop = threading.Event()
            big = torch.empty(64 << 20, dtype=torch.float32, device=dev)
            hb = torch.empty(64 << 20, dtype=torch.float32, pin_memory=True)
            hb2 = torch.empty(64 << 20, dtype=torch.float32, pin_memory=True)
            big2 = torch.empty(64 << 20, dtype=torch.float32, device=dev)
            st = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

            def loop(k):
                with torch.cuda.stream(st[k]):
                    while not stop.is_set():
                        for _ in range(4):
                            if k == 0:
                                hb.copy_(big, non_blocking=True)
                            else:
                                big2.copy_(hb2, non_blocking=True)
                        st[k].synchronize()

            th = [threading.Thread(target=loop, args=(k,)) for k in (0, 1) if a.dma_load & (1 << k)]
            for x_ in th:
                x_.start()
            time.sleep(0.2)
            res["device_under_dma"] = timed(lambda: fm.process_device(*d, o))
            stop.set()
            for x_ in th:
                x_.join()
        if not a.host_only:
            res["device"] = timed(lambda: fm.process_device(*d, o))
        res["host"] = timed(lambda: fm.process(*[v[0] for v in own], out=rec))
        if not a.host_only:
            res["host_over_device"] = round(res["host"]["ms_mean"] / res["device"]["ms_mean"], 3)
        print(json.dumps(res), flush=True)
        if a.trace:
            os.environ["FARMS_HOST_TRACE"] = "1"
            fm.reset()
            fm.process(*[v[0] for v in own], out=rec)
            os.environ.pop("FARMS_HOST_TRACE")


if __name__ == "__main__":
    main()
