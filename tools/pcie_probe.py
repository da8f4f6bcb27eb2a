"""PCIe rates of the box (pinned host <-> HBM), and one traced farms_process
call on the bench stream (FARMS_HOST_TRACE=1): a diagnostic for the host path."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
import farms  # noqa: E402

n = 1 << 28
a = torch.empty(n, dtype=torch.float32).pin_memory()
b = torch.empty(n, dtype=torch.float32).pin_memory()
d = torch.empty(n, dtype=torch.float32, device="cuda")
e = torch.empty(n, dtype=torch.float32, device="cuda")
for _ in range(2):
    d.copy_(a, non_blocking=True)
    a.copy_(d, non_blocking=True)
torch.cuda.synchronize()
for what, fn in [("H2D", lambda: d.copy_(a, non_blocking=True)), ("D2H", lambda: a.copy_(d, non_blocking=True))]:
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    print(f"{what} 1 GiB: {1.073741824 / (time.perf_counter() - t0):.1f} GB/s", flush=True)
s2 = torch.cuda.Stream()
t0 = time.perf_counter()
d.copy_(a, non_blocking=True)
with torch.cuda.stream(s2):
    b.copy_(e, non_blocking=True)
torch.cuda.synchronize()
print(f"H2D + D2H concurrent 2 GiB: {2 * 1.073741824 / (time.perf_counter() - t0):.1f} GB/s", flush=True)
del a, b, d, e
ev = farms.synth_config(3)
x, y, t, p = ev.relative()
fm = farms.FlowManager(720, 1280, 5, 5)
own = [farms.pinned(v) for v in (x, y, t, p)]
rec = farms.Records(len(x), pinned=True)
for env in ({}, {"FARMS_ECHO_DMA": "0"}, {"FARMS_SUBBATCHES": "1"}, {"FARMS_SUBBATCHES": "16"}):
    os.environ.pop("FARMS_ECHO_DMA", None)
    os.environ.pop("FARMS_SUBBATCHES", None)
    os.environ.update(env)
    for trace in ("0", "1"):
        os.environ["FARMS_HOST_TRACE"] = trace
        fm.reset()
        t0 = time.perf_counter()
        fm.process(*[o[0] for o in own], out=rec)
        print(f"pinned farms_process {env} trace={trace}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
