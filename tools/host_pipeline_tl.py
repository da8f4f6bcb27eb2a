#!/usr/bin/env python3
"""Host-path pipeline timeline (diagnostic).

run:     python3 tools/host_pipeline_tl.py run            -- two pinned farms_process calls on the C3 stream
analyse: python3 tools/host_pipeline_tl.py <kernel_trace.csv> [n_sub]
  per sub-batch of the last call (a sub-batch starts at a k_prep): when its prep, first / last fit, first chain
  and first / last pooling launch ran, relative to the call's first k_prep (ms)."""
import csv
import os
import re
import sys

if sys.argv[1] == "run":
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
    import farms  # noqa: E402
    import numpy as np  # noqa: E402
    import torch  # noqa: E402,F401

    if os.environ.get("TORCH_WARM") == "1":  # a torch stream in use beside the engine's (as in bench.py)
        a = torch.ones(1 << 20, device="cuda") * 2
        torch.cuda.synchronize()
    ev = farms.synth_config(3)
    x, y, t, p = ev.relative()
    own = [farms.pinned(v) for v in (x, y, t, p)]
    rec = farms.Records(len(x), pinned=True)
    with farms.FlowManager(720, 1280, 5, 5) as fm:
        if os.environ.get("DEVICE_FIRST") == "1":  # a device-resident call first, as bench.py runs them
            dev = torch.device("cuda", 0)
            nd = int(os.environ.get("DEVICE_N", len(x)))
            d = [torch.from_numpy(a[:nd]).to(dev) for a in (x, y, t.view(np.int32), p)]
            o = {c: torch.empty(nd, dtype=torch.int32 if c == "scale" else torch.float64, device=dev)
                 for c in farms.COLUMNS[4:]}
            if os.environ.get("DEVICE_OTHER_HANDLE") == "1":
                with farms.FlowManager(720, 1280, 5, 5) as fm2:
                    fm2.process_device(*d, o)
            else:
                fm.process_device(*d, o)
            torch.cuda.synchronize()
            if os.environ.get("DEVICE_FREE") == "1":
                del d, o
                torch.cuda.empty_cache()
            fm.reset()
        for _ in range(2):
            fm.reset()
            fm.process(*[o[0] for o in own], out=rec)
    sys.exit(0)

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:24]))
rows.sort()
nsub = int(sys.argv[2]) if len(sys.argv) > 2 else 8
preps = [i for i, r in enumerate(rows) if r[2] == "k_prep"][-nsub:]
t0 = rows[preps[0]][0]
ms = lambda v: (v - t0) / 1e6  # noqa: E731
bounds = preps + [len(rows)]
# kernels belong to the sub-batch whose prep came last before their *enqueue*; launches of a sub-batch's
# sweeps interleave with the next one's, so attribute by kernel type order within the stream instead:
fits = [r for r in rows[preps[0]:] if r[2].startswith("k_fit_quad")]
pools = [r for r in rows[preps[0]:] if r[2].startswith("k_pool") and r[2] != "k_pool_desc"]
chains = [r for r in rows[preps[0]:] if r[2] == "k_chain"]
print(f"call: {len(fits)} fit, {len(chains)} chain, {len(pools)} pool launches; "
      f"span {ms(max(r[1] for r in rows[preps[0]:])):.2f} ms")
for b in range(nsub):
    p = rows[preps[b]]
    nxt = rows[preps[b + 1]][0] if b + 1 < nsub else None
    f_b = [r for r in fits if r[0] >= p[0] and (nxt is None or r[0] < nxt)]
    print(f"sub {b}: prep {ms(p[0]):8.2f}  fits {len(f_b):4d} {ms(f_b[0][0]) if f_b else -1:8.2f}"
          f" .. {ms(f_b[-1][1]) if f_b else -1:8.2f}")
k = max(1, len(pools) // (2 * nsub))
for i in range(0, len(pools), k):
    r = pools[i]
    c = [x for x in chains if x[1] <= r[0]]
    print(f"  pool {i:4d}: {ms(r[0]):8.2f} .. {ms(r[1]):8.2f}   (last chain before it ended {ms(c[-1][1]) if c else -1:8.2f})")
