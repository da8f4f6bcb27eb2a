#!/usr/bin/env python3
"""Device timeline of the last host-path call (diagnostic): kernels and memory
copies from one rocprofv3 run with --kernel-trace --memory-copy-trace (csv),
relative to the end of the call's farms_reset fill.

usage: host_timeline.py KERNEL_TRACE.csv MEMORY_COPY_TRACE.csv [--all]
Without --all, the fit / pooling kernels and the per-sub-batch preps are
listed, and runs of consecutive copies are merged into one line."""
import csv
import re
import sys


def main():
    kt = []
    for r in csv.DictReader(open(sys.argv[1])):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        kt.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:20],
                   r.get("Queue_Id", "?")))
    mc = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           "H2D" if r["Direction"].startswith("HOST") else "D2H" if r["Direction"].startswith("DEVICE_TO_HOST") else
           r["Direction"][:8], "dma") for r in csv.DictReader(open(sys.argv[2]))]
    kt.sort()
    t0 = [k for k in kt if k[2] == "k_fill"][-1][1]
    ev = sorted([k for k in kt if k[0] >= t0] + [m for m in mc if m[0] >= t0])
    keep = ("k_prep", "k_fit_quad", "k_pool2", "k_pool", "k_cand", "k_true_polar", "k_flow")
    run = None
    for s, e, n, q in ev:
        if q == "dma" and "--all" not in sys.argv:
            if run and run[2] == n and s - run[1] < 20_000:
                run = (run[0], e, n, run[3] + 1)
                continue
            if run:
                print(f"{(run[0] - t0) / 1e3:9.1f} {(run[1] - t0) / 1e3:9.1f}  dma {run[2]} x{run[3]}")
            run = (s, e, n, 1)
            continue
        if "--all" in sys.argv or n in keep:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  q{q:>3} {n}")
    if run:
        print(f"{(run[0] - t0) / 1e3:9.1f} {(run[1] - t0) / 1e3:9.1f}  dma {run[2]} x{run[3]}")


if __name__ == "__main__":
    main()
