#!/usr/bin/env python3
"""The x-strip step of tests/test_multirank.py's HIP case run standalone
(diagnostic aid): WORLD ranks as processes on device 0, gloo collectives, each
rank dumping its Python stack every 20 s into gpurun_out/ranks_stack_<r>.txt
while it runs, and printing when its step is done.  Exit code 0 when the merged
owned records equal one whole-stream run bitwise.

usage: strips_hip_ranks.py [--world 2] [--split strips] [--per-rank 120000]
"""
import argparse
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rank_main(rank, world, port, split, per_rank, q):
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    f = open(os.path.join(out, f"ranks_stack_{rank}.txt"), "w")
    faulthandler.dump_traceback_later(20, repeat=True, file=f)
    import torch
    import torch.distributed as dist
    import farms
    import multirank
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sp = farms.synth_params(3)
    sp.n_events = per_rank * world
    hist = multirank.column_hist(sp, dist, rank)
    sh = multirank.make_share(sp, split, world, rank, 5, 50, hist)
    W, H = int(sp.width), int(sp.height)
    eng = farms.FlowManager(H, W, 5, 5, max_window=50, device=0, **multirank.engine_args(sh))
    st = multirank.Stepper(eng, sh, dist, torch.device("cuda", 0), torch.device("cpu"))
    t0 = time.time()
    st.step()
    print(f"rank {rank}: step done in {time.time() - t0:.2f} s", flush=True)
    merged = multirank.gather_owned(dist, st.owned_records(), sh.n_stream)
    if rank == 0:
        q.put(merged)
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--split", default="strips")
    ap.add_argument("--per-rank", type=int, default=120_000)
    a = ap.parse_args()
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(r, a.world, port, a.split, a.per_rank, q)) for r in range(a.world)]
    for p in procs:
        p.start()
    merged = q.get(timeout=100)
    for p in procs:
        p.join(timeout=30)
    import farms
    from parity import bitwise_equal
    sp = farms.synth_params(3)
    sp.n_events = a.per_rank * a.world
    x, y, t, p = farms.synth_generate(sp).relative()
    with farms.FlowManager(720, 1280, 5, 5) as fm:
        whole = fm.process(x, y, t, p)
    import numpy as np
    sc = np.asarray(merged["scale"])
    bad = sc[sc < 0]
    if len(bad):  # a FARMS_POOL2_CHECK build: -(1000 + bits of the load sites out of range)
        codes, counts = np.unique(bad, return_counts=True)
        print("flagged events", len(bad), dict(zip((-codes - 1000).tolist(), counts.tolist())), flush=True)
    ok = bitwise_equal(merged, whole)
    print("bitwise", ok, flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
