"""Spatial x-strips for multi-GPU runs.

Rank r owns the events of columns [own_lo, own_hi); strips are balanced by
event count (column histogram quantiles) over the whole stream.  Two things
cross a strip border:

  * the local fit of an event reads SAE columns +-2*fRad (vFlow.cpp:870-883);
  * the pooling of an event reads flow cells of columns [x-M, x+M] and, through
    the reference's x-major j-clip at W-1 (vFlow.cpp:1000/1113), the first
    rows of up to floor(min(H-1+M, W-1) / H) further columns.

Exchange mode (default, `import_halo`): the rank stores its owned columns
widened by the pooling halo (left M, right M + a, which also covers the SAE
halo), fits only its owned events, and receives the local flows of its halo
events from their owners — one exchange per step, between the fit sweep and
the pooling sweep (`exchange_lists`; grouped send/recv with the ranks whose
strips the halo reaches, over RCCL in bench.py).  Recompute mode stores the
owned columns widened by the pooling halo plus the SAE halo and fits every
stored event itself (no collective, ~1.7x the fits at 8 strips).

Either way the owned records are bitwise those of a whole-sensor run: the fit
is local, and the pooling sum order depends only on the contributor list.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def normalised_filter(fs: int) -> int:
    """vFlow.cpp:32-33."""
    if fs < 5:
        fs = 3
    if fs % 2 == 0:
        fs -= 1
    return fs


def pool_halo(max_window: int, width: int, height: int) -> tuple[int, int]:
    """Columns left / right of an event that its pooling window reads: the
    W-1 clip lets row i run to linear index i*H + min(y+M, W-1), i.e. into
    column i + floor(min(H-1+M, W-1) / H)."""
    return max_window, max_window + min(height - 1 + max_window, width - 1) // height


def halo(filter_size: int, max_window: int, width: int, height: int, exchange: bool = True) -> tuple[int, int]:
    """Stored columns beyond the owned ones, (left, right).  Exchange: the
    pooling halo (flows imported), at least the SAE halo 2*fRad.  Recompute:
    the pooling halo plus the SAE halo of its events."""
    sae = 2 * (normalised_filter(filter_size) // 2)
    left, right = pool_halo(max_window, width, height)
    if exchange:
        return max(left, sae), max(right, sae)
    return left + sae, right + sae


@dataclass(frozen=True)
class Strip:
    rank: int
    own_lo: int
    own_hi: int
    reg_lo: int
    reg_hi: int


def plan(x: np.ndarray, width: int, height: int, n_strips: int, filter_size: int, max_window: int,
         exchange: bool = True) -> list[Strip]:
    """Column ranges for n_strips ranks, balanced by the events of `x`."""
    return plan_hist(np.bincount(np.asarray(x, dtype=np.int64), minlength=width), height, n_strips, filter_size,
                     max_window, exchange)


def plan_hist(hist: np.ndarray, height: int, n_strips: int, filter_size: int, max_window: int,
              exchange: bool = True) -> list[Strip]:
    """Column ranges for n_strips ranks, balanced by a per-column event count
    (farms.synth_column_hist for a synthetic stream no rank holds whole)."""
    width = int(len(hist))
    if n_strips < 1 or n_strips > width:
        raise ValueError("need 1 <= n_strips <= width")
    cum = np.cumsum(np.asarray(hist, dtype=np.float64))
    total = cum[-1] if cum.size else 0.0
    cuts = [0]
    for r in range(1, n_strips):
        c = int(np.searchsorted(cum, total * r / n_strips, side="left")) + 1 if total > 0 else r * width // n_strips
        c = max(c, cuts[-1] + 1)
        c = min(c, width - (n_strips - r))
        cuts.append(c)
    cuts.append(width)
    hl, hr = halo(filter_size, max_window, width, height, exchange)
    return [Strip(r, cuts[r], cuts[r + 1], max(0, cuts[r] - hl), min(width, cuts[r + 1] + hr)) for r in range(n_strips)]


def region_mask(x: np.ndarray, s: Strip) -> np.ndarray:
    return (x >= s.reg_lo) & (x < s.reg_hi)


def owned_mask(x: np.ndarray, s: Strip) -> np.ndarray:
    return (x >= s.own_lo) & (x < s.own_hi)


def exchange_lists(x_stored: np.ndarray, strips: list[Strip], rank: int) -> dict[int, tuple[np.ndarray, np.ndarray]]:
    """Per peer s: (send, recv) indices into this rank's stored events.

    send: my owned events in s's stored region — s's halo events that I own;
    recv: my stored events that s owns — my halo events whose flows s sends.
    Both sides select the same columns of the same stream in stream order, so
    send of r -> s and recv of s <- r list the same events in the same order:
    only flows travel, no indices.  Peers with nothing either way are left out."""
    me = strips[rank]
    x = np.asarray(x_stored)
    out = {}
    for s in strips:
        if s.rank == rank:
            continue
        lo, hi = max(me.own_lo, s.reg_lo), min(me.own_hi, s.reg_hi)
        send = np.nonzero((x >= lo) & (x < hi))[0] if lo < hi else np.zeros(0, np.int64)
        lo, hi = max(s.own_lo, me.reg_lo), min(s.own_hi, me.reg_hi)
        recv = np.nonzero((x >= lo) & (x < hi))[0] if lo < hi else np.zeros(0, np.int64)
        if send.size or recv.size:
            out[s.rank] = (send.astype(np.int32), recv.astype(np.int32))
    return out


def exchange(dist, lists: dict, send_bufs: dict, recv_bufs: dict) -> None:
    """One grouped send/recv with every peer of `lists` (torch.distributed P2P:
    ncclSend / ncclRecv in one group over RCCL, or gloo): send_bufs[s] to s,
    recv_bufs[s] from s.  Pairs with empty buffers both ways are skipped by
    both ends alike."""
    ops = []
    for s in sorted(lists):
        if send_bufs[s].numel():
            ops.append(dist.P2POp(dist.isend, send_bufs[s], s))
        if recv_bufs[s].numel():
            ops.append(dist.P2POp(dist.irecv, recv_bufs[s], s))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
