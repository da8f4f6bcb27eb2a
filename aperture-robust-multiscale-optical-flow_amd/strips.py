"""Spatial x-strips for multi-GPU runs.

Rank r owns the events of columns [own_lo, own_hi): strips are balanced by
event count (column histogram quantiles) over the whole stream.  Its handle
stores the owned columns widened by `halo(...)` on each side:

  * pooling an owned event reads flow cells of columns [x-M, x+M] and, through
    the reference's x-major aliasing (vFlow.cpp:1000/1113), column x+M+1;
  * the local fit of each of those cells' events reads SAE columns +-2*fRad.

So every flow an owned event pools from is computed from complete data and the
owned records are bitwise those of a whole-sensor run (the fit is local and the
pooling sum order depends only on the contributor list).  No data-path
collective is needed; the halo all-gather is replaced by recomputation.
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


def halo(filter_size: int, max_window: int) -> int:
    return max_window + 1 + 2 * (normalised_filter(filter_size) // 2)


@dataclass(frozen=True)
class Strip:
    rank: int
    own_lo: int
    own_hi: int
    reg_lo: int
    reg_hi: int


def plan(x: np.ndarray, width: int, n_strips: int, filter_size: int, max_window: int) -> list[Strip]:
    """Column ranges for n_strips ranks, balanced by the events of `x`."""
    return plan_hist(np.bincount(np.asarray(x, dtype=np.int64), minlength=width), n_strips, filter_size, max_window)


def plan_hist(hist: np.ndarray, n_strips: int, filter_size: int, max_window: int) -> list[Strip]:
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
    h = halo(filter_size, max_window)
    return [Strip(r, cuts[r], cuts[r + 1], max(0, cuts[r] - h), min(width, cuts[r + 1] + h)) for r in range(n_strips)]


def region_mask(x: np.ndarray, s: Strip) -> np.ndarray:
    return (x >= s.reg_lo) & (x < s.reg_hi)


def owned_mask(x: np.ndarray, s: Strip) -> np.ndarray:
    return (x >= s.own_lo) & (x < s.own_hi)
