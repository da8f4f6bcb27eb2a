"""Temporal segments for multi-GPU runs on a time-ordered stream.

The per-event loop (/root/reference/src/vFlow.cpp:223-414) carries state from
one event to the next only through the sensor surfaces:

  * the local fit of event e reads the SAE (lastEventTime / cSurf, :264-267)
    as of e: the stamp of the latest earlier event at each pixel;
  * the pooling of e reads the flow surface and lastEventTime of cells with
    |t_e - t_cell| < 500 us (:1002 / :1115), flows that local fits produced.

So on a stream whose stamps never decrease, segment r = events [start, end)
can be run on its own, with records bitwise those of the whole run, from

  (a) the SAE as of `start` — a per-pixel "last stamp" surface, which is the
      merge of every earlier segment's own last-stamp surface; each rank
      computes its surface on the GPU (farms_last_stamps) and one RCCL
      all-gather hands every rank the surfaces of the ranks before it;
  (b) the local flows of the events of the last 500 us before `start`: the
      segment is prefixed with those events (the warm-up, [warm, start)),
      which are re-fitted from the SAE as of `warm` (the merge stops at
      `warm` inside the previous segment: its "head" surface) and whose own
      records are discarded.

A cell whose last event precedes `warm` has t_cell <= t[start] - 500 and can
never contribute to a segment event, so nothing else crosses the boundary.
Unlike x-strips (strips.py) no event is fitted twice except the warm-up
(~0.04% of a 50M-event segment at 1280x720).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

KILL_US = 500  # vFlow.cpp:961


@dataclass(frozen=True)
class Segment:
    rank: int
    start: int  # first owned event (global index)
    end: int    # one past the last owned event
    warm: int   # first warm-up event (global index); == start for rank 0

    @property
    def n_local(self) -> int:
        """Events the rank's handle processes: warm-up + owned."""
        return self.end - self.warm

    @property
    def n_warm(self) -> int:
        return self.start - self.warm


def is_time_ordered(t: np.ndarray) -> bool:
    t = np.asarray(t)
    return bool(t.size < 2 or np.all(t[1:].astype(np.int64) >= t[:-1].astype(np.int64)))


def plan(t_rel: np.ndarray, n_seg: int) -> list[Segment]:
    """Equal-count segments of a time-ordered stream, with their warm-ups."""
    t = np.asarray(t_rel).astype(np.int64)
    n = int(t.size)
    if n_seg < 1 or n_seg > max(n, 1):
        raise ValueError("need 1 <= segments <= events")
    if not is_time_ordered(t):
        raise ValueError("temporal segments need non-decreasing stamps; use strips.plan")
    cut = cuts(n, n_seg)
    segs = []
    for r in range(n_seg):
        start, end = cut[r], cut[r + 1]
        warm = start
        if r > 0 and start < n:
            # every event with t > t[start] - 500 before start (it may still
            # contribute to an owned event)
            warm = int(np.searchsorted(t[:start], t[start] - KILL_US, side="right"))
            if warm < cut[r - 1]:
                raise ValueError("segment shorter than the 500 us warm-up; use fewer segments")
        segs.append(Segment(r, start, end, warm))
    return segs


WARM_MAX = 4_000_000  # bound on a warm-up's length for plan_rank's stream window (events)


def cuts(n: int, n_seg: int) -> list[int]:
    return [r * n // n_seg for r in range(n_seg + 1)]


def rank_window(n: int, n_seg: int, r: int, warm_max: int = WARM_MAX) -> tuple[int, int]:
    """Stream indices [lo, hi) whose stamps plan_rank needs for rank r: its
    segment, up to warm_max events before it (its warm-up) and the events up to
    the next cut (the next rank's warm-up, which ends rank r's head)."""
    c = cuts(n, n_seg)
    return max(0, c[r] - warm_max), min(n, c[r + 1] + 1)


def plan_rank(t_window: np.ndarray, lo: int, n: int, n_seg: int, r: int) -> tuple[Segment, int]:
    """Segment r and its head length from the stamps of rank_window(n, n_seg, r)
    only (t_window = t[lo:hi]): what plan() and head_length() give on the whole
    stream, for ranks that never hold it."""
    t = np.asarray(t_window).astype(np.int64)
    if not is_time_ordered(t):
        raise ValueError("temporal segments need non-decreasing stamps; use strips")
    c = cuts(n, n_seg)
    start, end = c[r], c[r + 1]

    def warm_of(k: int) -> int:  # first event with t > t[k] - 500 (k > 0)
        w = lo + int(np.searchsorted(t[:k - lo], t[k - lo] - KILL_US, side="right"))
        if w == lo and lo > 0:
            raise ValueError("warm-up longer than the planning window; raise WARM_MAX")
        return w

    warm = start
    if r > 0 and start < n:
        warm = warm_of(start)
        if warm < c[r - 1]:
            raise ValueError("segment shorter than the 500 us warm-up; use fewer segments")
    head = end - start
    if r + 1 < n_seg and end < n:
        head = warm_of(end) - start
    return Segment(r, start, end, warm), head


def head_length(segs: list[Segment], r: int) -> int:
    """Events of segment r that precede the next segment's warm-up (its head
    surface is the SAE contribution the next rank needs at `warm`)."""
    if r + 1 >= len(segs):
        return segs[r].end - segs[r].start
    return segs[r + 1].warm - segs[r].start


def merge_rows(r: int) -> list[int]:
    """Rows of the all-gathered [head_0, full_0, head_1, full_1, ...] stack whose
    in-order merge is the SAE as of rank r's warm-up start."""
    if r == 0:
        return []
    return [2 * i + 1 for i in range(r - 1)] + [2 * (r - 1)]


def last_stamps_np(x, y, t, width: int, height: int) -> np.ndarray:
    """Reference (numpy) of farms_last_stamps: x-major last stamp per pixel, -1 if none."""
    q = np.asarray(x, np.int64) * height + np.asarray(y, np.int64)
    last = np.full(width * height, -1, np.int64)
    np.maximum.at(last, q, np.arange(q.size, dtype=np.int64))  # latest event index per pixel
    out = np.full(width * height, -1, np.int64)
    hit = last >= 0
    out[hit] = np.asarray(t, np.int64)[last[hit]]
    return out


def merge_np(rows) -> np.ndarray:
    out = None
    for a in rows:
        a = np.asarray(a, np.int64)
        out = a.copy() if out is None else np.where(a >= 0, a, out)
    return out
