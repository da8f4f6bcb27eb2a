"""Python binding of libfarms_hip.so (include/farms_hip.h) and libfarms_synth.so.

Mirrors the reference's vFlowManager batch interface (/root/reference/include/
vFlow.h:22-117): construct with (height, width, filterSize, minEvtsOnPlane),
feed events, get the 11-column _FARMSOut_ records (src/vFlow.cpp:438).  The
accelerated path is the HIP library; there is no CPU fallback — if the library
or a GPU is missing, every call raises FarmsError.
"""
from __future__ import annotations

import ctypes
import weakref
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.join(HERE, "build")
HIP_LIB = os.path.join(BUILD_DIR, "libfarms_hip.so")
SYNTH_LIB = os.path.join(BUILD_DIR, "libfarms_synth.so")

FARMS_OK = 0
FARMS_EINVAL = -1
FARMS_EHIP = -2
FARMS_ENOMEM = -3
FARMS_ENODEV = -4
FARMS_EINTERNAL = -5
PROF_TIMING = 1    # farms_set_profiling: HIP events around phases and k_fit / k_pool launches
PROF_COUNTERS = 2  # ... plus the U_loc / U_pool / candidate / contributor counters
PROF_POOL = 3      # HIP events around phases and k_pool launches only

# record columns, in the order of src/vFlow.cpp:438
COLUMNS = ("x", "y", "t", "p", "r_true", "theta_true", "vx", "vy", "r_local", "theta_local", "scale")
INT_COLUMNS = ("x", "y", "t", "p", "scale")


class FarmsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"farms error {code}: {msg}")
        self.code = code


class FarmsParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("filter_size", ctypes.c_int32),
        ("min_inliers", ctypes.c_int32),
        ("window_jump", ctypes.c_int32),
        ("max_window", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("fit_chunk", ctypes.c_int32),
        ("pool_chunk", ctypes.c_int32),
        ("region_x0", ctypes.c_int32),
        ("region_width", ctypes.c_int32),
        ("own_x0", ctypes.c_int32),
        ("own_x1", ctypes.c_int32),
        ("pool_batch", ctypes.c_int32),
        ("serial", ctypes.c_int32),
        ("import_halo", ctypes.c_int32),
    ]


class FarmsRecordsC(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in COLUMNS]


class FarmsStats(ctypes.Structure):
    _fields_ = [
        ("n_events", ctypes.c_int64),
        ("n_valid", ctypes.c_int64),
        ("sae_cells", ctypes.c_double),
        ("pool_cells", ctypes.c_double),
        ("fit_launches", ctypes.c_int32),
        ("pool_launches", ctypes.c_int32),
        ("ms_prep", ctypes.c_double),
        ("ms_fit", ctypes.c_double),
        ("ms_pool", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("ms_fit_kernel", ctypes.c_double),
        ("ms_pool_kernel", ctypes.c_double),
        ("pool_candidates", ctypes.c_double),
        ("pool_contributors", ctypes.c_double),
        ("n_owned", ctypes.c_int64),
        ("ms_fit_busy", ctypes.c_double),
        ("ms_pool_busy", ctypes.c_double),
        ("pool_scan_max", ctypes.c_int64),
        ("pool_scan_over_1k", ctypes.c_int64),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class SynthParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("n_events", ctypes.c_int64),
        ("n_bars", ctypes.c_int32),
        ("len_min", ctypes.c_double),
        ("len_max", ctypes.c_double),
        ("thick_min", ctypes.c_double),
        ("thick_max", ctypes.c_double),
        ("speed_min", ctypes.c_double),
        ("speed_max", ctypes.c_double),
        ("jitter_us", ctypes.c_int32),
        ("noise_frac", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("t0", ctypes.c_uint32),
        ("fixed_dir_deg", ctypes.c_double),
    ]


# exported symbols of include/farms_hip.h and include/farms_synth.h
HIP_SYMBOLS = (
    "farms_default_params", "farms_create", "farms_destroy", "farms_reset", "farms_process",
    "farms_process_device", "farms_set_profiling", "farms_get_stats", "farms_num_scales",
    "farms_get_last_event_time", "farms_last_error", "farms_last_stamps", "farms_merge_stamps",
    "farms_seed_sae", "farms_serial_first", "farms_fit_device", "farms_pool_device", "farms_export_flows",
    "farms_import_flows", "farms_export_flows_async", "farms_export_wait", "farms_import_flows_async",
    "farms_host_alloc", "farms_host_free", "farms_kernel_info",
)
SYNTH_SYMBOLS = ("farms_synth_preset", "farms_synth_generate", "farms_synth_write_text",
                 "farms_synth_generate_select", "farms_synth_column_hist")

_hip = None
_synth = None


def _ptr(a) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def load_hip_library() -> ctypes.CDLL:
    """Load the HIP library; raise if it has not been built (no fallback)."""
    global _hip
    if _hip is not None:
        return _hip
    # torch wheels ship their own HIP runtime under the same SONAME
    # (libamdhip64.so.7).  Whichever copy is loaded first serves the whole
    # process, and torch's GPU init fails on the system copy, so in a process
    # that has torch, let torch load its runtime before this library binds.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    # FARMS_HIP_LIB: an alternative build of the same library (tuning A/B runs
    # of tools/, e.g. `make -C ... variant NAME=x DEFS=...`); never set by the
    # tests, the bench or the driver entry points
    path = os.environ.get("FARMS_HIP_LIB") or HIP_LIB
    if not os.path.isabs(path):
        path = os.path.join(HERE, path)
    if not os.path.exists(path):
        raise FarmsError(FARMS_ENODEV, f"{path} not built; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    lib.farms_last_error.restype = ctypes.c_char_p
    for name in HIP_SYMBOLS:
        # (an older build in FARMS_HIP_LIB may lack the newest entry points;
        # tests/test_capi_and_synth.py checks that the built library has all)
        if name != "farms_last_error" and hasattr(lib, name):
            getattr(lib, name).restype = ctypes.c_int
    lib.farms_process.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_void_p]
    lib.farms_process_device.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_void_p]
    lib.farms_host_alloc.argtypes = [ctypes.c_int64, ctypes.c_void_p]
    lib.farms_host_free.argtypes = [ctypes.c_void_p]
    _hip = lib
    return lib


def load_synth_library() -> ctypes.CDLL:
    global _synth
    if _synth is not None:
        return _synth
    if not os.path.exists(SYNTH_LIB):
        raise FarmsError(FARMS_ENODEV, f"{SYNTH_LIB} not built; run __graft_entry__.build()")
    lib = ctypes.CDLL(SYNTH_LIB)
    lib.farms_synth_generate.restype = ctypes.c_int64
    lib.farms_synth_generate.argtypes = [ctypes.c_void_p] * 5
    lib.farms_synth_write_text.argtypes = [ctypes.c_char_p] + [ctypes.c_void_p] * 4 + [ctypes.c_int64]
    lib.farms_synth_generate_select.restype = ctypes.c_int64
    lib.farms_synth_generate_select.argtypes = ([ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                                 ctypes.c_int32, ctypes.c_int64] + [ctypes.c_void_p] * 6)
    lib.farms_synth_column_hist.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    _synth = lib
    return lib


def _check(lib, rc: int) -> None:
    if rc != FARMS_OK:
        raise FarmsError(rc, lib.farms_last_error().decode(errors="replace"))


# ---------------------------------------------------------------------------
# events and records


@dataclass
class Events:
    """An event stream: x, y (int32), t (uint32, absolute us), p (int32, +-1)."""

    x: np.ndarray
    y: np.ndarray
    t: np.ndarray
    p: np.ndarray

    def __len__(self) -> int:
        return int(self.x.shape[0])

    def head(self, n: int) -> "Events":
        return Events(self.x[:n].copy(), self.y[:n].copy(), self.t[:n].copy(), self.p[:n].copy())

    def relative(self, t0: int | None = None) -> tuple:
        """Host prologue of runFileCopy: t - t0 as uint32 (vFlow.cpp:194, 240-241)
        and polarity clamped to >= 0 (vFlow.cpp:245-247).  t0 defaults to the
        first stamp; a share of a longer stream passes the stream's."""
        if t0 is not None:
            t0 = np.uint32(t0)
        else:
            t0 = np.uint32(self.t[0]) if len(self) else np.uint32(0)
        t_rel = (self.t.astype(np.uint32) - t0).astype(np.uint32)
        p = np.maximum(self.p, 0).astype(np.int32)
        return (np.ascontiguousarray(self.x, dtype=np.int32), np.ascontiguousarray(self.y, dtype=np.int32),
                np.ascontiguousarray(t_rel), np.ascontiguousarray(p))


class PinnedArray:
    """A numpy array in pinned host memory (farms_host_alloc): farms_process
    DMAs it in place instead of through its staging.  The memory lives as long
    as the ctypes buffer the array views (a finalizer on the buffer frees it),
    so an array taken out of its PinnedArray, e.g. a column of
    Records(pinned=True), keeps it alive by itself."""

    def __init__(self, n: int, dtype):
        lib = load_hip_library()
        self.dtype = np.dtype(dtype)
        p = ctypes.c_void_p()
        _check(lib, lib.farms_host_alloc(ctypes.c_int64(max(n, 1) * self.dtype.itemsize), ctypes.byref(p)))
        buf = (ctypes.c_char * (max(n, 1) * self.dtype.itemsize)).from_address(p.value)
        # the ndarray holds buf through its base chain; free only when buf dies
        weakref.finalize(buf, lib.farms_host_free, ctypes.c_void_p(p.value))
        self.array = np.frombuffer(buf, dtype=self.dtype, count=n)


def pinned(a: np.ndarray):
    """A pinned copy of `a` and its owner (keep the owner alive while the array is used)."""
    own = PinnedArray(len(a), a.dtype)
    own.array[:] = a
    return own.array, own


class Records:
    """SoA of the 11 output columns (vFlow.cpp:438); pinned=True: in pinned host
    memory (farms_process then DMAs the records straight into them)."""

    def __init__(self, n: int, pinned: bool = False):
        self.n = n
        self._owners = []
        for name in COLUMNS:
            dt = np.int32 if name in INT_COLUMNS else np.float64
            if pinned:
                own = PinnedArray(n, dt)
                own.array[:] = 0
                self._owners.append(own)
                setattr(self, name, own.array)
            else:
                setattr(self, name, np.zeros(n, dtype=dt))

    def as_c(self) -> FarmsRecordsC:
        return FarmsRecordsC(*[getattr(self, name).ctypes.data for name in COLUMNS])

    @property
    def valid(self) -> np.ndarray:
        """Validity gate of vFlow.cpp:315 as seen in the output: RLocal > 0
        (an event that passes the gate has RLocal = sqrt(Vx^2 + Vy^2) > 0)."""
        return self.r_local > 0

    def to_text(self) -> str:
        """The _FARMSOut_ lines with ostream defaults (%g, 6 significant digits)."""
        lines = []
        for i in range(self.n):
            lines.append("%d %d %d %d %s %s %s %s %s %s %d" % (
                self.x[i], self.y[i], self.t[i], self.p[i],
                *("%g" % getattr(self, c)[i] for c in ("r_true", "theta_true", "vx", "vy", "r_local", "theta_local")),
                self.scale[i]))
        return "\n".join(lines) + ("\n" if lines else "")


# ---------------------------------------------------------------------------
# synthetic streams


def synth_params(config: int, n_events: int | None = None) -> SynthParams:
    lib = load_synth_library()
    p = SynthParams()
    if lib.farms_synth_preset(int(config), ctypes.byref(p)) != 0:
        raise ValueError(f"unknown synthetic configuration {config}")
    if n_events is not None:
        p.n_events = int(n_events)
    return p


def synth_generate(params: SynthParams) -> Events:
    lib = load_synth_library()
    n = int(params.n_events)
    x = np.zeros(n, np.int32)
    y = np.zeros(n, np.int32)
    t = np.zeros(n, np.uint32)
    p = np.zeros(n, np.int32)
    got = lib.farms_synth_generate(ctypes.byref(params), _ptr(x), _ptr(y), _ptr(t), _ptr(p))
    if got != n:
        raise RuntimeError(f"farms_synth_generate returned {got}")
    return Events(x, y, t, p)


def synth_select(params: SynthParams, e0: int, e1: int, x_lo: int = 0, x_hi: int | None = None,
                 count: int | None = None):
    """Events [e0, e1) of the stream with column in [x_lo, x_hi), their stream
    indices and the stream's first stamp, without materialising the whole
    stream (farms_synth_generate_select): one rank's share.  `count`: the
    number of matching events when known (from synth_column_hist), else the
    arrays are sized for e1 - e0."""
    lib = load_synth_library()
    x_hi = int(params.width) if x_hi is None else int(x_hi)
    e1 = min(int(e1), int(params.n_events))
    cap = max(e1 - int(e0), 0) if count is None else int(count)
    x = np.empty(cap, np.int32)
    y = np.empty(cap, np.int32)
    t = np.empty(cap, np.uint32)
    p = np.empty(cap, np.int32)
    idx = np.empty(cap, np.int64)
    t_first = ctypes.c_uint32(0)
    got = lib.farms_synth_generate_select(ctypes.byref(params), ctypes.c_int64(int(e0)), ctypes.c_int64(e1),
                                          ctypes.c_int32(int(x_lo)), ctypes.c_int32(x_hi), ctypes.c_int64(cap),
                                          _ptr(x), _ptr(y), _ptr(t), _ptr(p), _ptr(idx), ctypes.byref(t_first))
    if got < 0 or got > cap or (count is not None and got != cap):
        raise RuntimeError(f"farms_synth_generate_select returned {got} (expected {cap})")
    return Events(x[:got].copy(), y[:got].copy(), t[:got].copy(), p[:got].copy()), idx[:got].copy(), int(t_first.value)


def synth_column_hist(params: SynthParams) -> np.ndarray:
    """Events per column of the whole stream (farms_synth_column_hist)."""
    lib = load_synth_library()
    hist = np.zeros(int(params.width), np.int64)
    if lib.farms_synth_column_hist(ctypes.byref(params), _ptr(hist)) != 0:
        raise RuntimeError("farms_synth_column_hist failed")
    return hist


def synth_config(config: int, n_events: int | None = None) -> Events:
    return synth_generate(synth_params(config, n_events))


def write_events_text(path: str, ev: Events) -> None:
    lib = load_synth_library()
    x, y = np.ascontiguousarray(ev.x, np.int32), np.ascontiguousarray(ev.y, np.int32)
    t, p = np.ascontiguousarray(ev.t, np.uint32), np.ascontiguousarray(ev.p, np.int32)
    if lib.farms_synth_write_text(path.encode(), _ptr(x), _ptr(y), _ptr(t), _ptr(p), len(ev)) != 0:
        raise OSError(f"cannot write {path}")


# ---------------------------------------------------------------------------
# the accelerated path


class FlowManager:
    """GPU counterpart of vFlowManager's batch path (vFlow.h:100,104).

    FlowManager(height, width, filter_size, min_evts_on_plane) — argument order
    of the reference constructor.  process() runs the per-event loop of
    runFileCopy on events whose time is already relative to t0 and whose
    polarity is already clamped (see Events.relative()).  State persists across
    calls.
    """

    def __init__(self, height: int = 320, width: int = 320, filter_size: int = 3, min_evts_on_plane: int = 5,
                 window_jump: int = 5, max_window: int = 50, device: int = 0, fit_chunk: int = 0,
                 pool_chunk: int = 0, region: tuple | None = None, owned: tuple | None = None,
                 pool_batch: int = 0, serial: bool = False, import_halo: bool = False):
        self._lib = load_hip_library()
        prm = FarmsParams()
        _check(self._lib, self._lib.farms_default_params(ctypes.byref(prm)))
        prm.width, prm.height = int(width), int(height)
        prm.filter_size, prm.min_inliers = int(filter_size), int(min_evts_on_plane)
        prm.window_jump, prm.max_window = int(window_jump), int(max_window)
        prm.device, prm.fit_chunk, prm.pool_chunk = int(device), int(fit_chunk), int(pool_chunk)
        prm.pool_batch = int(pool_batch)
        prm.serial = 1 if serial else 0
        prm.import_halo = 1 if import_halo else 0
        if region is not None:  # (x0, x1): stored columns
            prm.region_x0, prm.region_width = int(region[0]), int(region[1]) - int(region[0])
        if owned is not None:  # (x0, x1): pooled columns
            prm.own_x0, prm.own_x1 = int(owned[0]), int(owned[1])
        self.params = prm
        h = ctypes.c_void_p()
        _check(self._lib, self._lib.farms_create(ctypes.byref(prm), ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.farms_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def num_scales(self) -> int:
        return int(self._lib.farms_num_scales(self._h))

    def kernel_info(self) -> dict:
        """The kernels the next call runs (farms_kernel_info), e.g.
        {"fit": "k_fit_box<2>", "pool": "k_pool<11>", ...}."""
        import json

        buf = ctypes.create_string_buffer(512)
        _check(self._lib, self._lib.farms_kernel_info(self._h, buf, ctypes.c_int32(512)))
        return json.loads(buf.value.decode())

    def reset(self) -> None:
        _check(self._lib, self._lib.farms_reset(self._h))

    def set_profiling(self, on: bool | int) -> None:
        """True: timing events and work counters; PROF_TIMING: timing only."""
        _check(self._lib, self._lib.farms_set_profiling(self._h, int(on) if not isinstance(on, bool) else (255 if on else 0)))

    def stats(self) -> dict:
        st = FarmsStats()
        _check(self._lib, self._lib.farms_get_stats(self._h, ctypes.byref(st)))
        return st.as_dict()

    def process(self, x, y, t_rel, p, out: Records | None = None) -> Records:
        """farms_process: host arrays in, host records out (into `out` when
        given, e.g. to reuse its pages across calls)."""
        x = np.ascontiguousarray(x, dtype=np.int32)
        y = np.ascontiguousarray(y, dtype=np.int32)
        t_rel = np.ascontiguousarray(t_rel, dtype=np.uint32)
        p = np.ascontiguousarray(p, dtype=np.int32)
        n = int(x.shape[0])
        if not (y.shape[0] == t_rel.shape[0] == p.shape[0] == n):
            raise ValueError("x, y, t, p must have the same length")
        rec = Records(n) if out is None else out
        if rec.n != n:
            raise ValueError("records length differs from the event count")
        oc = rec.as_c()
        _check(self._lib, self._lib.farms_process(self._h, _ptr(x), _ptr(y), _ptr(t_rel), _ptr(p), n,
                                                  ctypes.byref(oc)))
        return rec

    def serial_first(self, x: int, y: int, t_abs: int) -> None:
        """Serial mode: the file's first line only stamps lastEventTime
        (vFlow.cpp:531-556); call before the first process()."""
        _check(self._lib, self._lib.farms_serial_first(self._h, ctypes.c_int32(int(x)), ctypes.c_int32(int(y)),
                                                       ctypes.c_uint32(int(t_abs) & 0xFFFFFFFF)))

    def process_events(self, ev: Events) -> Records:
        return self.process(*ev.relative())

    # ---- temporal segments (segments.py); device int64 tensors
    def last_stamps(self, x, y, t_rel, n_head: int, head, full) -> None:
        """Per-pixel last stamp (x-major W x H, -1 = none) over the device events
        [0, n_head) into `head` and over all of them into `full`."""
        n = int(x.shape[0])
        _check(self._lib, self._lib.farms_last_stamps(
            self._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
            ctypes.c_void_p(t_rel.data_ptr()), ctypes.c_int64(n), ctypes.c_int64(int(n_head)),
            ctypes.c_void_p(head.data_ptr() if head is not None else 0), ctypes.c_void_p(full.data_ptr())))

    def merge_stamps(self, stack, out) -> None:
        """out = in-order merge of the rows of `stack` (count x W*H, contiguous)."""
        _check(self._lib, self._lib.farms_merge_stamps(self._h, ctypes.c_void_p(stack.data_ptr()),
                                                       ctypes.c_int32(int(stack.shape[0])),
                                                       ctypes.c_void_p(out.data_ptr())))

    def seed_sae(self, stamp) -> None:
        """Start this (fresh or reset) handle from the SAE surface `stamp`."""
        _check(self._lib, self._lib.farms_seed_sae(self._h, ctypes.c_void_p(stamp.data_ptr())))

    # ---- x-strips with a flow-halo exchange (strips.py)
    def fit_device(self, x, y, t_rel, p, out: dict) -> None:
        """Phase 1 of process_device: prep and the local fits (owned columns
        only with import_halo).  Then export_flows / import_flows, then
        pool_device()."""
        n = int(x.shape[0])
        rec = self._device_records(out)
        _check(self._lib, self._lib.farms_fit_device(
            self._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(t_rel.data_ptr()),
            ctypes.c_void_p(p.data_ptr()), ctypes.c_int64(n), ctypes.byref(rec)))

    def export_flows(self, idx, flows) -> None:
        """flows[i] = {L, L cos theta, L sin theta} of event idx[i] (device int32 /
        float64 (count, 3) tensors)."""
        _check(self._lib, self._lib.farms_export_flows(self._h, ctypes.c_void_p(idx.data_ptr()),
                                                       ctypes.c_int64(int(idx.shape[0])),
                                                       ctypes.c_void_p(flows.data_ptr())))

    def import_flows(self, idx, flows) -> None:
        """Set the local flows of events idx (their owners' export_flows)."""
        _check(self._lib, self._lib.farms_import_flows(self._h, ctypes.c_void_p(idx.data_ptr()),
                                                       ctypes.c_int64(int(idx.shape[0])),
                                                       ctypes.c_void_p(flows.data_ptr())))

    def export_flows_async(self, idx, flows) -> None:
        """export_flows without the wait: the gather is queued behind the fit
        (export_wait before reading `flows`), so that the next fit_device can be
        issued before the exchange completes."""
        _check(self._lib, self._lib.farms_export_flows_async(self._h, ctypes.c_void_p(idx.data_ptr()),
                                                             ctypes.c_int64(int(idx.shape[0])),
                                                             ctypes.c_void_p(flows.data_ptr())))

    def export_wait(self) -> None:
        """Wait for the last export_flows_async's gather."""
        _check(self._lib, self._lib.farms_export_wait(self._h))

    def import_flows_async(self, idx, flows) -> None:
        """import_flows queued ahead of the fit's pooling; `flows` stays valid and
        unchanged until that pool_device has completed."""
        _check(self._lib, self._lib.farms_import_flows_async(self._h, ctypes.c_void_p(idx.data_ptr()),
                                                             ctypes.c_int64(int(idx.shape[0])),
                                                             ctypes.c_void_p(flows.data_ptr())))

    def pool_device(self) -> None:
        """Phase 2: the pooling sweep of the events of the last fit_device."""
        _check(self._lib, self._lib.farms_pool_device(self._h))

    @staticmethod
    def _device_records(out: dict) -> FarmsRecordsC:
        ptr = {c: (ctypes.c_void_p(out[c].data_ptr()) if c in out else None) for c in COLUMNS}
        return FarmsRecordsC(*[ptr[c] for c in COLUMNS])

    def process_device(self, x, y, t_rel, p, out: dict) -> None:
        """Device-resident variant: torch tensors (int32 x/y/p, int32 view of the
        uint32 t) on this handle's device; `out` maps column name -> tensor
        (float64 for the six float columns, int32 for scale)."""
        n = int(x.shape[0])
        rec = FarmsRecordsC(0, 0, 0, 0, *[out[c].data_ptr() for c in COLUMNS[4:]])
        _check(self._lib, self._lib.farms_process_device(
            self._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
            ctypes.c_void_p(t_rel.data_ptr()), ctypes.c_void_p(p.data_ptr()), n, ctypes.byref(rec)))
