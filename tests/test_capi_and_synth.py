"""CPU-side checks of the shipped libraries: every symbol declared in
include/*.h is exported, the HIP library loads without a GPU and fails loudly
(no CPU fallback), and the synthetic stream generator is deterministic."""
import ctypes
import os
import re

import numpy as np
import pytest

import farms

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(farms_\w+)\s*\(", text, flags=re.M)))


def exported(path):
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.mark.parametrize("header,lib", [("farms_hip.h", farms.HIP_LIB), ("farms_synth.h", farms.SYNTH_LIB)])
def test_every_declared_symbol_is_exported(header, lib):
    names = declared_functions(header)
    assert len(names) >= 3
    missing = [n for n in names if n not in exported(lib)]
    assert not missing, missing


def test_python_binding_lists_match_headers():
    assert sorted(farms.HIP_SYMBOLS) == declared_functions("farms_hip.h")
    assert sorted(farms.SYNTH_SYMBOLS) == declared_functions("farms_synth.h")


def test_hip_library_loads_and_fails_loudly_without_a_device():
    lib = farms.load_hip_library()
    prm = farms.FarmsParams()
    assert lib.farms_default_params(ctypes.byref(prm)) == 0
    # defaults of the reference ctor / CLI (main.cpp:21-24, vFlow.cpp:73-74)
    assert (prm.width, prm.height, prm.filter_size, prm.min_inliers, prm.window_jump, prm.max_window) == (
        320, 320, 3, 5, 5, 50)
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the no-device path does not apply")
    with pytest.raises(farms.FarmsError) as ei:
        farms.FlowManager()
    assert ei.value.code == farms.FARMS_ENODEV


def test_bad_parameters_are_rejected_before_touching_a_device():
    lib = farms.load_hip_library()
    prm = farms.FarmsParams()
    lib.farms_default_params(ctypes.byref(prm))
    prm.window_jump, prm.max_window = 1, 50  # 51 scales > maxWindow: the reference throws
    h = ctypes.c_void_p()
    assert lib.farms_create(ctypes.byref(prm), ctypes.byref(h)) == farms.FARMS_EINVAL
    prm.window_jump, prm.max_window, prm.width = 5, 50, 0
    assert lib.farms_create(ctypes.byref(prm), ctypes.byref(h)) == farms.FARMS_EINVAL
    # a stored region narrower than the owned columns' halo (vFlow.cpp:870-883,
    # 1000): owned [100, 200) of a 1280 x 720 sensor needs [50, 251) with the
    # flow exchange, [48, 253) when halo events are re-fitted (fs 5)
    prm.width, prm.height, prm.filter_size = 1280, 720, 5
    prm.own_x0, prm.own_x1 = 100, 200
    for imp, lo, hi in [(1, 51, 251), (1, 50, 250), (0, 50, 251), (0, 48, 252)]:
        prm.import_halo, prm.region_x0, prm.region_width = imp, lo, hi - lo
        assert lib.farms_create(ctypes.byref(prm), ctypes.byref(h)) == farms.FARMS_EINVAL, (imp, lo, hi)
        assert b"halo" in lib.farms_last_error()


@pytest.mark.parametrize("cfg,W,H", [(1, 128, 128), (2, 320, 320), (3, 1280, 720)])
def test_synth_streams_are_deterministic_and_well_formed(cfg, W, H):
    n = 60_000
    a = farms.synth_config(cfg, n)
    b = farms.synth_config(cfg, n)
    for c in ("x", "y", "t", "p"):
        np.testing.assert_array_equal(getattr(a, c), getattr(b, c))
    assert len(a) == n
    assert a.x.min() >= 0 and a.x.max() < W and a.y.min() >= 0 and a.y.max() < H
    assert np.all(np.diff(a.t.astype(np.int64)) >= 0)  # sorted by time
    assert set(np.unique(a.p)) <= {-1, 1}
    assert a.t[0] >= 1_000_000


def test_synth_presets_follow_survey():
    p = farms.synth_params(3)
    assert (p.width, p.height, p.n_events, p.n_bars) == (1280, 720, 50_000_000, 64)
    assert p.seed == 0x5EED0003
    p1 = farms.synth_params(1)
    assert (p1.width, p1.height, p1.n_events, p1.n_bars, p1.fixed_dir_deg) == (128, 128, 100_000, 1, 30.0)


def test_relative_time_and_polarity_clamp():
    ev = farms.Events(np.array([1, 2], np.int32), np.array([3, 4], np.int32),
                      np.array([1_000_000, 999_999], np.uint32), np.array([-1, 1], np.int32))
    x, y, t, p = ev.relative()
    assert t.tolist() == [0, 2 ** 32 - 1]  # uint32 wrap (vFlow.cpp:241)
    assert p.tolist() == [0, 1]


def test_text_round_trip(tmp_path):
    ev = farms.synth_config(1, 2000)
    path = str(tmp_path / "ev.txt")
    farms.write_events_text(path, ev)
    rows = np.loadtxt(path, dtype=np.int64)
    assert rows.shape == (2000, 4)
    np.testing.assert_array_equal(rows[:, 0], ev.x)
    np.testing.assert_array_equal(rows[:, 2], ev.t)
