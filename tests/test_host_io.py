"""Text formats of the batch path (host/event_io.cpp), CPU only.

Input semantics follow the reference parser (src/vFlow.cpp:147,173-188; SURVEY
§A Q9): getline + `stream >> x >> y >> t >> p` into variables that survive
across lines.  Output: the 11 columns of vFlow.cpp:438 with ostream defaults.
"""
import ctypes
import os

import numpy as np
import pytest

import farms

IO_LIB = os.path.join(farms.BUILD_DIR, "libfarms_io.so")


@pytest.fixture(scope="module")
def io():
    lib = ctypes.CDLL(IO_LIB)
    lib.farms_io_parse.restype = ctypes.c_int64
    lib.farms_io_parse.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 4 + [
        ctypes.c_int64]
    lib.farms_io_format.restype = ctypes.c_int64
    lib.farms_io_format.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    return lib


def parse(io, text: bytes, max_events=1 << 40):
    cap = text.count(b"\n") + 2
    x, y, p = (np.zeros(cap, np.int32) for _ in range(3))
    t = np.zeros(cap, np.uint32)
    n = io.farms_io_parse(text, len(text), max_events, x.ctypes.data, y.ctypes.data, t.ctypes.data, p.ctypes.data,
                          cap)
    assert n >= 0
    return [(int(x[i]), int(y[i]), int(t[i]), int(p[i])) for i in range(n)]


def test_plain_lines(io):
    assert parse(io, b"1 2 30 1\n3 4 50 -1\n") == [(1, 2, 30, 1), (3, 4, 50, -1)]


def test_last_line_without_newline_and_crlf(io):
    assert parse(io, b"1 2 30 1\r\n3 4 50 -1") == [(1, 2, 30, 1), (3, 4, 50, -1)]


def test_blank_and_short_lines_repeat_previous_values(io):
    # a blank line re-pushes the previous event; a short line keeps the missing tail
    assert parse(io, b"1 2 30 1\n\n7 8\n") == [(1, 2, 30, 1), (1, 2, 30, 1), (7, 8, 30, 1)]


def test_failed_conversion_zeroes_field_and_skips_rest(io):
    # "x" cannot convert: y = 0, t and p keep their values
    assert parse(io, b"1 2 30 1\n5 x 40 0\n") == [(1, 2, 30, 1), (5, 0, 30, 1)]
    # "12.5": x = 12, then ".5" fails -> y = 0
    assert parse(io, b"12.5 3 4 1\n")[0][:2] == (12, 0)


def test_overflow_saturates(io):
    ev = parse(io, b"1 2 30 1\n4 5 99999999999 0\n")
    assert ev[1] == (4, 5, 4294967295, 1)  # t saturates, p not read
    assert parse(io, b"99999999999 1 2 3\n")[0][0] == 2147483647


def test_negative_stamp_wraps(io):
    assert parse(io, b"1 2 -5 1\n")[0][2] == 2 ** 32 - 5


def test_max_events_caps_lines(io):
    assert len(parse(io, b"1 1 1 1\n2 2 2 2\n3 3 3 3\n", max_events=2)) == 2


def test_record_format_matches_ostream_defaults(io):
    rec = farms.Records(4)
    rec.x[:] = [1, 2, 3, 4]
    rec.y[:] = [5, 6, 7, 8]
    rec.t[:] = [0, 10, -5, 2 ** 31 - 1]
    rec.p[:] = [1, 0, 1, 0]
    rec.r_true[:] = [0.0, 123.456789, float("inf"), 1e-7]
    rec.theta_true[:] = [-0.0, 3.14159265, 1.0, -2.5]
    rec.vx[:] = [0.0, 1234567.0, float("nan"), 0.1]
    rec.vy[:] = [0.0, -1e-5, 2.0, 100000.0]
    rec.r_local[:] = [0.0, 12.0, 1e20, 5.0]
    rec.theta_local[:] = [0.0, 0.5, -1.0, 1.0]
    rec.scale[:] = [0, 5, 50, 25]
    c = rec.as_c()
    buf = ctypes.create_string_buffer(4096)
    n = io.farms_io_format(ctypes.byref(c), 4, buf, 4096)
    lines = buf.value.decode().splitlines()
    assert n > 0 and len(lines) == 4
    assert lines[0] == "1 5 0 1 0 -0 0 0 0 0 0"
    assert lines[1] == "2 6 10 0 123.457 3.14159 1.23457e+06 -1e-05 12 0.5 5"
    assert lines[2] == "3 7 -5 1 inf 1 nan 2 1e+20 -1 50"
    assert lines[3] == "4 8 2147483647 0 1e-07 -2.5 0.1 100000 5 1 25"
    # the Python formatter produces the same text
    assert rec.to_text().splitlines() == lines
