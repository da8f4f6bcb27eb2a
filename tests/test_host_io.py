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
    lib.farms_io_parse_threads.restype = ctypes.c_int64
    lib.farms_io_parse_threads.argtypes = lib.farms_io_parse.argtypes + [ctypes.c_int]
    lib.farms_io_write.restype = ctypes.c_int
    lib.farms_io_write.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64]
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


def _libc_g(v: float) -> str:
    """glibc printf("%g") of one double: what `ostream << double` prints."""
    libc = ctypes.CDLL(None)
    b = ctypes.create_string_buffer(64)
    libc.snprintf(b, 64, b"%g", ctypes.c_double(v))
    return b.value.decode()


def test_float_format_matches_printf_g(io):
    """The writer's to_chars path equals printf %g on rounding boundaries,
    exponent switch points, subnormals, signed zero and non-finite values."""
    rng = np.random.default_rng(7)
    vals = [0.0, -0.0, float("inf"), -float("inf"), float("nan"), -float("nan"), 5e-324, 2.2250738585072014e-308,
            1.7976931348623157e308, 9.999995, 9.9999949999, 0.00010000005, 0.0001, 9.99999e-05, 123456.5,
            999999.5, 999999.4, 1e6, 1e-5, 0.5, 2.5, 1234565.0]
    vals += list(rng.standard_normal(400) * 10.0 ** rng.integers(-12, 12, 400))
    vals += list(np.round(rng.standard_normal(200), 6))  # many exact ties of the 6-digit rounding
    n = len(vals)
    rec = farms.Records(n)
    rec.x[:] = rng.integers(-2 ** 31, 2 ** 31, n, dtype=np.int64).astype(np.int32)
    for col in ("r_true", "theta_true", "vx", "vy", "r_local", "theta_local"):
        getattr(rec, col)[:] = vals
        vals = vals[1:] + vals[:1]
    c = rec.as_c()
    buf = ctypes.create_string_buffer(n * 160)
    assert io.farms_io_format(ctypes.byref(c), n, buf, n * 160) > 0
    for i, line in enumerate(buf.value.decode().splitlines()):
        f = line.split(" ")
        assert f[0] == str(int(rec.x[i]))
        want = [_libc_g(float(getattr(rec, col)[i])) for col in ("r_true", "theta_true", "vx", "vy", "r_local",
                                                                     "theta_local")]
        assert f[4:10] == want, (i, f[4:10], want)


def test_threaded_writer_equals_formatter(io, tmp_path):
    """write_records formats blocks of 128k records on several threads; the file
    equals the one-pass formatter's text byte for byte."""
    n = 700_000
    rng = np.random.default_rng(3)
    rec = farms.Records(n)
    rec.x[:] = np.arange(n, dtype=np.int32)
    rec.y[:] = rng.integers(0, 720, n)
    rec.t[:] = np.arange(n, dtype=np.int32) * 3
    rec.p[:] = rng.integers(0, 2, n)
    for col in ("r_true", "theta_true", "vx", "vy", "r_local", "theta_local"):
        getattr(rec, col)[:] = rng.standard_normal(n) * 100
    rec.scale[:] = rng.integers(0, 11, n) * 5
    c = rec.as_c()
    path = tmp_path / "out.txt"
    assert io.farms_io_write(str(path).encode(), ctypes.byref(c), n) == 0
    cap = n * 160
    buf = ctypes.create_string_buffer(cap)
    m = io.farms_io_format(ctypes.byref(c), n, buf, cap)
    assert path.read_bytes() == buf.raw[:m]


def _parse_arrays(io, text: bytes, threads: int, max_events=1 << 40):
    cap = text.count(b"\n") + 2
    x, y, p = (np.zeros(cap, np.int32) for _ in range(3))
    t = np.zeros(cap, np.uint32)
    n = io.farms_io_parse_threads(text, len(text), max_events, x.ctypes.data, y.ctypes.data, t.ctypes.data,
                                  p.ctypes.data, cap, threads)
    assert n >= 0
    return n, x[:n], y[:n], t[:n], p[:n]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_chunk_parallel_parse_equals_one_thread(io, seed):
    """Lines are parsed in chunks on several threads; fields a chunk's leading
    lines carry over from earlier lines (short, blank, failed lines) are filled
    in afterwards. Any thread count gives the one-thread result, including
    chunks made only of carrying lines and a max_events cap inside a chunk."""
    rng = np.random.default_rng(seed)
    kinds = [b"%d %d %d %d", b"%d %d", b"%d", b"", b"   ", b"%d %d x 1", b"%d -%d %d -1", b"99999999999 %d %d %d",
             b"%d %d %d %d\r", b"a b c d", b"%d\t%d  %d %d extra"]
    lines = []
    for i in range(3000):
        k = kinds[rng.integers(0, len(kinds))] if rng.random() < 0.5 else kinds[0]
        vals = tuple(int(v) for v in rng.integers(0, 5000, k.count(b"%d")))
        lines.append(k % vals if vals else k)
    if seed == 1:  # a long run of carrying lines, longer than a chunk
        lines[1000:2500] = [b""] * 1500
    text = b"\n".join(lines) + (b"" if seed == 2 else b"\n")
    ref = _parse_arrays(io, text, 1)
    for threads in (2, 3, 7, 16):
        got = _parse_arrays(io, text, threads)
        assert got[0] == ref[0]
        for a, b in zip(got[1:], ref[1:]):
            assert np.array_equal(a, b), threads
    for cap in (1, 777, 2999):
        r1 = _parse_arrays(io, text, 1, cap)
        r7 = _parse_arrays(io, text, 7, cap)
        assert r1[0] == r7[0] == cap
        for a, b in zip(r1[1:], r7[1:]):
            assert np.array_equal(a, b)


def parse_serial(io, text: bytes, numevents=1 << 40):
    io.farms_io_parse_serial.restype = ctypes.c_int64
    io.farms_io_parse_serial.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64] + [ctypes.c_void_p] * 5 + [
        ctypes.c_int64]
    cap = text.count(b"\n") + 2
    first = np.zeros(4, np.int32)
    x, y, p = (np.zeros(cap, np.int32) for _ in range(3))
    t = np.zeros(cap, np.uint32)
    n = io.farms_io_parse_serial(text, len(text), numevents, first.ctypes.data, x.ctypes.data, y.ctypes.data,
                                 t.ctypes.data, p.ctypes.data, cap)
    assert n >= 0
    f = (int(first[0]), int(first[1]), int(first[2]), int(np.uint32(first[3])))
    return f, [(int(x[i]), int(y[i]), int(t[i]), int(p[i])) for i in range(n)]


def test_serial_parse_first_line_and_relative_time(io):
    """vFlowManager::run (vFlow.cpp:520-580): line 1 is (x0, y0, t0) only; the
    loop subtracts t0 and clamps the polarity in place."""
    f, ev = parse_serial(io, b"3 4 1000 -1\n1 2 1030 -1\n5 6 1050 1\n")
    assert f == (1, 3, 4, 1000)
    assert ev == [(1, 2, 30, 0), (5, 6, 50, 1)]


def test_serial_parse_carry_subtracts_t0_again(io):
    """A line without a time field keeps the carried *relative* stamp, from
    which `time_ = time_ - t0` subtracts t0 once more (uint32 wrap); a missing
    polarity keeps the clamped one."""
    f, ev = parse_serial(io, b"0 0 100 1\n1 2 130 -1\n7 8\n")
    assert ev[0] == (1, 2, 30, 0)
    assert ev[1] == (7, 8, (30 - 100) % (1 << 32), 0)


def test_serial_parse_numevents_cap(io):
    """while (getline && eventsComputed <= NUMEVENTS): NUMEVENTS + 1 events."""
    text = b"".join(b"%d 1 %d 1\n" % (i, 100 + i) for i in range(10))
    _, ev = parse_serial(io, text, numevents=3)
    assert len(ev) == 4 and ev[-1] == (4, 1, 4, 1)
    _, ev = parse_serial(io, b"")
    assert ev == []
