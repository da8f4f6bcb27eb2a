"""The FARMS_Flow command line (host/main.cpp): flags and console behaviour of
/root/reference/src/main.cpp, and — on the GPU — the _FARMSOut_batch.txt file
against the oracle."""
import os
import subprocess

import numpy as np
import pytest

import farms
from oracle import OracleFlow
from parity import compare

CLI = os.path.join(farms.BUILD_DIR, "FARMS_Flow")


def run(*args, cwd=None):
    return subprocess.run([CLI, *args], capture_output=True, text=True, cwd=cwd, timeout=600)


def test_help_lists_the_reference_flags():
    r = run("--help")
    assert r.returncode == 0
    for flag in ("--help", "--filename arg", "--height arg", "--width arg", "--filtersize arg",
                 "--inlierCheck arg", "--numEvents arg", "--numevents arg", "--NUMEVENTS arg", "--SERIAL arg",
                 "--v arg"):
        assert flag in r.stdout


def test_unknown_and_ambiguous_options_fail():
    r = run("--bogus", "1")
    assert r.returncode == 1 and "unrecognised option" in r.stderr
    r = run("--fil", "x")  # filename / filtersize
    assert r.returncode == 1 and "ambiguous" in r.stderr
    r = run("--width")
    assert r.returncode == 1 and "missing" in r.stderr
    r = run("--width", "abc")
    assert r.returncode == 1 and "invalid" in r.stderr


def test_flag_echo_and_missing_file(tmp_path):
    r = run("--filename", str(tmp_path / "none"), "--width=64", "--height", "48", "--filtersize", "5",
            "--inlierCheck", "4", "--numEvents", "10", "--SERIAL", "0")
    assert "filename set to" in r.stdout and "width set to 64." in r.stdout and "height set to 48." in r.stdout
    assert "filtersize set to 5." in r.stdout and "inlierCheck set to 4." in r.stdout
    assert "numEvents set to 10." in r.stdout and "Running batch" in r.stdout
    # the reference reads 0 events and dies on T.at(0) (vFlow.cpp:194)
    assert "Done reading 0 Events." in r.stdout
    assert r.returncode == 2 and "no events" in r.stderr


def read_out(path):
    cols = np.loadtxt(path, dtype=np.float64, ndmin=2)
    names = farms.COLUMNS
    return {c: cols[:, i].astype(np.int32) if c in farms.INT_COLUMNS else cols[:, i] for i, c in enumerate(names)}


@pytest.mark.gpu
def test_cli_batch_output_matches_oracle(tmp_path):
    ev = farms.synth_config(2, 40_000)
    base = str(tmp_path / "bars")
    farms.write_events_text(base + ".txt", ev)
    r = run("--filename", base, "--width", "320", "--height", "320", "--filtersize", "5", "--inlierCheck", "5",
            "--SERIAL", "0")
    assert r.returncode == 0, r.stderr
    assert "Done reading 40000 Events." in r.stdout and "[Benchmark Main]" in r.stdout
    got = read_out(base + "_FARMSOut_batch.txt")
    x, y, t, p = ev.relative()
    ref = OracleFlow(320, 320, 5, 5).process(x, y, t, p)
    # the text carries 6 significant digits: compare at that resolution
    rep = compare(got, ref)
    assert rep["valid_mismatch"] == 0 and rep["x_mismatch"] == 0 and rep["t_mismatch"] == 0
    assert rep["r_true_max_rel"] < 1e-5 and rep["r_local_max_rel"] < 1e-5
    assert rep["theta_true_max_abs"] < 1e-4


@pytest.mark.gpu
def test_cli_numevents_caps_input(tmp_path):
    ev = farms.synth_config(1, 5000)
    base = str(tmp_path / "c1")
    farms.write_events_text(base + ".txt", ev)
    r = run("--filename", base, "--width", "128", "--height", "128", "--numevents", "1234", "--SERIAL", "0")
    assert r.returncode == 0, r.stderr
    assert len(open(base + "_FARMSOut_batch.txt").read().splitlines()) == 1234


@pytest.mark.gpu
def test_cli_serial_mode_runs_the_serial_engine(tmp_path):
    """--SERIAL 1 (the reference default): vFlowManager::run semantics — the
    first line only stamps lastEventTime, NUMEVENTS + 1 events are processed
    (vFlow.cpp:565), nothing is written (the writer is commented out, :487-489)."""
    ev = farms.synth_config(1, 3000)
    base = str(tmp_path / "s1")
    farms.write_events_text(base + ".txt", ev)
    r = run("--filename", base, "--width", "128", "--height", "128", "--numevents", "2000", "--SERIAL", "1")
    assert r.returncode == 0, r.stderr
    assert "Running serially" in r.stdout and f"First time = {int(ev.t[0])}" in r.stdout and "Done!" in r.stdout
    assert not os.path.exists(base + "_FARMSOut_batch.txt")
    # the reference's per-event timing lines (vFlow.cpp:641, 719) have no
    # counterpart in one batched call: one honestly labelled line for the call
    # instead, and no synthetic "Local" / "true" lines
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith(("Local ", "true "))]
    assert not lines
    batch = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("Batch ")]
    assert len(batch) == 1 and batch[0][1] == "2001" and batch[0][2] == "events"
    assert 0 < int(batch[0][3]) < 2001 and int(batch[0][5]) >= 0
