"""bench.py's multi-rank plumbing on the CPU (gloo): `bench.py --gpus N` starts N
ranks itself, every rank builds only its own share of the weak-scaling stream,
and the shares partition the stream.  --plan-only stops before the GPU."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd"))

import farms  # noqa: E402
import segments  # noqa: E402
import strips  # noqa: E402


def run_bench(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


def last_json(stdout: str) -> dict:
    return json.loads([ln for ln in stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("split", ["segments", "strips"])
def test_gpus_2_launches_two_ranks(split):
    r = run_bench("--gpus", "2", "--plan-only", "--config", "2", "--events", "60000", "--split", split)
    assert r.returncode == 0, r.stderr[-2000:]
    d = last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["plan_only"] and d["value"] is None
    assert d["detail"]["owned_events_all_ranks"] == 120000 == d["detail"]["stream_events"]
    assert d["detail"]["rank0_owned_events"] < 120000


@pytest.mark.parametrize("cfg,want", [(2, "segments"), (4, "strips"), (5, "strips")])
def test_default_split_follows_the_baseline_partition(cfg, want):
    """BASELINE configs 4 and 5 state a spatial partition with a border halo:
    their N > 1 lines default to the x-strips; the one-GPU configs' N > 1
    lines run temporal segments.  config.workload names the split either way."""
    r = run_bench("--gpus", "2", "--plan-only", "--config", str(cfg), "--events", "60000")
    assert r.returncode == 0, r.stderr[-2000:]
    d = last_json(r.stdout)
    assert d["config"]["split"] == want
    assert ("-tile spatial partition" in d["config"]["workload"]) == (want == "strips")


def test_world_size_must_match_gpus():
    r = run_bench("--gpus", "1", "--plan-only", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_synth_select_is_a_slice_of_the_stream():
    sp = farms.synth_params(2, 150_000)
    ev = farms.synth_generate(sp)
    sub, idx, t_first = farms.synth_select(sp, 2_000, 120_000, 40, 200)
    keep = np.nonzero((ev.x >= 40) & (ev.x < 200))[0]
    keep = keep[(keep >= 2_000) & (keep < 120_000)]
    assert t_first == int(ev.t[0])
    np.testing.assert_array_equal(idx, keep)
    for a, b in ((sub.x, ev.x), (sub.y, ev.y), (sub.t, ev.t), (sub.p, ev.p)):
        np.testing.assert_array_equal(a, b[keep])
    np.testing.assert_array_equal(farms.synth_column_hist(sp), np.bincount(ev.x, minlength=320))


@pytest.mark.parametrize("n_seg", [2, 3, 8])
def test_plan_rank_matches_the_whole_stream_plan(n_seg):
    ev = farms.synth_config(2, 400_000)
    _, _, t, _ = ev.relative()
    segs = segments.plan(t, n_seg)
    for r in range(n_seg):
        lo, hi = segments.rank_window(len(t), n_seg, r, warm_max=30_000)
        seg, head = segments.plan_rank(t[lo:hi], lo, len(t), n_seg, r)
        assert seg == segs[r]
        assert head == segments.head_length(segs, r)


def test_strip_plan_from_histogram_equals_plan_from_events():
    ev = farms.synth_config(2, 100_000)
    a = strips.plan(ev.x, 320, 320, 4, 5, 50)
    b = strips.plan_hist(np.bincount(ev.x, minlength=320), 320, 4, 5, 50)
    assert a == b


def test_rooflines_name_the_dominant_kernel_per_config():
    """bench.py reports the roofline of the kernel with more time per step (the
    pooling at filtersize 5, the fit at filtersize 7), with the other kernel's
    figures beside it, from live launch timings and the committed PMC summary
    of the same per-GPU workload (none committed for a config: frac null)."""
    sys.path.insert(0, ROOT)
    import bench

    ts = {"fit_launches": 100, "pool_launches": 10, "ms_fit_kernel": 50.0, "ms_pool_kernel": 20.0}
    cs = {"n_events": 1000, "n_owned": 1000, "n_valid": 400, "sae_cells": 169e3, "pool_cells": 4e6}
    ki = {"fit": "k_fit_box<3>", "pool": "k_pool<11>"}  # farms_kernel_info's names
    rl = bench.rooflines(4, "segments", ts, cs, ki)
    assert rl["dominant"] == "k_fit" and rl["k_fit"]["kernel"] == "k_fit_box"
    assert rl["k_fit"]["avg_launch_us"] == 500.0 and rl["k_pool"]["avg_launch_us"] == 2000.0
    assert rl["k_fit"]["algorithmic_bytes_per_launch"] == round((4 * 169e3 + 33 * 1000) / 100)
    ts.update(ms_fit_kernel=10.0)
    rl = bench.rooflines(3, "segments", ts, cs, dict(ki, fit="k_fit_box<2>"))
    assert rl["dominant"] == "k_pool"
    for k in ("k_fit", "k_pool"):
        r = rl[k]
        if r["traffic"]:
            assert r["frac"] == round(r["traffic"] / (r["avg_launch_us"] * 1e-6) / 1e9 / 8000.0, 4)
        else:
            assert r["frac"] is None


def test_rooflines_use_busy_wall_time_for_overlapping_launches():
    """With two fit streams the launch brackets overlap: the roofline's launch
    duration is the busy wall time (union of the brackets, farms_stats
    ms_*_busy) per launch, so launches x duration stays within the step; the
    bracket sum is reported beside it (round-4 review: C4 summed 93.7 ms of fit
    brackets in a 61.4 ms step)."""
    sys.path.insert(0, ROOT)
    import bench

    ts = {"fit_launches": 763, "pool_launches": 48, "ms_fit_kernel": 93.7, "ms_pool_kernel": 55.0,
          "ms_fit_busy": 56.6, "ms_pool_busy": 55.0}
    cs = {"n_events": 1000, "n_owned": 1000, "n_valid": 400, "sae_cells": 169e3, "pool_cells": 4e6}
    rl = bench.rooflines(4, "segments", ts, cs, {"fit": "k_fit_quad<3>", "pool": "k_pool<11>"})
    f = rl["k_fit"]
    assert f["avg_launch_us"] == round(56.6e3 / 763, 2)
    assert f["ms_busy_per_step"] == 56.6 and f["ms_bracket_sum_per_step"] == 93.7
    assert rl["dominant"] == "k_fit"
    assert f["launches_per_step"] * f["avg_launch_us"] / 1e3 <= 61.4


def test_one_gpu_lines_read_the_whole_sensor_pmc_summaries():
    """Configs 4 and 5 default to x-strips for N > 1; their one-GPU lines still
    run the whole-sensor call and take its committed PMC traffic (the round-6
    lines first looked for strip summaries and reported frac null)."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.profile_split("strips", 1) == "none" and bench.profile_split("strips", 4) == "strips"
    for cfg in (4, 5):
        tr = bench.committed_profile("traffic", cfg, bench.profile_split(bench.default_split(cfg), 1),
                                     "k_fit_quad<3>")
        assert tr and tr["traffic_bytes_per_launch"] > 0 and "_strips" not in tr["source"]
