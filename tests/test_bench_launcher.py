"""bench.py's rank launcher (CPU): `bench.py --gpus N` started directly must run N ranks --
the driver's `python bench.py --gpus 1` form, and the same form with N > 1, may not silently
measure one GPU -- and an external launcher's WORLD_SIZE must agree with --gpus.

--dry-run stops after the process group is up (gloo) and one all-reduce has counted the
ranks, so the real torch.distributed.run child and rendezvous run here without a GPU.  The
rendering side of the N-rank path is tests/test_bench_ranks.py (GPU).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_without_launcher():
    assert bench.launch_plan(None, {}) == ("run", 1)
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(4, {}) == ("spawn", 4)
    assert bench.launch_plan(0, {})[0] == "error"


def test_plan_under_launcher():
    assert bench.launch_plan(None, {"WORLD_SIZE": "8"}) == ("run", 8)
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == ("run", 8)
    how, msg = bench.launch_plan(8, {"WORLD_SIZE": "1"})
    assert how == "error" and "WORLD_SIZE=1" in msg and "--gpus 8" in msg


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("n", [1, 3])
def test_gpus_flag_spawns_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_in_group"] == n
    # the per-rank summary rank 0 prints (all-gathered over the ranks' process group): every rank's
    # wall / render / gather time per step and rays, and which rank was slowest (the dry run's
    # stand-in timings give rank r r + 1 ms of render per step)
    rk = d["ranks"]
    assert rk["n"] == n
    for key in ("wall_ms_per_step", "render_ms_per_step", "gather_ms_per_step", "rays_per_step"):
        assert len(rk[key]) == n, key
    assert rk["render_ms_per_step"] == [float(r + 1) for r in range(n)]
    assert rk["slowest_rank"] == n - 1 and rk["slowest_render_ms_per_step"] == float(n)
    assert rk["fastest_render_ms_per_step"] == 1.0
    # the CPU baseline is timed (by rank 0) at every N, not only at N = 1,
    # and the roofline's frac is the guide's VALU peak (frac_vs_spec), the chip-measured one beside it
    assert d["cpu_baseline_rank"] == 0
    v = d["roofline_valu"]
    assert v is not None and v["frac"] == v["frac_vs_spec"]
    assert v["spec_peak"] == pytest.approx(256 * 2 * 64 * 2.4 / 1e3, rel=1e-3)
    assert v["frac_vs_measured"] > v["frac"]  # the measured peak (1.73 per CU-cycle) is below the spec


def test_cpu_baseline_rank_and_valu_block():
    import types
    assert bench.cpu_baseline_rank(types.SimpleNamespace(no_cpu_baseline=False)) == 0
    assert bench.cpu_baseline_rank(types.SimpleNamespace(no_cpu_baseline=True)) is None
    pv = {"valu_g_wave_instr_per_s": 640.0, "lane_utilisation": 0.5, "label": "x"}
    v = bench.valu_block(pv, os.path.join(ROOT, "profiles", "x.json"), 1.733, "ubench")
    assert v["achieved"] == pytest.approx(640.0 * 64 * 0.5 / 1e3, rel=1e-6)
    assert v["frac"] == v["frac_vs_spec"] == pytest.approx(v["achieved"] / 78.6432, rel=1e-3)


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "8", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr and r.stdout.strip() == ""


def test_frames_per_call_rule():
    """bench.py's frames per rt_render_frames call (r06): up to eight whole frames' samples per
    call -- 8 frames of a whole frame, 8N of a rank's share of an N-way split -- at most 2^30
    samples; small frames (C2: 1M samples) as many as make 64M; the step pipeline one;
    --frames-per-call overrides for one-pass scenes only."""
    M = 2 ** 20
    assert bench.frames_per_call(0, True, 1, 100 * M) == 8  # the headline frame (104.9M samples)
    assert bench.frames_per_call(0, True, 8, 13 * M) == 64  # a rank's eighth: 8 whole frames' samples
    assert bench.frames_per_call(0, True, 4, 26 * M) == 32
    assert bench.frames_per_call(0, True, 2, 52 * M) == 16
    assert bench.frames_per_call(0, True, 8, 134 * M) == 7  # C5's eighth: 2^30 samples at most
    assert bench.frames_per_call(0, True, 1, 1024 * M) == 1  # C5's whole frame
    assert bench.frames_per_call(0, True, 1, 1 * M) == 64  # C2
    assert bench.frames_per_call(0, True, 1, 3 * M) == 22
    assert bench.frames_per_call(0, False, 8, 13 * M) == 1
    assert bench.frames_per_call(5, True, 1, 100 * M) == 5
    assert bench.frames_per_call(5, False, 1, 100 * M) == 1


@pytest.mark.parametrize("n,b", [(20, 8), (20, 7), (5, 8), (1, 8), (16, 8), (30, 8), (0, 3)])
def test_frame_groups(n, b):
    seeds = list(range(100, 100 + n))
    g = bench.frame_groups(seeds, b)
    assert [x for grp in g for x in grp] == seeds  # every frame once, in order
    assert all(1 <= len(grp) <= b for grp in g)
    if g:
        assert max(map(len, g)) - min(map(len, g)) <= 1 and len(g) == -(-n // b)
