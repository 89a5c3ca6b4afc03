"""bench.py's N-rank path on the GPU: the lattice tile deal, per-rank rendering into packed
device buffers, the gather to rank 0 and the unpack must give the same frame, bit for bit, as
one rank rendering every tile (the counter RNG is keyed by pixel/sample, not by rank).

`bench.py --gpus N` is started directly, as the driver does: it spawns its N ranks (a child
torch.distributed.run) and the JSON line must say n_gpus N.  The ranks share the one GPU
of the test box and gather through gloo (RT_BENCH_BACKEND=gloo):
this exercises everything bench.py does for N > 1 except the RCCL transport itself, which
tests/test_comm.py and the driver's multi-GPU runs cover.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--tris", "20000", "--res", "320", "--spp-sqrt", "3", "--tile", "64", "--steps", "1", "--warmup", "0",
         "--no-cpu-baseline", "--pmc-traffic", ""]


def _bench(tmp_path, n, tag):
    frame = str(tmp_path / f"frame_{tag}.npy")
    env = dict(os.environ, RT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    # the driver's form: `bench.py --gpus N` started directly spawns its N ranks
    cmd = [sys.executable, "bench.py", "--gpus", str(n)]
    r = subprocess.run(cmd + SMALL + ["--dump-frame", frame], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == n
    # the per-rank summary: every rank's wall / render / gather time and rays
    rk = line["ranks"]
    assert rk["n"] == n and len(rk["render_ms_per_step"]) == n and len(rk["gather_ms_per_step"]) == n
    assert sum(rk["rays_per_step"]) == line["config"]["rays_per_step"]
    assert 0 <= rk["slowest_rank"] < n and all(v > 0 for v in rk["render_ms_per_step"])
    return np.load(frame)


@pytest.mark.gpu
def test_bench_ranks_gather_bit_exact(tmp_path, gpu):
    one = _bench(tmp_path, 1, "n1")
    # 320x320 with 64-px tiles = 5x5 tiles: 3 ranks get 9/8/8 tiles, padded buffers
    three = _bench(tmp_path, 3, "n3")
    assert one.shape == three.shape == (320, 320, 3)
    assert np.isfinite(one).all() and one.max() > 0
    assert int((one.view(np.uint32) != three.view(np.uint32)).sum()) == 0
