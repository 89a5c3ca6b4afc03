"""host_gap.py -- host time around rt_render_tiles: wall time per call vs the GPU span the call
reports (kernel_ms, init to reduce), for one rank's share of the headline frame.
Usage: python3 tools/host_gap.py [N_WAY] [calls]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import ray_tracying_amd as rt  # noqa: E402
from ray_tracying_amd import tiles as tl  # noqa: E402

n_way = int(sys.argv[1]) if len(sys.argv) > 1 else 8
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
path = "/tmp/rt_hostgap_soup.json"
if not os.path.exists(path):
    rt.make_soup(path, 1_000_000, seed=20251226, width=1024, height=1024)
sc = rt.Scene(path, resolution=(1024, 1024))
ds = rt.DeviceScene(sc, 0)
tx, ty = tl.tile_grid(1024, 1024, 64)
mine = tl.assign_tiles(tx * ty, n_way, n_way - 1, tx)
out = torch.zeros(len(mine) * 64 * 64 * 3, dtype=torch.float32, device="cuda:0")
params = rt.RenderParams(spp_sqrt=10, light_samples=1, use_bvh=True, seed=1)
for _ in range(3):
    ds.render_tiles(mine, 64, 64, out.data_ptr(), params)
torch.cuda.synchronize()
walls, spans = [], []
t_prev = time.perf_counter()
for i in range(calls):
    params.seed = i
    t0 = time.perf_counter()
    st = ds.render_tiles(mine, 64, 64, out.data_ptr(), params)
    t1 = time.perf_counter()
    walls.append((t1 - t0) * 1e3)
    spans.append(st.kernel_ms)
walls.sort()
spans.sort()
print(f"spin={os.environ.get('RT_SPIN_WAIT', '0')} share 1/{n_way}: call wall median {walls[len(walls) // 2]:.3f} ms, "
      f"GPU span median {spans[len(spans) // 2]:.3f} ms, host overhead {walls[len(walls) // 2] - spans[len(spans) // 2]:.3f} ms")
