#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X ray-trace path.

Metric (BASELINE.json): Mrays/sec (primary+secondary), 1024x1024 @ 100 spp; % HBM roofline.
Workload (north_star / SURVEY.md 8(d) C5 at the headline resolution): synthetic 1M-triangle
soup (planes with c3 == c0, splitmix64 seed 20251226), 1024x1024, -s 10 (100 jittered spp),
-bvh, -light_sample 1.  A ray is one BVH::get_intersection call (camera + reflection +
refraction + shadow rays), counted by the kernels.  One step = one full frame.

N GPUs: one process per GPU (torch.distributed, RCCL).  `bench.py --gpus N` started directly
spawns the N ranks itself (a child torch.distributed.run, before any GPU call); under an
external launcher WORLD_SIZE must equal --gpus.  The frame's 64x64 tiles are dealt
to the ranks on a 2-D lattice (tiles.tile_rank; --deal balanced: equal counts balanced by a
projected-centre cost estimate, measured slower; image-tile data parallelism, fixed total
work -> "strong" scaling), each rank renders its tiles into a device buffer and rank 0 gathers the packed
tiles over RCCL/xGMI inside the timed step.  value = all ranks' rays / max-over-ranks time.

roofline: the traversal kernel (trace_refill_kernel) is bound by
VALU issue, not by bytes -- the tree and primitives (~0.1 GB) stay on-die -- so the line
reports it against the VALU peak: useful lane-operations per second (wave64 VALU
instructions x 64 x lane utilisation, from the committed rocprofv3 PMC pass of the same
build) over 256 CUs x the highest wave64 VALU issue rate per CU-cycle that SQ_INSTS_VALU
shows for tools/ubench_valu.hip's instruction streams (1.73, a mixed int / convert / fp32
stream; the guide's spec 2 per CU-cycle beside it) x 2.4 GHz.  Beside it, per average trace launch (HIP
events on the launch stream over the timed steps): `hbm` = PMC HBM bytes (traffic) / launch
time vs 8 TB/s, and `l2` = algorithmic bytes (80 B per BVH4 node visit in planes-only scenes,
64 B otherwise, + the primitive record per primitive test, counted by an instrumented run of the same frame) / launch time vs the L2's 34.5 TB/s.
Scenes of a few primitives (C1-C4) get no roofline claim.
cpu_baseline: the compiled reference (oracle/_ref/ref_driver; kind "reference") -- or the
oracle restatement if the reference binary is absent (kind "port") -- on rank 0 at every N, after timing,
single-threaded, on a bounded sample of the same frame (12 rows spread evenly over it; its
rays/sample beside the frame's); plus the same number of rows run as 16 concurrent
single-threaded processes (the job's CPU share on the GPU box).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec (primary+secondary), 1024x1024 @100spp; % HBM roofline"
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md "L2 (per XCD)": ~34.5 TB/s aggregate over 8 XCDs
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
# VALU peaks (T lane-ops/s = wave64 instructions per CU-cycle x 256 CUs x 64 lanes x 2.4 GHz):
#   measured -- the highest rate SQ_INSTS_VALU shows for tools/ubench_valu.hip's independent
#     instruction streams (rocprofv3 --pmc, tools/pmc_ubench.py; profiles/<label>_ubench_valu_pmc.json)
#   spec     -- MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles on a SIMD-32,
#     4 SIMDs per CU = 2 instructions per CU-cycle (78.6 T lane-ops/s)
N_CU, MAX_CLOCK_GHZ = 256, 2.4
SPEC_VALU_WAVE_INSTR_PER_CU_CYCLE = 2.0
UBENCH_PROFILE = "r06_v6"  # committed counter-measured VALU microbenchmark (profiles/)


def valu_peak(path):
    """(wave64 VALU instructions per CU-cycle, source) from a pmc_ubench.py summary."""
    if path and os.path.exists(path):
        d = json.load(open(path))
        if d.get("max_valu_wave_instr_per_cu_cycle"):
            return float(d["max_valu_wave_instr_per_cu_cycle"]), f"{os.path.relpath(path, ROOT)} ({d.get('label', '')})"
    return 1.0, "assumed 1 wave64 instruction per CU-cycle (no counter-measured microbenchmark found)"
def valu_block(pv: dict, pmc_valu: str, peak_ipc: float, peak_src: str) -> dict:
    """The traversal kernel's VALU roofline from a pmc_valu.py summary: useful lane-ops/s (PMC wave64
    VALU instructions/s x 64 x lane utilisation) against the guide's peak (`frac`, VERDICT r05 item
    6), and against the highest issue rate measured on this chip (`frac_vs_measured`)."""
    peak_tops = N_CU * peak_ipc * 64 * MAX_CLOCK_GHZ / 1e3
    spec_tops = N_CU * SPEC_VALU_WAVE_INSTR_PER_CU_CYCLE * 64 * MAX_CLOCK_GHZ / 1e3
    achieved = pv["valu_g_wave_instr_per_s"] * 64 * pv["lane_utilisation"] / 1e3
    return {"achieved": round(achieved, 3), "frac": round(achieved / spec_tops, 4),
            "frac_vs_spec": round(achieved / spec_tops, 4), "spec_peak": round(spec_tops, 2),
            "frac_vs_measured": round(achieved / peak_tops, 4), "measured_peak": round(peak_tops, 2),
            "measured_peak_source": peak_src,
            "issue_frac": round(pv["valu_g_wave_instr_per_s"] / (N_CU * peak_ipc * MAX_CLOCK_GHZ), 4),
            "lane_utilisation": pv["lane_utilisation"], "measured_clock_ghz": pv.get("clock_ghz"),
            "source": f"{os.path.relpath(pmc_valu, ROOT)} ({pv.get('label', '')})"}


def frames_per_call(requested: int, one_pass: bool, split: int, units: int) -> int:
    """Frames per rt_render_frames call (--frames-per-call; 0 = auto).  Auto: up to eight whole
    frames' samples per call -- 8 frames of a whole frame, 8N of a rank's share of an N-way split,
    so a share's launch has the whole-frame run's size -- and at most 2^30 samples (C5: 1); a frame
    of fewer than 4M samples (C2) as many as make 64M (at most 64).  One traversal launch per call:
    its tail, and the camera and shading launches, are paid once per call (r06 sweep, same box:
    headline 1 / 4 / 8 frames 8,322-8,374 / 8,535-8,567 / 8,566-8,576 Mrays/s, C3 +3 % at 8, C2
    5,494 / 6,516-6,583 at 8 / 64; profiles/r06ad_frames_per_call_sweep.txt).  The step pipeline
    renders one frame per call (rt_render_frames would run them one after another)."""
    if not one_pass:
        return 1
    if requested > 0:
        return requested
    if split <= 1 and units < 4 * 2 ** 20:
        return max(1, min(64, -(-(64 * 2 ** 20) // max(units, 1))))
    return max(1, min(8 * max(split, 1), (2 ** 30) // max(units, 1)))


def frame_groups(seeds, b: int):
    """The frames split into calls of at most b, as evenly as possible (20 frames, b = 8:
    7 + 7 + 6), so that no call is much smaller than the others."""
    n = len(seeds)
    if n == 0:
        return []
    k = -(-n // b)
    sizes = [n // k + (1 if i < n % k else 0) for i in range(k)]
    out, i = [], 0
    for sz in sizes:
        out.append(list(seeds[i:i + sz]))
        i += sz
    return out


def cpu_baseline_rank(args) -> int | None:
    """The rank that times the reference CPU path after the timed steps: rank 0 at every N (the
    north_star asks for it beside the 1, 2, 4 and 8-GPU numbers), none with --no-cpu-baseline."""
    return None if args.no_cpu_baseline else 0


# one BVH4 node per visit: 80 B in planes-only scenes (fp16 plane codes), 64 B otherwise;
# one 64-B plane / 128-B transformed record per primitive test
NODE_BYTES_PLANES, NODE_BYTES_OTHER = 80, 64
PMC_PROFILE = "r06_v6"  # committed rocprofv3 PMC summaries of the headline workload (profiles/)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_quota():
    """The job's CPU quota from its cgroup (v2 cpu.max, or v1 cfs quota / period) in cores, with
    the file it came from; (None, None) when no quota is set."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return float(q) / float(per), path
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0 and per > 0:
            return q / per, "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
    except (OSError, ValueError):
        pass
    return None, None


def usable_cpus() -> int:
    """Cores this process may run on: its affinity mask, capped by the cgroup CPU quota (the
    job's share; os.cpu_count() is the whole host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q, _ = cpu_quota()
    if q is not None:
        n = max(1, min(n, int(q)))
    return n


def host_cpus() -> dict:
    """Where the multi-process CPU baseline's core count comes from (BENCH line evidence)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    q, src = cpu_quota()
    return {"affinity": aff, "os_cpu_count": os.cpu_count(), "cgroup_quota_cores": q, "cgroup_quota_file": src,
            "usable": usable_cpus(),
            "rule": "usable = affinity capped by the cgroup quota; processes = min(16, usable) (the job's "
                    "OMP_NUM_THREADS-style share on the GPU pool is 16)",
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def launch_plan(gpus, env) -> tuple[str, object]:
    """How this invocation runs, decided before anything touches the GPU:
    ("run", world)    -- render as one rank of `world` (WORLD_SIZE from torchrun, or 1);
    ("spawn", n)      -- --gpus n > 1 without WORLD_SIZE: start n ranks as a child
                         torch.distributed.run (one process per GPU), relay its exit code;
    ("error", msg)    -- --gpus disagrees with the WORLD_SIZE an external launcher set."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if gpus is None else int(gpus)
        if n < 1:
            return "error", f"bench.py: --gpus {n} must be >= 1"
        return ("spawn", n) if n > 1 else ("run", 1)
    world = int(ws)
    if gpus is not None and int(gpus) != world:
        return "error", (f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (set by the launcher); "
                         "pass the same rank count to both, or drop the launcher and let --gpus spawn the ranks")
    return "run", world


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus n` run directly: the ranks are a child `torch.distributed.run` (this
    process imports neither torch nor HIP, so nothing is exec'd after GPU init).  Every rank
    inherits stdout, so rank 0's JSON line is the run's output; a failed rank fails the run."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log(f"bench.py: spawning {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.run(cmd, env=env).returncode


def rank_summary(dist, coll: str, world: int, steps: int, wall_s: float, render_ms: float, gather_ms: float,
                 rays: float) -> dict:
    """Per-rank timing of the timed steps, all-gathered so rank 0's line shows which rank was slow
    and what the collective cost.  Per rank and per step: `wall_ms` -- its own
    time from the start barrier until its last frame was gathered (before the end barrier, which
    makes every rank wait for the slowest); `render_ms` -- the GPU time of its frames' kernels
    (rt_stats.kernel_ms: HIP events from a frame's first kernel to its last, after any earlier work
    on the stream -- frames in flight overlap, so with frames_in_flight > 1 the sum can exceed the
    step); `gather_ms` -- its part of the framebuffer gather (HIP events around
    torch.distributed.gather on the collective's stream, or host time over gloo), including the
    wait for the other ranks to arrive; `rays`.  slowest_rank = the largest render_ms."""
    import torch
    mine = torch.tensor([wall_s * 1e3 / steps, render_ms / steps, gather_ms / steps, rays / steps],
                        dtype=torch.float64, device=coll)
    if dist is not None and world > 1:
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
    else:
        parts = [mine]
    rows = [p.cpu().tolist() for p in parts]
    render = [r[1] for r in rows]
    slow = max(range(len(rows)), key=lambda i: render[i])
    return {
        "n": len(rows),
        "wall_ms_per_step": [round(r[0], 4) for r in rows],
        "render_ms_per_step": [round(r[1], 4) for r in rows],
        "gather_ms_per_step": [round(r[2], 4) for r in rows],
        "rays_per_step": [int(r[3]) for r in rows],
        "slowest_rank": slow,
        "slowest_render_ms_per_step": round(render[slow], 4),
        "fastest_render_ms_per_step": round(min(render), 4),
        "mean_render_ms_per_step": round(sum(render) / len(render), 4),
        "definitions": "per rank and step: wall = own time from the start barrier to its last gather (before the "
                       "end barrier); render = GPU time of its frames' kernels (rt_stats.kernel_ms; overlapping "
                       "frames in flight each counted); gather = its torch.distributed.gather incl. waiting for the "
                       "other ranks (HIP events on GPU, host time over gloo); slowest_rank = largest render",
    }


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); > 1 without WORLD_SIZE spawns them (torch.distributed.run), "
                         "with WORLD_SIZE set it must equal it; default: WORLD_SIZE, else 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="diagnostic: set up the ranks and their process group, print the rank count, render nothing")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp-sqrt", type=int, default=10)
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--seed", type=int, default=20251226)
    ap.add_argument("--scene", default=None, help="render this scene.json instead of the soup")
    ap.add_argument("--cpu-rows", type=int, default=12, help="rows of the frame in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--light-samples", type=int, default=1, help="-light_sample (shadow rays per light with radius > 0)")
    ap.add_argument("--emulate", type=int, default=0,
                    help="diagnostic: render only rank --emulate-rank's tiles of an N-way split on this one GPU")
    ap.add_argument("--emulate-rank", type=int, default=0)
    ap.add_argument("--deal", choices=["balanced", "measured", "lattice"], default="lattice",
                    help="tiles -> ranks: the 2-D lattice; or equal counts balanced by a per-tile cost -- the "
                         "projected-centre estimate (balanced), or the node visits of one instrumented render of the "
                         "whole frame before timing (measured; rank 0 deals and broadcasts)")
    ap.add_argument("--light-radius", type=float, default=None,
                    help="override every light's radius (SURVEY.md 8(d) C4: soft shadows, e.g. 1.0)")
    ap.add_argument("--primary-only", action="store_true",
                    help="SURVEY.md 8(d) C2 BVH-stress variant: the soup without lights (one ray per sample)")
    ap.add_argument("--cpu-procs", type=int, default=min(16, usable_cpus()),
                    help="concurrent reference processes for the multi-core CPU figure (<= 1: skip); default: one "
                         "per usable core (affinity capped by the cgroup CPU quota), at most 16 (the GPU pool's "
                         "per-job share: OMP_NUM_THREADS / MAX_JOBS are 16 there)")
    ap.add_argument("--pmc-traffic", default=None,
                    help="JSON with per-launch HBM bytes of the trace kernel (tools/pmc_traffic.py); default: the "
                         "committed profile of the headline workload, attached to that workload only")
    ap.add_argument("--pmc-valu", default=None,
                    help="JSON with the trace kernel's VALU issue fraction / lane utilisation (tools/pmc_valu.py); "
                         "default as --pmc-traffic")
    ap.add_argument("--ubench", default=None,
                    help="JSON of the counter-measured VALU microbenchmark (tools/pmc_ubench.py): the measured VALU "
                         "peak; default: the committed profile")
    ap.add_argument("--frames-in-flight", type=int, default=0,
                    help="frames rendered concurrently (scene handles on their own streams; one-pass scenes): the next "
                         "frame's camera rays and trace fill the tail of the other frame's trace launch; 0 (auto): 3 "
                         "when this rank renders at most 4M samples per frame (C2), 2 up to 32M (a rank's share of a 4- "
                         "or 8-way split), else 1 (whole frames lose: their traversals interleave instead of overlapping "
                         "at the tail)")
    ap.add_argument("--frames-per-call", type=int, default=0,
                    help="frames rendered by one rt_render_frames call (one camera pass, one traversal launch, one "
                         "shading pass for all of them; one-pass scenes): 0 (auto) = the split N for a rank's share "
                         "of an N-way split (so each call has the whole frame's samples), frames of fewer than 4M "
                         "samples as many as make 8M (at most 8: C2), else 1")
    ap.add_argument("--dump-frame", default=None,
                    help="after timing, render the frame at --seed with the timed steps' calls (same frames in "
                         "flight), gather it and save it (rank 0) as an (H, W, 3) .npy; unrendered tiles NaN")
    return ap.parse_args()


def _cpu_cmd(scene_path: str, args, y0: int, y1: int, step: int = 1):
    W = args.res
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if os.path.exists(ref):
        return [ref, "-input", scene_path, "-bvh", "-s", str(args.spp_sqrt), "-light_sample", str(args.light_samples),
                "-seed", "42", "-rows", str(y0), str(y1), "-row-step", str(step)], "reference"
    # the oracle restatement renders one contiguous band (its -region)
    return [os.path.join(ROOT, "oracle", "oracle_cli"), "-input", scene_path, "-bvh", "-s", str(args.spp_sqrt),
            "-light_sample", str(args.light_samples), "-rng", "counter", "-seed", str(args.seed), "-region", "0",
            str(y0), str(W),
            str(y1 - y0)], "port"


def cpu_baseline(scene_path: str, args, rank: int, frame_rays_per_sample: float | None = None):
    """Reference CPU path on a bounded sample of the same frame: --cpu-rows rows spread evenly
    over it (every k-th row, k = H // rows, starting at k // 2: the soup's dense centre and its
    background in proportion), on one core; then the same number of rows on
    each of N cores at once, as N concurrent single-threaded processes on disjoint row sets
    (offset within the stride; the reference cannot split one image across threads)."""
    W = H = args.res
    n_rows = max(1, min(args.cpu_rows, H))
    k = max(1, H // n_rows)
    spp = max(1, args.spp_sqrt) ** 2

    def rows_for(off):  # rows off, off + k, ... : n_rows of them
        return off, min(H, off + (n_rows - 1) * k + 1)

    y0, y1 = rows_for(k // 2)
    cmd, kind = _cpu_cmd(scene_path, args, y0, y1, k)
    if kind == "port":  # contiguous centre band
        y0 = H // 2 - n_rows // 2
        y1 = y0 + n_rows
        cmd, kind = _cpu_cmd(scene_path, args, y0, y1)
    if not os.path.exists(cmd[0]):
        return None
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp")
    wall = time.time() - t0
    if r.returncode != 0:
        log("cpu baseline failed:", r.stderr[-2000:])
        return None
    st = json.loads(r.stdout.strip().splitlines()[-1])
    rays = st["rays"]
    secs = st["render_seconds"]
    rows_desc = (f"{n_rows} rows spread over the {W}x{H} frame (rows {y0}, {y0 + k}, ... {y1 - 1}: every {k}th)"
                 if kind == "reference" else f"rows {y0}-{y1 - 1} of the {W}x{H} frame")
    rps = rays / (W * n_rows * spp)
    out = {
        "value": rays / secs / 1e6, "unit": "Mrays/s", "cores": 1, "kind": kind,
        "sample": (f"{rows_desc} at {spp} spp ({W * n_rows} px, {rays} rays = {rps:.3f} rays/sample"
                   + (f" vs the whole frame's {frame_rays_per_sample:.3f}" if frame_rays_per_sample else "")
                   + f"; render {secs:.1f} s single-threaded; scene load + BVH build {st['load_seconds']:.1f} s "
                   f"excluded; wall {wall:.1f} s)"),
        "sample_rays_per_sample": round(rps, 4),
        "frame_rays_per_sample": round(frame_rays_per_sample, 4) if frame_rays_per_sample else None,
    }
    n = args.cpu_procs
    if n > 1:
        jobs = []
        for j in range(n):
            if kind == "reference":  # disjoint row sets: offsets spread within the stride
                a0, a1 = rows_for((k // 2 + j * max(1, k // n)) % k)
                c, _ = _cpu_cmd(scene_path, args, a0, a1, k)
            else:  # disjoint bands packed around the centre
                first = max(0, H // 2 - (n * n_rows) // 2)
                a0 = min(H - n_rows, first + j * n_rows)
                c, _ = _cpu_cmd(scene_path, args, a0, a0 + n_rows)
            jobs.append(subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd="/tmp"))
        rates, total = [], 0
        for jb in jobs:
            so, se = jb.communicate()
            if jb.returncode != 0:
                log("cpu baseline (all cores) failed:", se[-1000:])
                return out
            stk = json.loads(so.strip().splitlines()[-1])
            rates.append(stk["rays"] / stk["render_seconds"] / 1e6)
            total += stk["rays"]
        out["value_multi_proc"] = sum(rates)
        out["procs"] = n
        out["host_cpus"] = host_cpus()
        out["sample_multi_proc"] = (f"{n} concurrent single-threaded processes (one per usable core, at most 16), "
                                    f"{n_rows} rows each ({total} rays); value = sum of the per-process rates")
    return out


def main():
    args = parse()
    how, what = launch_plan(args.gpus, os.environ)
    if how == "error":
        log(what)
        sys.exit(2)
    if how == "spawn":
        sys.exit(spawn_ranks(what))
    world = what
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    # RT_BENCH_BACKEND=gloo: rehearsal of the N-rank path with more ranks than GPUs (ranks
    # share devices, collectives through host memory) -- functional checks only, not a metric
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    dist = None
    if args.dry_run:  # launcher check without a GPU: process group, one collective, the rank count
        ranks_in_group = 1
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            t = torch.tensor([1.0])
            dist.all_reduce(t)
            ranks_in_group = int(t.item())
        # the per-rank summary's collective with stand-in timings (rank r: r + 1 ms of render per step)
        summ = rank_summary(dist, "cpu", world, 1, 0.001 * (rank + 2), 1.0 * (rank + 1), 0.5, 1000.0 * (rank + 1))
        if rank == 0:
            # what the rendered line would carry besides: the rank timing the CPU baseline, and the
            # VALU roofline block from the committed headline PMC summary
            pv_path = os.path.join(ROOT, "profiles", PMC_PROFILE + "_pmc_valu.json")
            pv = json.load(open(pv_path)) if os.path.exists(pv_path) else None
            peak_ipc, peak_src = valu_peak(os.path.join(ROOT, "profiles", UBENCH_PROFILE + "_ubench_valu_pmc.json"))
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_in_group": ranks_in_group, "ranks": summ,
                              "cpu_baseline_rank": cpu_baseline_rank(args),
                              "roofline_valu": valu_block(pv, pv_path, peak_ipc, peak_src) if pv else None}),
                  flush=True)
        if dist:
            dist.destroy_process_group()
        return
    import ray_tracying_amd as rt
    from ray_tracying_amd import tiles as tl

    dev = local_rank if backend == "nccl" else local_rank % max(torch.cuda.device_count(), 1)
    coll = f"cuda:{dev}" if backend == "nccl" else "cpu"
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)

    # ---- scene: every rank builds the identical scene locally (deterministic generator)
    if args.scene:
        scene_path = args.scene
        workload = os.path.basename(args.scene)
        # the same file for the GPU and the CPU baseline: resolution (and light radius) set here
        sc_json = json.load(open(args.scene))
        sc_json["render"] = {"resolution_x": args.res, "resolution_y": args.res}
        if args.light_radius is not None:
            for light in sc_json.get("lights", []):
                light["radius"] = args.light_radius
            workload += f", light radius {args.light_radius}"
        scene_path = f"/tmp/rt_bench_scene_{os.getpid()}_{rank}.json"
        with open(scene_path, "w") as f:
            json.dump(sc_json, f)
    else:
        tag = "_nolights" if args.primary_only else ""
        scene_path = f"/tmp/rt_bench_soup_{args.tris}_{args.res}{tag}_{rank}.json"
        if not os.path.exists(scene_path):
            rt.make_soup(scene_path, args.tris, seed=20251226, width=args.res, height=args.res)
            if args.primary_only:  # the soup with "lights": [] -> 1 ray/sample
                txt = open(scene_path).read()
                i = txt.index('"lights": [')
                j = txt.index("\n", i)
                open(scene_path, "w").write(txt[:i] + '"lights": [],' + txt[j:])
        workload = f"synthetic triangle soup, {args.tris} triangles (planes c3=c0), splitmix64 seed 20251226"
        if args.primary_only:
            workload += ", no lights (primary rays only)"
    t0 = time.time()
    scene = rt.Scene(scene_path, resolution=(args.res, args.res))
    load_s = time.time() - t0
    W, H = scene.width, scene.height
    ds = rt.DeviceScene(scene, dev)
    T = args.tile
    tiles_x, tiles_y = tl.tile_grid(W, H, T)
    n_tiles = tiles_x * tiles_y
    # tiles -> ranks: the 2-D lattice; --deal balanced: equal tile counts balanced by the
    # projected-centre cost estimate (every rank computes the same deal from the same scene;
    # its slowest rank measured slower than the lattice's)
    split = world if world > 1 else (args.emulate if args.emulate > 1 else 1)
    deal = None
    if split > 1 and args.deal == "balanced":
        deal = tl.balanced_deal(ds.tile_costs(T, T), split)
    elif split > 1 and args.deal == "measured":  # one instrumented render of the whole frame (not timed)
        full = torch.empty(n_tiles * T * T * 3, dtype=torch.float32, device=f"cuda:{dev}")
        ds.render_tiles(np.arange(n_tiles, dtype=np.int32), T, T, full.data_ptr(),
                        rt.RenderParams(spp_sqrt=args.spp_sqrt, light_samples=args.light_samples, use_bvh=True,
                                        seed=args.seed, count_work=True))
        del full
        costs = ds.tile_costs_measured(T, T, args.spp_sqrt)
        if (costs < 0).any():
            raise SystemExit("bench.py --deal measured: the instrumented render measured no per-tile costs "
                             "(the step pipeline does not; one-pass scenes only)")
        deal_t = torch.as_tensor(tl.balanced_deal(costs, split), dtype=torch.int32, device=coll)
        if dist:  # the measurement varies in its last bits between GPUs: rank 0's deal for everyone
            dist.broadcast(deal_t, src=0)
        deal = deal_t.cpu().numpy()
    mine = tl.assign_tiles(n_tiles, world, rank, tiles_x, deal)
    if args.emulate > 1 and world == 1:  # one rank's share of an N-way split (scaling prediction)
        mine = tl.assign_tiles(n_tiles, args.emulate, args.emulate_rank, tiles_x, deal)
    out = torch.zeros(tl.tiles_per_rank(n_tiles, world, tiles_x, deal) * T * T * 3, dtype=torch.float32,
                      device=f"cuda:{dev}")
    gathered = None
    log(f"[rank {rank}] scene {W}x{H}, {scene.info.n_shapes} shapes, {scene.info.n_nodes} nodes, depth "
        f"{scene.info.tree_depth}, load+build {load_s:.1f} s; {len(mine)} tiles on cuda:{dev}")

    params = rt.RenderParams(spp_sqrt=args.spp_sqrt, light_samples=args.light_samples, use_bvh=True, seed=args.seed)
    timing = {"on": False, "render_ms": 0.0, "gather_s": 0.0, "gather_ev": []}

    def gather(buf):
        """Framebuffer gather to rank 0 over RCCL / xGMI; timed (HIP events on the collective's
        stream, or host time over gloo) during the timed steps."""
        nonlocal gathered
        if not dist:
            return
        if timing["on"] and coll != "cpu":
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gathered = tl.gather_to_root(dist, buf, rank, world)
            e1.record()
            timing["gather_ev"].append((e0, e1))
        else:
            t = time.perf_counter()
            gathered = tl.gather_to_root(dist, buf if coll != "cpu" else buf.cpu(), rank, world)
            if timing["on"]:
                timing["gather_s"] += time.perf_counter() - t

    def step(seed):
        params.seed = seed
        st = ds.render_tiles(mine, T, T, out.data_ptr(), params)
        gather(out)
        return st

    # ---- instrumented frame: algorithmic bytes per ray (same seed as the first timed step); its
    # path decides whether frames in flight apply (one-pass calls only)
    cp = rt.RenderParams(spp_sqrt=args.spp_sqrt, light_samples=args.light_samples, use_bvh=True, seed=args.seed,
                         count_work=True)
    cst = ds.render_tiles(mine, T, T, out.data_ptr(), cp)
    prim_bytes = scene.info.prim_stride  # 64 B planes / 128 B transformed records
    node_bytes = NODE_BYTES_PLANES if prim_bytes == 64 else NODE_BYTES_OTHER
    bytes_per_ray = (node_bytes * cst.node_visits + prim_bytes * cst.prim_tests) / max(cst.rays, 1)
    log(f"[rank {rank}] instrumented: rays {cst.rays}, node visits {cst.node_visits} "
        f"({cst.node_visits / max(cst.rays, 1):.2f}/ray), box tests {cst.box_tests} "
        f"({cst.box_tests / max(cst.rays, 1):.1f}/ray), prim tests {cst.prim_tests} "
        f"({cst.prim_tests / max(cst.rays, 1):.2f}/ray), {bytes_per_ray:.0f} B/ray")

    # Frames in flight (--frames-in-flight F > 1): frame k renders on scene handle k % F and its
    # own HIP stream, deferred (RenderParams.sync=False), and is finished -- waited for, its
    # framebuffer gathered -- only once frame k + F - 1 is enqueued, so the next frame's camera
    # rays and this frame's shading run in the idle tail of the other frame's trace launch.
    # Every frame is rendered in full and gathered; steps are timed exactly as with F = 1.
    units = len(mine) * T * T * max(1, args.spp_sqrt) ** 2
    # Frames per call (r06): B consecutive frames render in ONE rt_render_frames call -- every
    # sample of them in one camera pass, one traversal launch and one shading pass -- so a
    # launch's drain tail and the short camera / shading launches are paid once per B frames.
    # Auto (frames_per_call): up to eight whole frames' samples per call, so a rank's share of an
    # N-way split renders 8N frames per call and its launches have the whole-frame run's size (the
    # 7-wave traversal, the same tail share) -- r05's eighth, one launch an eighth the size, ran at
    # 0.84 of the whole frame's rate; small frames (C2: 1M samples, one short launch
    # bound by its own tail) as many as make 64M.  Every frame is still rendered in full (its own
    # seed) and gathered; the timed steps are the same K frames (profiles/r06ad_frames_per_call_sweep.txt,
    # r06t_c2_frames_per_call.txt).  Step-pipeline scenes render one frame per call.
    one_pass_path = cst.path == rt.PATH_ONE_PASS
    B = frames_per_call(args.frames_per_call, one_pass_path, split, units)
    if B > 1:
        out = torch.zeros(B * out.numel(), dtype=torch.float32, device=f"cuda:{dev}")
    share_floats = out.numel() // B  # per frame, padded to the largest rank's share (equal gathers)
    # auto (one box, r04): C2's 1.05M samples 2,606 / 2,786 / 2,690 Mrays/s at F = 2 / 3 / 4; one
    # rank's eighth (18M) 6,322 at F = 2, 5,926 at F = 3; whole frames keep one.  Step-pipeline
    # calls (reflection, refraction, soft lights) complete before returning: nothing to overlap
    # (ADVICE r04), so they keep one frame in flight; multi-frame calls are whole-frame sized
    F = args.frames_in_flight if args.frames_in_flight > 0 else (
        1 if not one_pass_path or B > 1 else 3 if units <= 4 * 2 ** 20 else 2 if units <= 32 * 2 ** 20 else 1)
    if B > 1 and F > 1:
        raise SystemExit("bench.py: --frames-per-call > 1 renders synchronous calls (--frames-in-flight 1)")
    fl_ds = [ds] + [rt.DeviceScene(scene, dev) for _ in range(F - 1)]
    fl_out = [out] + [torch.zeros_like(out) for _ in range(F - 1)]
    fl_st = [torch.cuda.Stream(device=dev) for _ in range(F)] if F > 1 else []
    last_group = [1]  # frames in the last call's buffer (the last gathered frame is its last)

    def multi(seeds):
        """B > 1: each group of frames is one rt_render_frames call into `out` (frame-major), then
        one gather of the group's frames."""
        sts = []
        for g in frame_groups(seeds, B):
            params.seed = g[0]
            st = ds.render_frames(g, mine, T, T, out.data_ptr(), params)
            last_group[0] = len(g)
            gather(out[:len(g) * share_floats])
            sts.append(st)
        return sts

    def issue(k, seed):
        i = k % F
        p = rt.RenderParams(spp_sqrt=args.spp_sqrt, light_samples=args.light_samples, use_bvh=True, seed=seed,
                            sync=False)
        fl_ds[i].render_tiles(mine, T, T, fl_out[i].data_ptr(), p, stream=fl_st[i].cuda_stream)

    def finish(k):
        i = k % F
        st = fl_ds[i].wait()  # a deferred frame, or the held stats of one that completed in issue()
        gather(fl_out[i])  # the frame is complete (wait)
        return st

    def run_frames(seeds):
        """Render the frames (F in flight) and return their stats in order; the last frame's
        buffer is fl_out[(len(seeds) - 1) % F] (gathered: `gathered`).  With B > 1 frames per
        call: one entry per call, and the last frame is the last of `out`'s last_group[0]."""
        if B > 1:
            return multi(seeds)
        if F == 1:
            return [step(sd) for sd in seeds]
        sts = []
        for k, sd in enumerate(seeds):
            issue(k, sd)
            if k >= F - 1:
                sts.append(finish(k - F + 1))
        for k in range(max(0, len(seeds) - F + 1), len(seeds)):
            sts.append(finish(k))
        return sts

    if B > 1:
        # Workspace sizing (setup, like the instrumented frame above; not a warmup step): the
        # library grows its per-call workspace to the largest call it has seen, so one untimed call
        # of B frames makes it the size of every timed call -- without it the first timed call
        # larger than the warmup's would reallocate GBs of workspace inside the timed region.
        ds.render_frames([args.seed + 3000 + k for k in range(B)], mine, T, T, out.data_ptr(), params)
        torch.cuda.synchronize()
    run_frames([args.seed + 1000 + w for w in range(args.warmup)])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rays = 0
    trace_ms = 0.0
    busy_ms = 0.0
    render_ms = 0.0
    launches = 0
    one_pass = True
    timing["on"] = True
    for st in run_frames([args.seed + k for k in range(args.steps)]):
        one_pass = one_pass and st.path == rt.PATH_ONE_PASS
        rays += st.rays
        trace_ms += st.trace_ms
        busy_ms += st.trace_busy_ms
        render_ms += st.kernel_ms
        launches += st.iterations
    timing["on"] = False
    torch.cuda.synchronize()
    own_wall = time.perf_counter() - t0  # before the end barrier: this rank's own time
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gather_ms = timing["gather_s"] * 1e3 + sum(e0.elapsed_time(e1) for e0, e1 in timing["gather_ev"])
    ranks = rank_summary(dist, coll, world, args.steps, own_wall, render_ms, gather_ms, float(rays))

    tot = torch.tensor([float(rays), trace_ms, float(launches), bytes_per_ray * rays, busy_ms], dtype=torch.float64,
                       device=coll)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=coll)
    if dist:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    rays_all, trace_ms_all, launches_all, alg_bytes_all, busy_ms_all = tot.tolist()
    elapsed = tmax.item()

    def last_frame(buf, r):
        """The last frame of rank r's gathered / rendered buffer (B > 1: rt_render_frames wrote its
        frames end to end, rank r's own tile count apart; the buffer is padded to the largest
        share so that every rank gathers the same size)."""
        a = buf.cpu().numpy()
        if B > 1:
            n = last_group[0]
            own = len(tl.assign_tiles(n_tiles, split, r, tiles_x, deal)) * T * T * 3
            a = a[:n * own].reshape(n, own)[-1]
        return a

    if rank == 0 and dist:  # sanity: the gathered frame has every pixel, all finite
        img = tl.unpack([last_frame(g, r) for r, g in enumerate(gathered)], world, n_tiles, T, W, H, deal)
        assert np.isfinite(img).all()
    if args.dump_frame:
        # The frame at --seed rendered by the calls the timed steps make (same F, handles and
        # streams), issued last behind F - 1 other frames still in flight -- or, with B frames per
        # call, as the last frame of a call of B -- gathered, saved by rank 0 as an (H, W, 3)
        # float32 image; tiles no rank rendered (--emulate) are NaN.
        run_frames([args.seed + 2000 + k for k in range(max(F, B) - 1)] + [args.seed])
        torch.cuda.synchronize()
        if rank == 0:
            if dist:
                img = tl.unpack([last_frame(g, r) for r, g in enumerate(gathered)], world, n_tiles, T, W, H, deal)
            else:
                last = fl_out[F - 1] if F > 1 else out
                img = np.full((H, W, 3), np.nan, dtype=np.float32)
                buf = last_frame(last, args.emulate_rank if args.emulate > 1 else 0).reshape(-1, T, T, 3)
                for k, tid in enumerate(mine):
                    x0, y0 = (tid % tiles_x) * T, (tid // tiles_x) * T
                    w, h = min(T, W - x0), min(T, H - y0)
                    img[y0:y0 + h, x0:x0 + w] = buf[k, :h, :w]
            np.save(args.dump_frame, img)

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    value = rays_all / elapsed / 1e6
    # average trace-kernel launch (per-rank launches run concurrently on different GPUs, so
    # average per launch = one GPU's kernel)
    avg_launch_ms = trace_ms_all / max(launches_all, 1)
    avg_launch_bytes = alg_bytes_all / max(launches_all, 1)
    alg_rate = avg_launch_bytes / (avg_launch_ms * 1e-3) / 1e9
    # the slot pipelines' trace launches overlap (two streams), so a launch's HIP-event time
    # includes time it shares the GPU with the other pipeline's: per launch the rate reads low.
    # busy = the union of the launches' intervals (rt_stats.trace_busy_ms): per-frame bytes over
    # it is the kernel's rate on the GPU
    busy_ms_step = busy_ms_all / world / args.steps
    alg_rate_busy = alg_bytes_all / world / args.steps / (busy_ms_step * 1e-3) / 1e9 if busy_ms_step > 0 else None
    # PMC summaries of this workload measured by rocprofv3 on this build (tools/pmc_traffic.py,
    # tools/pmc_valu.py; label = the build they were measured on): the headline frame and C5
    # (4096^2 x 64 spp, SURVEY.md 8(d)'s roofline config) each have their own, and a summary is
    # never attached to another workload's line
    soup = args.scene is None and not args.primary_only and args.tris == 1_000_000 and args.light_samples == 1
    headline = soup and args.res == 1024 and args.spp_sqrt == 10 and args.emulate <= 1 and world == 1
    c5 = soup and args.res == 4096 and args.spp_sqrt == 8 and args.emulate <= 1 and world == 1
    prof = os.path.join(ROOT, "profiles", PMC_PROFILE + ("_c5" if c5 else ""))
    pmc_traffic = args.pmc_traffic or (prof + "_pmc_traffic.json" if headline or c5 else None)
    pmc_valu = args.pmc_valu or (prof + "_pmc_valu.json" if headline or c5 else None)
    traffic, traffic_src, pv = None, None, None
    frames_per_launch = args.steps * world / launches_all if launches_all else 1.0
    if pmc_traffic and os.path.exists(pmc_traffic):
        pm = json.load(open(pmc_traffic))
        # per frame (the profiled launches' frame count: tools/pmc_traffic.py --frames), then per
        # launch of this run
        per_frame = pm.get("hbm_bytes_per_frame", pm.get("hbm_bytes_per_launch", 0) / pm.get("frames_per_launch", 1))
        traffic = round(per_frame * frames_per_launch) if per_frame else None
        traffic_src = (f"{os.path.relpath(pmc_traffic, ROOT)} ({pm.get('label', '')}; "
                       f"{pm.get('frames_per_launch', 1)} frame(s) per profiled launch)")
    if pmc_valu and os.path.exists(pmc_valu):
        pv = json.load(open(pmc_valu))
    # Few-primitive scenes (at most RT_FLAT_PRIMS bounded primitives, no textures) launch no
    # traversal: the instrumented frame -- which keeps the traversal launches --
    # tested them from one leaf item, no node visit; the timed one-pass calls then run
    # flat_render_kernel and step-pipeline calls a logic step answering its own queries, whose
    # launches are the "trace" times below
    def _textured(o) -> bool:  # some material names a texture file (an empty name is none)
        if isinstance(o, dict):
            return bool(o.get("texture_file")) or any(_textured(v) for v in o.values())
        return isinstance(o, list) and any(_textured(v) for v in o)
    textured = args.scene is not None and _textured(json.load(open(scene_path)))
    flat = cst.node_visits == 0 and cst.prim_tests > 0 and not textured and os.environ.get("RT_FLAT_RENDER", "1") != "0"
    kernel = {
        "kernel": ("flat_render_kernel" if flat and one_pass else "logic_kernel (answering its own queries)" if flat
                   else "trace_refill_kernel"),
        "avg_launch_ms": round(avg_launch_ms, 4),
        "launches_per_step": round(launches_all / args.steps / world, 3),
        "trace_busy_ms_per_step": round(busy_ms_step, 3),
        # with F > 1 frames in flight the frames' launches overlap: their busy times sum past the
        # step time, and no share of it is measured
        "trace_share_of_step": round(busy_ms_step / (elapsed / args.steps * 1e3), 3) if F == 1 else None,
        "launch_timing": "HIP events around each trace launch on its call's stream (rocprofv3 agrees: "
                         "profiles/<label>_kernel_stats.csv); trace_busy_ms_per_step is the union of one frame's "
                         "launches (the step pipeline's slot pipelines overlap theirs).  With config.frames_in_flight "
                         "> 1 the frames' launches overlap each other, so avg_launch_ms includes time shared with "
                         "the other frame's and trace_share_of_step is null",
    }
    if args.scene:  # C1-C4: a few primitives, LDS/L1-resident -- no roofline claim
        roofline = {"bound": None, "frac": None, "achieved": None, "peak": None, "unit": None, "traffic": None,
                    "note": "scene of a few primitives (on-die): no roofline claim (SURVEY.md 8(d))", **kernel}
    else:
        peak_ipc, peak_src = valu_peak(args.ubench or os.path.join(ROOT, "profiles", UBENCH_PROFILE + "_ubench_valu_pmc.json"))
        spec_tops = N_CU * SPEC_VALU_WAVE_INSTR_PER_CU_CYCLE * 64 * MAX_CLOCK_GHZ / 1e3
        valu = valu_block(pv, pmc_valu, peak_ipc, peak_src) if pv else None
        # PMC bytes per launch (a serialised --pmc run) x launches per frame over the busy time
        hbm_rate = (traffic * launches_all / world / args.steps / (busy_ms_step * 1e-3) / 1e9
                    if traffic and busy_ms_step > 0 else None)
        roofline = {
            "bound": "valu",
            "achieved": valu["achieved"] if valu else None, "peak": round(spec_tops, 2),
            "unit": "T VALU lane-ops/s", "frac": valu["frac"] if valu else None,
            "traffic": traffic, "traffic_unit": "HBM bytes per trace launch (PMC)", "traffic_source": traffic_src,
            "traffic_per_frame": round(traffic / frames_per_launch) if traffic else None,
            "peak_definition": "the guide's VALU peak (MI355X_MICROARCH.md: a wave64 instruction issues over 2 "
                               "cycles on each of 4 SIMD-32 per CU = 2 wave64 instructions per CU-cycle) x 256 CUs x "
                               "64 lanes x 2.4 GHz; achieved = PMC wave64 VALU instructions/s x 64 x lane utilisation; "
                               f"valu.frac_vs_measured prices it against the highest rate measured on this chip, "
                               f"{peak_ipc:.3f} per CU-cycle ({peak_src})",
            "valu": valu,
            "hbm": {"achieved_gbs": round(hbm_rate, 1) if hbm_rate else None, "peak_gbs": HBM_PEAK_GBS,
                    "frac": round(hbm_rate / HBM_PEAK_GBS, 4) if hbm_rate else None,
                    "alg_frac": round(alg_rate_busy / HBM_PEAK_GBS, 4) if alg_rate_busy else None,
                    "note": "the metric's '% HBM roofline': PMC HBM bytes (frac) and algorithmic bytes (alg_frac) "
                            "per busy second vs 8 TB/s.  alg_frac above 1 is no HBM rate: the tree and primitives "
                            "(~0.1 GB) are served from L2 / Infinity Cache, HBM carries a few % of the algorithmic "
                            "bytes, and the north_star's HBM-read target does not apply at this working set; the "
                            "binding roof is VALU issue (frac above)"},
            "l2": {"alg_bytes_per_launch": int(avg_launch_bytes), "alg_bytes_per_ray": round(bytes_per_ray, 1),
                   "model": "80 B (planes-only scenes: fp16 plane codes) / 64 B per BVH4 node visit + prim_stride B per primitive test",
                   "achieved_gbs_per_launch": round(alg_rate, 1),
                   "achieved_gbs": round(alg_rate_busy, 1) if alg_rate_busy else None, "peak_gbs": L2_PEAK_GBS,
                   "frac": round(alg_rate_busy / L2_PEAK_GBS, 4) if alg_rate_busy else None},
            **kernel,
        }
    cpu = None
    if cpu_baseline_rank(args) == rank:  # after timing, at every N (north_star: beside 1/2/4/8 GPUs)
        cpu = cpu_baseline(scene_path, args, rank, rays_all / args.steps / (W * H * max(1, args.spp_sqrt) ** 2))
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("reference scene " + os.path.basename(args.scene) if args.scene
                 else "synthetic (generated triangle soup)"),
        "config": {
            "workload": workload,
            "resolution": f"{W}x{H}", "spp": max(1, args.spp_sqrt) ** 2, "flags": f"-bvh -s {args.spp_sqrt} -light_sample {args.light_samples}",
            "rays_per_step": int(rays_all / args.steps), "tile": T, "parallelism": f"image tiles x{world}" + (f" ({args.deal} deal)" if split > 1 else ""),
            "rng": "counter (splitmix64 per pixel/sample)",
            "frames_in_flight": F,
            "frames_per_call": B,
            "pipeline": ("one-pass, few primitives (one flat_render_kernel launch per call: camera ray, queries and "
                         "shading per thread)" if one_pass and flat
                         else "one-pass (camera_kernel -> one trace_refill_kernel launch -> shade_reduce_kernel)" if one_pass
                         else "steps, few primitives (logic -> start over slot state, the logic step answering its own "
                              "queries: no traversal launches; then reduce)" if flat
                         else "steps (logic -> start -> trace over slot state, then reduce)"),
            **({"emulated_rank": f"{args.emulate_rank}/{args.emulate}"} if args.emulate > 1 and world == 1 else {}),
        },
        "roofline": roofline,
        "ranks": ranks,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
