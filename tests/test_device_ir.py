"""Guards for bit-exactness of the device code: compile rt_hip.hip to LLVM IR for gfx950 with
the production flags and check that no float op may be contracted or approximated.

(ROCm's __fsqrt_rn / __fdiv_rn carry !fpmath 3.0 / 2.5 -> approximate sqrt/div: this test
is what caught it.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def ir(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("ir") / "rt.ll")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", "--cuda-device-only", "-emit-llvm", "-S",
                    os.path.join(ROOT, "ray_tracying_amd", "csrc", "hip", "rt_hip.hip"), "-o", out],
                   check=True, capture_output=True)
    return open(out).read()


def test_no_fp_contraction(ir):
    assert "fmuladd" not in ir
    for flag in (" contract ", " afn ", " reassoc ", " fast "):
        assert flag not in ir, flag


def test_no_approximate_div_sqrt(ir):
    assert "!fpmath" not in ir


def _culling_fmas(ir: str) -> tuple[int, int]:
    """(scalar f32 fmas whose first operand is a converted plane code -- the BVH slab test's
    `fma(float(code), step * inv, (origin - o) * inv)`, node_visit: a byte code (uitofp) or, in
    planes-only instances, an fp16 code (fpext half) -- , all scalar f32 fmas)."""
    import re
    conv, cull, total = set(), 0, 0
    for line in ir.splitlines():
        if line.startswith("define "):
            conv = set()  # value names are per function
        m = re.match(r"\s*(%[\w.]+) = (uitofp|fpext half) ", line)
        if m:
            conv.add(m.group(1))
        if re.search(r"call (noundef )?float @llvm\.fma\.f32\(float ", line):
            total += 1
            first = re.search(r"@llvm\.fma\.f32\(float (%[\w.]+)", line)
            if first and first.group(1) in conv:
                cull += 1
    return cull, total


def test_fma_only_in_powf_div_and_culling(ir):
    # fused ops allowed: the f64 fma of the glibc powf restatement, the f32 / f64 fma of the
    # Markstein quotient (rt_div.h: exact remainder and correction, == IEEE division,
    # tests/test_div.py), and the fma of the BVH slab test, which only culls (padded boxes, exact
    # re-check of every candidate hit) -- one scalar fma per plane (r05: it issues beside the
    # byte converts; a packed fma does not), recognised by its converted-code first operand
    # (a byte, or the fp16 code v_fma_mix_f32 converts inside the fma).
    # Every other scalar f32 fma is one of rt_div_by's two, whose first takes an fneg (the
    # remainder's -q0); CSE may merge one of a pair across identical quotients, so the count
    # need not be even.
    cull, total = _culling_fmas(ir)
    assert cull >= 24  # every instance's node visit: 24 planes
    assert cull % 24 == 0, cull
    assert total - cull <= 2 * ir.count("fneg float")
    assert "@llvm.fma.v2f32" not in ir  # no packed f32 fma left
