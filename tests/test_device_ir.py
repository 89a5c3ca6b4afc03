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


def test_fma_only_in_powf_div_and_culling(ir):
    # fused ops allowed: the f64 fma of the glibc powf restatement, the f32 / f64 fma of the
    # Markstein quotient (rt_div.h: exact remainder and correction, == IEEE division,
    # tests/test_div.py), and the packed (v2f32) fma of the BVH slab test, which only culls
    # (padded boxes, exact re-check of every candidate hit).  Every scalar f32 fma is one of
    # rt_div_by's two, whose first takes an fneg (the remainder's -q0); CSE may merge one of a
    # pair across identical quotients, so the count need not be even.
    f32_fma = ir.count("call float @llvm.fma.f32")
    assert f32_fma <= 2 * ir.count("fneg float")
    assert "@llvm.fma.v2f32" in ir  # the culling slab is where the packed form is expected
