"""rt_div_by (ray_tracying_amd/csrc/common/rt_div.h) == IEEE division, bit for bit.

The camera kernels divide by the jitter's s, the image resolution and a camera ray's length
through Markstein's correction on a precomputed correctly rounded reciprocal (three
operations instead of the division sequence).  Markstein's theorem makes that the correctly
rounded quotient whenever nothing over- or underflows; checked here against the CPU's
division on random binary32 / binary64 pairs, the stratified-jitter operands of every s the
benchmarks use, and every binary32 numerator of 16 binades for the resolution divisors.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("div") / "div_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "native", "div_check.cpp"),
                    "-o", exe, "-lm"], check=True)
    return exe


def run(exe, *args):
    out = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, check=True)
    checked, bad = map(int, out.stdout.split())
    return checked, bad


def test_div_random_f32(checker):
    checked, bad = run(checker, "f32", "random", 20_000_000, 1)
    assert checked == 20_000_000 and bad == 0


def test_div_random_f64(checker):
    checked, bad = run(checker, "f64", "random", 10_000_000, 2)
    assert checked == 10_000_000 and bad == 0


@pytest.mark.parametrize("s", [2, 3, 8, 10, 64])
def test_div_jitter_f64(checker, s):
    checked, bad = run(checker, "f64", "jitter", s, 2_000_000, s)
    assert bad == 0


@pytest.mark.parametrize("b", ["1024", "4096", "800", "600", "320", "35.123"])
def test_div_sweep_f32(checker, b):
    checked, bad = run(checker, "f32", "sweep", b, -1, 13)  # px in [0.5, 8192): every binary32 value
    assert checked == 14 * 2 ** 23 and bad == 0


def test_normalize_rcp_f32(checker):
    """rt_normalize3 (the camera's normalize_rcp) == three divisions by the length, bit for bit,
    including vectors with zero, -0, subnormal, tiny and huge components (the
    Markstein quotient needs a normal numerator and quotient; such vectors take the divisions)."""
    checked, bad = run(checker, "f32", "norm", 5_000_000, 3)
    assert checked == 5_000_000 and bad == 0
