"""Direct comparison with the REFERENCE's own renders (tests/golden/ref/*.f32: the compiled
reference, std::mt19937 seeded 42) -- SURVEY.md 8(c) parity chain items (3) and (4).

The GPU path uses the counter RNG, so it can equal the reference
pixel-for-pixel only where no random number is drawn:
  * deterministic configurations (s = 1, no soft shadow / glossy / DOF / motion blur):
    bit-identical float framebuffer;
  * stochastic configurations: the image mean of every channel within STAT_TOL (relative
    to the brightest channel mean).  Calibrated on the oracle (== GPU bit for bit in counter
    mode) over seeds 1..5: worst case 1.8 % on the 32x32 soup_s3 fixture.
The CPU half runs the oracle (counter mode) against the same fixtures; the GPU half runs
librt_hip.so.  blend_c3_s10 / blend_c4_s10 are the C3 / C4 bench settings (100 spp; C4 with
4 soft-shadow samples) at 128^2 (SURVEY.md 8(c) item (4) at 100 spp), held to tighter bars.
"""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
import scenes

SEED = 20251226
STAT_TOL = 0.03
# 100-spp cases (C3 / C4 at the bench's -s 10, C4 with -light_sample 4): tighter bars, both
# calibrated on the oracle over seeds 1, 2, 3, 20251226 -- channel-mean deviation at most
# 2.1e-5 (C3) / 3.6e-4 (C4), per-pixel RMS deviation relative to the reference's mean 0.18 %
# (C3) / 2.4 % (C4: glossy reflections and soft shadows stay noisy per pixel at 100 spp).
STAT_TOL_100SPP = 0.002
PIXEL_RMS_TOL = {"blend_c3_s10": 0.005, "blend_c4_s10": 0.04}
DETERMINISTIC = ["ascii_k1_bvh", "ascii_primary", "soup_linear", "soup_s1", "blend_test3"]
STOCHASTIC = ["ascii_glossy_bvh", "ascii_glossy_s2_linear", "ascii_textured", "features_dof", "features_linear",
              "features_s1", "features_s2_ls3", "soup_s3", "blend_c3_antialiasing", "blend_c4_glossy_soft",
              "blend_distributed", "blend_dop", "blend_motion_blur", "blend_test1", "blend_c3_s10", "blend_c4_s10"]

MAN = json.load(open(os.path.join(scenes.GOLDEN, "manifest.json")))


def reference_image(name):
    v = MAN["cases"][name]
    return np.fromfile(os.path.join(scenes.GOLDEN, "ref", name + ".f32"), dtype=np.float32).reshape(
        v["height"], v["width"], 3)


def check(name, img):
    ref = reference_image(name)
    assert img.shape == ref.shape
    if name in DETERMINISTIC:
        bad = int((img.view(np.uint32) != ref.view(np.uint32)).sum())
        assert bad == 0, f"{name}: {bad} channels differ from the reference"
    else:
        m_img = img.reshape(-1, 3).astype(np.float64).mean(0)
        m_ref = ref.reshape(-1, 3).astype(np.float64).mean(0)
        rel = np.abs(m_img - m_ref).max() / m_ref.max()
        tol = STAT_TOL_100SPP if name in PIXEL_RMS_TOL else STAT_TOL
        assert rel <= tol, f"{name}: channel means {m_img} vs reference {m_ref} (rel {rel:.4f})"
        if name in PIXEL_RMS_TOL:
            rms = float(np.sqrt(((img.astype(np.float64) - ref) ** 2).mean()) / ref.mean())
            assert rms <= PIXEL_RMS_TOL[name], f"{name}: per-pixel RMS deviation {rms:.4f} of the reference mean"


@pytest.mark.parametrize("name", DETERMINISTIC + STOCHASTIC)
def test_oracle_counter_vs_reference(name, tmp_path):
    path, args = scenes.materialise(name, str(tmp_path))
    img, _, _ = ob.render(path, rng=ob.RNG_COUNTER, seed=SEED, texture_root=scenes.TEXTURES, **args)
    check(name, img)


@pytest.mark.gpu
@pytest.mark.parametrize("name", DETERMINISTIC + STOCHASTIC)
def test_gpu_vs_reference(name, tmp_path, gpu):
    import ray_tracying_amd as rt
    path, args = scenes.materialise(name, str(tmp_path))
    sc = rt.Scene(path, texture_root=scenes.TEXTURES)
    try:
        img, _ = sc.render(rt.RenderParams(spp_sqrt=args["spp_sqrt"], light_samples=args["light_samples"],
                                           use_bvh=args["use_bvh"], seed=SEED))
    finally:
        sc.close()
    check(name, img)
