"""Host-side logic on the CPU: configs/nerf/*.json parsing, the transforms.json loader and camera
conversion (nerf_loader.h:112-134, nerf_loader.cu:197-751), the synthetic scenes and occupancy
bitfields used by the bench, and the CPU train-step composer."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_base_config_values():
    from neus2_amd import config
    cfg = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    c = config.network_config(cfg)
    assert (c.n_levels, c.n_features_per_level, c.log2_hashmap_size, c.base_resolution) == (14, 2, 19, 16)
    assert c.top_resolution == 2048 and c.n_neurons == 64 and c.n_density_hidden == 1 and c.n_rgb_hidden == 2
    assert abs(c.learning_rate - 1e-3) < 1e-9 and abs(c.beta2 - 0.99) < 1e-7 and c.epsilon == pytest.approx(1e-15)
    assert c.l2_reg == pytest.approx(1e-6) and c.ema_decay == pytest.approx(0.95)
    assert (c.decay_start, c.decay_interval) == (20000, 10000) and c.decay_base == pytest.approx(0.33)
    assert c.batch_size == 1 << 18 and c.ek_loss_weight == pytest.approx(0.01) and c.anneal_end == 0
    assert config.density_input_width(14) == 32 and config.density_input_width(16) == 48


def test_config_comments_and_parent(tmp_path):
    from neus2_amd import config
    (tmp_path / "p.json").write_text('{"encoding": {"n_levels": 8, "log2_hashmap_size": 17}, // c\n "x": "a//b"}')
    (tmp_path / "c.json").write_text('/* block */ {"parent": "p.json", "encoding": {"n_levels": 4}}')
    cfg = config.load_json(str(tmp_path / "c.json"))
    assert cfg["encoding"] == {"n_levels": 4, "log2_hashmap_size": 17} and cfg["x"] == "a//b"
    with pytest.raises(ValueError):
        config.network_config({"loss": {"otype": "L2"}})


def test_nerf_matrix_to_ngp():
    from neus2_amd.pyngp import nerf_matrix_to_ngp
    m = np.eye(4, dtype=np.float32)
    m[:3, 3] = [1, 2, 3]
    r = nerf_matrix_to_ngp(m, 0.5, [0.5, 0.5, 0.5], from_na=True)
    np.testing.assert_allclose(r[:, 3], [1.0, 1.5, 2.0])
    np.testing.assert_allclose(r[:, :3], np.eye(3))
    r2 = nerf_matrix_to_ngp(m, 0.33, [0.5, 0.5, 0.5], from_na=False)
    # NeRF -> ngp: flip y/z columns, then cycle rows (x, y, z) -> (y, z, x)
    np.testing.assert_allclose(r2[:, 3], np.array([2, 3, 1]) * 0.33 + 0.5, rtol=1e-6)


def test_load_transforms(tmp_path):
    from PIL import Image
    from neus2_amd.pyngp import load_transforms
    img = np.zeros((12, 16, 4), np.uint8)
    img[..., 0] = 200
    img[..., 3] = 255
    Image.fromarray(img).save(tmp_path / "a.png")
    m = np.eye(4).tolist()
    js = {"from_na": True, "w": 16, "h": 12, "aabb_scale": 1, "scale": 0.5, "offset": [0.5, 0.5, 0.5],
          "frames": [{"file_path": "a.png", "transform_matrix": m, "intrinsic_matrix": [[20, 0, 8], [0, 21, 6], [0, 0, 1]]},
                     {"file_path": "a", "transform_matrix": m}], "fl_x": 30.0}
    (tmp_path / "transforms.json").write_text(json.dumps(js))
    d = load_transforms(str(tmp_path / "transforms.json"))
    assert len(d["images"]) == 2 and d["images"][0].shape == (12, 16, 4)
    np.testing.assert_allclose(d["focal"][0], [30.0, 30.0])   # fl_x takes precedence over the intrinsic matrix
    np.testing.assert_allclose(d["xforms"][0][:, 3], [0.5, 0.5, 0.5])
    js["frames"][0].pop("intrinsic_matrix")
    del js["fl_x"]
    js["frames"] = [dict(js["frames"][0], intrinsic_matrix=[[20, 0, 8], [0, 21, 6], [0, 0, 1]])]
    (tmp_path / "transforms.json").write_text(json.dumps(js))
    d = load_transforms(str(tmp_path / "transforms.json"))
    np.testing.assert_allclose(d["focal"][0], [20.0, 21.0])
    np.testing.assert_allclose(d["principal"][0], [0.5, 0.5])


def test_shell_bitfield_structure():
    from neus2_amd import scenes
    bf = scenes.shell_bitfield()
    G3 = 128 ** 3
    assert bf.size == G3 // 8 * 8
    lvl0 = np.unpackbits(bf[: G3 // 8], bitorder="little")
    frac = lvl0.mean()
    # shell of radius 0.25, half-thickness 2/128: volume 4 pi r^2 * 2t ~ 0.0245 of the unit cube
    assert 0.015 < frac < 0.035, frac
    # max-pooled mips: every coarser level covers the finer one (mip 1 centre region non-empty)
    assert np.unpackbits(bf[G3 // 8: 2 * G3 // 8]).sum() > 0


def test_sphere_scene_geometry():
    from neus2_amd import scenes
    sc = scenes.small_scene(n_views=4, width=32, height=24)
    assert len(sc["images"]) == 4 and sc["images"][0].shape == (24, 32, 4)
    a = np.stack(sc["images"])[..., 3]
    assert 0.05 < (a > 0).mean() < 0.95  # the sphere is in view and does not fill it
    for M in sc["xforms"]:
        c = M[:, 3]
        fwd = M[:, 2]
        to_centre = np.array([0.5, 0.5, 0.5]) - c
        assert np.dot(fwd, to_centre / np.linalg.norm(to_centre)) > 0.99  # cameras look at the centre


def test_cpu_trainer_step_counters():
    """The CPU composition of Testbed::train (oracle/cpu_step.py) runs and adapts R like
    Counters::update_after_training (testbed_nerf.cu:3399-3438)."""
    import oracle as O
    from cpu_step import CpuTrainer
    from neus2_amd import scenes
    sc = scenes.small_scene(n_views=4, width=32, height=24)
    cfg = O.make_cfg(n_levels=2, log2_hashmap_size=12, base_resolution=8, per_level_scale=2.0)
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    tr = CpuTrainer(cfg, ds, O.init_params(cfg), batch=512, rays_per_batch=512)
    p0 = tr.params.copy()
    tr.step()
    assert tr.training_step == 1 and tr.adam_step == 1
    meas = tr.last["compacted"]
    assert meas > 0
    r = int(np.float32(512) * np.float32(512) / np.float32(meas))
    assert tr.R == min((r + 127) // 128 * 128, 1 << 18)
    assert not np.array_equal(tr.params, p0)


def test_eval_psnr_matches_render_utils_formula():
    """pyngp.eval_psnr restates render_img_training_view's metric (render_utils.py:252-359): the 8-bit
    reference (sRGB, alpha) premultiplied in linear space, re-composited on a black background in sRGB,
    PSNR = mse2psnr(mean((clip(srgb(pred)) - clip(srgb(gt)))^2))."""
    import numpy as np
    from neus2_amd import pyngp
    rng = np.random.default_rng(0)
    rgba8 = rng.integers(0, 256, (6, 5, 4)).astype(np.uint8)
    s = rgba8[..., :3] / 255.0
    a = rgba8[..., 3:4] / 255.0
    gt_srgb = s * a  # black background: sRGB colour times alpha
    pred = pyngp.srgb_to_linear(np.clip(gt_srgb + 0.05, 0, 1)).astype(np.float32)
    pred = np.concatenate([pred, a.astype(np.float32)], -1)
    psnr, mse = pyngp.eval_psnr(pred, rgba8)
    want = np.mean((np.clip(gt_srgb + 0.05, 0, 1) - gt_srgb) ** 2)
    assert abs(mse - want) < 1e-6
    assert abs(psnr - (-10 * np.log10(want))) < 1e-3
    exact = np.concatenate([pyngp.srgb_to_linear(gt_srgb), a], -1).astype(np.float32)
    assert pyngp.eval_psnr(exact, rgba8)[0] > 60
