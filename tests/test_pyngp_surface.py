"""The pyngp driver surface the reference scripts call (scripts/run.py, run_dynamic.py; src/python_api.cu:216-600),
checked on the CPU: every attribute those scripts touch exists on the mirror, the module-level enums and
BoundingBox, the tonemap restatement (render_buffer.cu:254-334, 474-500) against hand-evaluated values, the camera
conventions (set_nerf_camera_matrix, fov <-> relative focal length) and the loss-target options in the oracle
(testbed_nerf.cu:1642-1671). The device side of the same options is tests/test_gpu_parity.py."""
import math

import numpy as np
import pytest

from neus2_amd import pyngp

# run.py / run_dynamic.py: methods and properties read from a Testbed (instance attributes set in __init__ are
# checked by test_gpu_* through a real testbed)
RUN_PY_TESTBED = [
    "load_training_data", "load_snapshot", "reload_network_from_file", "compute_and_save_marching_cubes_mesh",
    "init_window", "frame", "want_repl", "training_step", "loss", "ek_loss", "mask_loss", "save_snapshot",
    "background_color", "color_space", "fov", "set_nerf_camera_matrix", "render", "set_camera_to_training_view",
    "change_to_frame", "prepare_for_test", "save_transform", "training_network_next_frame",
    "current_training_time_frame", "all_training_time_frame", "first_frame_max_training_step",
    "next_frame_max_training_step", "compute_marching_cubes_mesh", "reset_camera", "camera_matrix", "fov_xy",
    "screen_center", "n_params", "n_encoding_params", "train",
]


def test_run_scripts_surface_exists():
    for name in RUN_PY_TESTBED:
        assert hasattr(pyngp.Testbed, name), name
    for name in ("random_bg_color", "near_distance", "linear_colors", "n_images_for_training", "dataset", "transforms"):
        assert hasattr(pyngp._Training, name) or name == "dataset", name
    assert hasattr(pyngp._Nerf, "cone_angle_constant")
    assert {m.name for m in pyngp.ColorSpace} == {"Linear", "SRGB"}
    assert [m.name for m in pyngp.TonemapCurve] == ["Identity", "ACES", "Hable", "Reinhard"]
    assert pyngp.TestbedMode.Nerf == 0


def test_bounding_box():
    """run_dynamic.py builds ngp.BoundingBox(min, max) for the mesh aabb; the default box is empty."""
    assert pyngp.BoundingBox().is_empty()
    assert pyngp._aabb_pair(pyngp.BoundingBox()) is None
    bb = pyngp.BoundingBox(np.array([0, 0.1, 0]), np.array([1.0, 0.9, 1.0]))
    lo, hi = pyngp._aabb_pair(bb)
    np.testing.assert_array_equal(lo, np.float32([0, 0.1, 0]))
    np.testing.assert_array_equal(hi, np.float32([1, 0.9, 1]))
    assert bb.contains([0.5, 0.5, 0.5]) and not bb.contains([0.5, 0.95, 0.5])
    np.testing.assert_allclose(bb.center(), [0.5, 0.5, 0.5])
    assert bb.get_vertices().shape == (8, 3)
    bb.inflate(0.1)
    np.testing.assert_allclose(bb.min, [-0.1, 0.0, -0.1], atol=1e-7)
    assert pyngp._aabb_pair(((0, 0, 0), (1, 1, 1)))[1].dtype == np.float32


def _aces(x):
    a, b, c, d, e = 0.36 * 2.51, 0.6 * 0.03, 0.0, 0.36 * 2.43, 0.6 * 0.59
    return (x * x * a + b * x + c) / (d * x * x + e * x + 0.14)


def _hable(x):
    A, B, C, D, E, F = 0.15, 0.50, 0.10, 0.20, 0.02, 0.30
    k0, k1, k3, k4, k5 = A * F - A * E, C * B * F - B * E, A * F, B * F, D * F * F
    W = 11.2
    ws = (k3 * W * W + k4 * W + k5) / (k0 * W * W + k1 * W)
    return (x * x * 4 * k0 * ws + 2 * k1 * ws * x) / (4 * k3 * x * x + 2 * k4 * x + k5)


def test_tonemap_curves_match_formulas():
    x = np.linspace(-0.5, 4.0, 37, dtype=np.float32).reshape(-1, 1).repeat(3, 1)
    x[:, 1] *= 0.5
    xp = np.maximum(x.astype(np.float64), 0)
    np.testing.assert_array_equal(pyngp.tonemap_curve(x, pyngp.TonemapCurve.Identity), x)
    np.testing.assert_allclose(pyngp.tonemap_curve(x, pyngp.TonemapCurve.ACES), _aces(xp), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(pyngp.tonemap_curve(x, pyngp.TonemapCurve.Hable), _hable(xp), rtol=2e-6, atol=1e-7)
    Y = xp @ np.array([0.2126, 0.7152, 0.0722])
    np.testing.assert_allclose(pyngp.tonemap_curve(x, pyngp.TonemapCurve.Reinhard), xp / (Y[:, None] + 1), rtol=2e-6, atol=1e-7)


def test_tonemap_image_background_and_spaces():
    """tonemap_kernel: weight = (1 - a) * bg.a added to rgb (bg sRGB -> linear unless the colour space is SRGB)
    and to alpha; SRGB colour space -> linear before the exposure 2^e; sRGB output for render(linear=False)."""
    rng = np.random.default_rng(0)
    acc = rng.uniform(0, 1, (5, 7, 4)).astype(np.float32)
    acc[..., :3] *= acc[..., 3:4]
    bg = np.float32([0.8, 0.4, 0.1, 0.75])
    bgl = pyngp.srgb_to_linear(bg[:3].astype(np.float64))
    w = (1 - acc[..., 3:4].astype(np.float64)) * 0.75
    exp_rgb = (acc[..., :3] + bgl * w) * 2.0 ** 0.5
    out = pyngp.tonemap_image(acc, 0.5, bg, pyngp.ColorSpace.Linear, pyngp.TonemapCurve.Identity, to_srgb=False)
    np.testing.assert_allclose(out[..., :3], exp_rgb, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out[..., 3:], acc[..., 3:] + w, rtol=1e-6, atol=1e-7)
    out = pyngp.tonemap_image(acc, 0.0, bg, pyngp.ColorSpace.SRGB, pyngp.TonemapCurve.Identity, to_srgb=True)
    comp = acc[..., :3] + bg[:3].astype(np.float64) * w
    np.testing.assert_allclose(out[..., :3], pyngp.linear_to_srgb(pyngp.srgb_to_linear(comp)), rtol=1e-5, atol=1e-6)
    # defaults of render(): transparent black background, Linear, Identity -> unchanged
    np.testing.assert_array_equal(pyngp.tonemap_image(acc, 0.0, (0, 0, 0, 0)), acc)


def test_camera_conventions():
    """set_nerf_camera_matrix = dataset.nerf_matrix_to_ngp (testbed.cu:238-240, nerf_loader.h:112-134);
    fov <-> relative focal length (testbed.cu:1830-1844)."""
    m = np.array([[0.0, 0.0, 1.0, 2.0], [1.0, 0.0, 0.0, -1.0], [0.0, 1.0, 0.0, 0.5], [0, 0, 0, 1]], np.float32)
    r = pyngp.nerf_matrix_to_ngp(m, 0.33, np.float32([0.5, 0.5, 0.5]), False)
    # columns 1, 2 flipped, translation scaled + offset, rows cycled (y, z, x)
    exp = m[:3, :4].copy()
    exp[:, 1] *= -1
    exp[:, 2] *= -1
    exp[:, 3] = exp[:, 3] * np.float32(0.33) + 0.5
    np.testing.assert_array_equal(r, exp[[1, 2, 0]])
    rna = pyngp.nerf_matrix_to_ngp(m, 1.0, np.zeros(3, np.float32), True)
    np.testing.assert_array_equal(rna[:, :3], m[:3, :3])
    fl = pyngp.fov_to_focal_length(1, 50.625)
    assert abs(2 * math.atan(0.5 / fl) * 180 / math.pi - 50.625) < 1e-9
    assert abs(pyngp.fov_to_focal_length(800, 90.0) - 400.0) < 1e-9


def _const_dataset(O, rgba):
    img = np.zeros((6, 8, 4), np.uint8)
    img[...] = rgba
    xf = np.float32([[1, 0, 0, 0.5], [0, 1, 0, 0.5], [0, 0, 1, -1.0]])
    return O.Dataset([img, img], np.float32([[8, 8], [8, 8]]), np.float32([[0.5, 0.5], [0.5, 0.5]]), np.stack([xf, xf]))


def test_oracle_loss_targets_options():
    """The oracle's loss target (testbed_nerf.cu:1642-1671) for a constant RGBA image, per option: random
    background (default), fixed background x {Linear colour space, SRGB colour space, linear_colors}."""
    import oracle as O
    rgba = (200, 100, 50, 128)
    ds = _const_dataset(O, rgba)
    a = rgba[3] / 255.0
    tex = pyngp.srgb_to_linear(np.array(rgba[:3]) / 255.0) * a  # read_rgba: premultiplied linear
    s2l, l2s = pyngp.srgb_to_linear, pyngp.linear_to_srgb
    bg = np.array([0.9, 0.3, 0.6])
    expect = {
        0: (l2s(tex + (1 - a) * s2l(bg)), l2s(s2l(bg))),
        1: (l2s(tex / a) * a + (1 - a) * l2s(s2l(bg)), l2s(s2l(bg))),
        2: (tex + (1 - a) * s2l(bg), s2l(bg)),
    }
    rs, ri = 0x1234, 0xDA3E39CB94B95BDB | 1
    for mode, (t_exp, bg_exp) in expect.items():
        ds.set_target(bg, mode)
        for ray in (0, 5, 77):
            t, b = O.ray_target(ds, ray, 128, 0, rs, ri)
            np.testing.assert_allclose(t, t_exp, rtol=2e-5, atol=2e-6)
            np.testing.assert_allclose(b, bg_exp, rtol=2e-5, atol=2e-6)
    ds.set_target(None, 0)
    bgs = [tuple(O.ray_target(ds, ray, 128, 0, rs, ri)[1]) for ray in range(8)]
    assert len(set(bgs)) == 8  # a random background per ray


def test_ctypes_options_struct_matches_header():
    import ctypes as C
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "neus2_hip.h")).read()
    body = re.search(r"typedef struct NeusTrainingOptions \{(.*?)\} NeusTrainingOptions;", hdr, re.S).group(1)
    names = re.findall(r"(\w+)(?:\[\d+\])?;", body)
    assert names == [f for f, _ in pyngp._lib.NeusTrainingOptions._fields_]
    assert C.sizeof(pyngp._lib.NeusTrainingOptions) == 36


@pytest.mark.parametrize("val", [True])
def test_training_snap_to_pixel_centers_rejected(val):
    class _Tb:
        pass
    tr = pyngp._Training(_Tb())
    assert tr.snap_to_pixel_centers is False
    with pytest.raises(pyngp.NeusError):
        tr.snap_to_pixel_centers = val


class _RecordingLib:
    """Stand-in for libneus2_hip.so on the CPU: answers the C-ABI calls the pyngp mirror makes with plausible
    values and records the arguments (training steps, options, render requests)."""

    def __init__(self):
        self.step = 0
        self.calls = []
        self.options = pyngp._lib.NeusTrainingOptions()
        self.options.random_bg_color = 1
        self.renders = []

    def __getattr__(self, name):
        if not name.startswith("neus_"):
            raise AttributeError(name)

        def call(*args):
            self.calls.append(name)
            return 0
        return call

    def neus_testbed_create(self, dev, h):
        self.calls.append("neus_testbed_create")
        h._obj.value = 0x1000
        return 0

    def neus_testbed_layout(self, h, l):
        o = l._obj
        o.n_params, o.n_density, o.n_rgb, o.grid_offset, o.n_grid_params, o.variance_offset, o.n_matrix = 64, 16, 16, 32, 24, 56, 32
        o.per_level_scale, o.n_levels = 1.5, 14
        return 0

    def neus_testbed_get_stats(self, h, s):
        s._obj.training_step = self.step
        s._obj.loss = 1.0 / (1 + self.step)
        return 0

    def neus_testbed_train(self, h, n):
        self.step += n.value
        self.calls.append("neus_testbed_train")
        return 0

    def neus_testbed_get_training_options(self, h, o):
        C.memmove(C.addressof(o._obj), C.addressof(self.options), C.sizeof(self.options))
        return 0

    def neus_testbed_set_training_options(self, h, o):
        C.memmove(C.addressof(self.options), C.addressof(o._obj), C.sizeof(self.options))
        self.calls.append("neus_testbed_set_training_options")
        return 0

    def neus_testbed_render(self, h, rq, out, it):
        r = rq._obj
        self.renders.append(dict(width=r.width, height=r.height, spp=r.spp, view=r.training_view, xform=list(r.xform),
                                 focal=list(r.focal), sc=list(r.screen_center), snap=r.snap_to_pixel_centers,
                                 min_t=r.min_transmittance))
        C.memset(out, 0, r.width * r.height * 16)
        return 0


import ctypes as C  # noqa: E402


def test_run_py_sequence_through_the_module(tmp_path, monkeypatch):
    """scripts/run.py's training + evaluation call sequence (tests/run_sequence.py) through the pyngp mirror, with
    the C library replaced by a recorder: the frame() loop trains exactly n_steps, the nerf-compatibility options
    reach the device (color space SRGB, cone angle 0, near distance), the snapshot and mesh files are written, and
    every evaluation render carries the camera run.py sets (set_nerf_camera_matrix -> nerf_matrix_to_ngp,
    fov_axis 0: focal = fov_to_focal_length(1, camera_angle_x) * width, screen centre 0.5, pixel centres,
    min transmittance 1e-4) with the black background composited (alpha 1)."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from run_sequence import run_py_sequence
    from neus2_amd import scenes
    fake = _RecordingLib()
    monkeypatch.setattr(pyngp, "lib", lambda: fake)
    sc = scenes.small_scene(n_views=4, width=32, height=24)
    scene_json = scenes.write_transforms(sc, str(tmp_path / "scene"))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = run_py_sequence(pyngp, scene_json, os.path.join(root, "configs", "nerf", "base.json"), str(tmp_path / "out"), n_steps=6,
                        test_transforms=scene_json, spp=2)
    assert r["steps"] == 6 and fake.calls.count("neus_testbed_train") == 6
    assert fake.options.color_space == 1 and fake.options.cone_angle_constant == 0.0 and fake.options.random_bg_color == 1
    assert os.path.exists(r["snapshot"]) and os.path.exists(r["mesh"])
    assert len(fake.renders) == 4 and len(r["psnr"]) == 4
    tt = json.load(open(scene_json))
    fl = pyngp.fov_to_focal_length(1, tt["camera_angle_x"] * 180 / math.pi) * 32
    for rq, fr in zip(fake.renders, tt["frames"]):
        assert rq["view"] == -1 and rq["spp"] == 2 and rq["snap"] == 1 and abs(rq["min_t"] - 1e-4) < 1e-9
        np.testing.assert_allclose(rq["focal"], [fl, fl], rtol=1e-6)
        np.testing.assert_allclose(rq["sc"], [0.5, 0.5])
        exp = pyngp.nerf_matrix_to_ngp(np.array(fr["transform_matrix"], np.float32)[:3], 0.33, np.float32([0.5] * 3), False)
        np.testing.assert_allclose(np.array(rq["xform"]).reshape(3, 4), exp, atol=1e-6)
    # the written cameras round-trip to the scene's ngp cameras (the focal above is the scene's own)
    np.testing.assert_allclose(np.array(fake.renders[1]["xform"]).reshape(3, 4), sc["xforms"][1], atol=1e-5)
    assert abs(fl - sc["focal"][0][0]) < 1e-3
    tb = r["testbed"]
    assert tb.background_color[3] == 1.0
    img = tb.render(8, 6)
    np.testing.assert_array_equal(img[..., 3], 1.0)  # empty accumulation + opaque black background
    tb._h = None  # the recorder owns no device testbed
