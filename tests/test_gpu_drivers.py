"""The reference drivers' call sequences on the MI355X through the pyngp mirror (tests/run_sequence.py):
scripts/run.py (train from a transforms.json on disk, snapshot, mesh, test-transforms evaluation through
set_nerf_camera_matrix + fov) and scripts/run_dynamic.py (per-frame snapshots / save_transform / meshes while
frame() walks the sequence, then the --dynamic_test pass: change_to_frame, load_snapshot, prepare_for_test)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _record(test, **metrics):
    import json
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "parity_metrics.jsonl"), "a") as f:
        f.write(json.dumps({"test": test, **{k: float(v) for k, v in metrics.items()}}) + "\n")


def _config(tmp_path, **hyper):
    import json
    from neus2_amd import config
    cfg = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    cfg["hyperparams"].update(hyper)
    p = tmp_path / "net.json"
    p.write_text(json.dumps(cfg))
    return str(p)


def test_run_py_sequence(tmp_path, torch_cuda):
    """run.py on the 64x48 sphere written to disk: 300 steps through frame(), the snapshot reloads to the same
    renders, the mesh file is non-empty, and the test-transforms PSNR (black background, pixel centres, spp 1) is
    that of a trained model. (--nerf_compatibility's SRGB colour space converts the network colour to linear twice on
    render in the reference - shade_kernel_nerf and tonemap_kernel - so its PSNR is not a quality measure; the loss
    targets of that mode are checked in test_gpu_parity.test_loss_target_options_parity.)"""
    from neus2_amd import pyngp, scenes
    from run_sequence import run_py_sequence
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    scene_json = scenes.write_transforms(sc, str(tmp_path / "scene"))
    net = _config(tmp_path)
    r = run_py_sequence(pyngp, scene_json, net, str(tmp_path / "out"), n_steps=300, test_transforms=scene_json, spp=1,
                        nerf_compatibility=False)
    tb = r["testbed"]
    assert r["steps"] == 300 and tb.color_space == pyngp.ColorSpace.Linear and tb.nerf.cone_angle_constant == 0.0
    assert all(np.isfinite(l[1]) for l in r["losses"])
    assert r["losses"][-1][1] < r["losses"][0][1]
    psnr = float(np.mean(r["psnr"]))
    _record("run_py_sequence", psnr=psnr, psnr_min=min(r["psnr"]), loss=r["losses"][-1][1])
    assert psnr > 24.0, r["psnr"]
    assert os.path.getsize(r["mesh"]) > 1000
    # load_snapshot into a fresh testbed on the same data renders the same image (EMA weights + grid restored)
    tb2 = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb2.load_training_data(scene_json)
    tb2.load_snapshot(r["snapshot"])
    for t in (tb, tb2):
        t.background_color = [0.0, 0.0, 0.0, 1.0]
        t.snap_to_pixel_centers = True
        t.set_camera_to_training_view(2)
    a, b = tb.render(64, 48, 1), tb2.render(64, 48, 1)
    assert np.abs(a - b).mean() < 2e-3, np.abs(a - b).mean()


def test_run_dynamic_sequence(tmp_path, torch_cuda):
    """run_dynamic.py on a 2-frame sequence (the sphere moved by +0.02 x in frame 1), 150 + 100 steps per frame
    (global-movement phase 50): each frame's last step writes its snapshot, transform and mesh; the transform file
    has the reference's layout (3 rotation rows, the translation, a blank line), frame 1's translation points back
    (t_x < 0); the --dynamic_test pass restores every frame from its snapshot, uses the DeltaNetwork on frame 1
    (prepare_for_test) and reproduces the training-time PSNR."""
    from neus2_amd import pyngp, scenes
    from run_sequence import run_dynamic_sequence
    frames = scenes.dynamic_scene(n_frames=2, shift=(0.02, 0.0, 0.0))
    d = tmp_path / "seq"
    for k, fr in enumerate(frames):
        scenes.write_transforms(fr, str(d), name=f"frame_{k:03d}.json")
    net = _config(tmp_path, first_frame_max_training_step=150, next_frame_max_training_step=100,
                  predict_global_movement_training_step=50)
    r = run_dynamic_sequence(pyngp, str(d), net, str(tmp_path / "out"))
    assert r["frames_seen"] == [0, 1]
    rows = r["transforms"][1].split("\n")
    assert len(rows) == 6 and rows[4] == "" and rows[5] == ""
    R = np.array([[float(v) for v in rows[i].split()] for i in range(3)])
    t = np.array([float(v) for v in rows[3].split()])
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=5e-3)
    assert t[0] < 0, t
    rows0 = r["transforms"][0].split("\n")
    np.testing.assert_allclose(np.array([[float(v) for v in rows0[i].split()] for i in range(3)]), np.eye(3), atol=1e-6)
    assert r["use_delta"] == [False, True]
    _record("run_dynamic_sequence", psnr_f0=r["train_psnr"][0], psnr_f1=r["train_psnr"][1], test_f0=r["test_psnr"][0],
            test_f1=r["test_psnr"][1], t_x=t[0])
    assert min(r["train_psnr"]) > 20.0, r["train_psnr"]
    for a, b in zip(r["train_psnr"], r["test_psnr"]):
        assert abs(a - b) < 0.5, (r["train_psnr"], r["test_psnr"])


def test_snapshot_optimizer_state_round_trip(tmp_path, torch_cuda):
    """save_snapshot(include_optimizer_state=True) -> load_snapshot restores the Ema(ExponentialDecay(Adam)) state
    exactly (moments, per-parameter steps, current step, EMA weights; trainer.h:281-305) and training continues
    from it: the next step's Adam update uses the restored moments (step count carries on)."""
    from neus2_amd import pyngp, scenes
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
    tb.train_steps(40)
    p = str(tmp_path / "s.msgpack")
    tb.save_snapshot(p, include_optimizer_state=True)
    o = tb.get_optimizer_state()
    tb2 = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb2.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb2.load_snapshot(p)
    o2 = tb2.get_optimizer_state()
    assert o2["current_step"] == o["current_step"] == 40
    for k in ("m1", "m2", "param_steps"):
        np.testing.assert_array_equal(o2[k], o[k])
    np.testing.assert_array_equal(o2["ema"].view(np.uint16), o["ema"].view(np.uint16))
    np.testing.assert_array_equal(tb2.get_half_params(inference=True).view(np.uint16), o["ema"].view(np.uint16))
    tb2.train_steps(1)
    o3 = tb2.get_optimizer_state()
    assert o3["current_step"] == 41 and int(o3["param_steps"].max()) == int(o["param_steps"].max()) + 1
    # without the optimizer state the reload starts a fresh Adam
    tb3 = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb3.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    p2 = str(tmp_path / "s2.msgpack")
    tb.save_snapshot(p2)
    tb3.load_snapshot(p2)
    assert tb3.get_optimizer_state()["current_step"] == 0 and not tb3.get_optimizer_state()["m1"].any()


def test_zero_sample_and_nonfinite_guards(torch_cuda):
    """The zero-sample guard (testbed_nerf.cu:3542-3548): cameras that look away from the aabb give no training
    samples -> loss scalars 0, training_aborted, and frame() stops training. A NaN in the colour network -> the
    logged loss sum is non-finite -> nonfinite_loss and training_aborted (SURVEY §5 health flag)."""
    import warnings
    from neus2_amd import pyngp, scenes
    sc = scenes.small_scene(n_views=4, width=32, height=24)
    away = []
    for k in range(4):
        m = np.zeros((3, 4), np.float32)
        m[:, 0], m[:, 1], m[:, 2] = (1, 0, 0), (0, -1, 0), (0, 0, 1)  # looking along +z
        m[:, 3] = (0.5 + 0.1 * k, 0.5, 3.0)                            # from beyond z = 1
        away.append(m)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], away, 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        assert tb.frame() is True
    st = tb.stats()
    assert st["measured_batch_size"] == 0 and st["training_aborted"] == 1 and st["loss"] == 0.0
    assert tb.shall_train is False and tb.frame() is False
    tb2 = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb2.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb2.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
    tb2.train_steps(1)
    assert tb2.stats()["training_aborted"] == 0 and tb2.stats()["nonfinite_loss"] == 0
    p = tb2.get_params()
    lay = tb2.layout()
    p[lay["n_density"]:lay["n_matrix"]] = np.nan
    tb2.set_params(p)
    tb2.train_steps(16)  # the next logged step (every 16th)
    st2 = tb2.stats()
    assert st2["nonfinite_loss"] == 1 and st2["training_aborted"] == 1
