"""The call sequence of the reference's training driver (scripts/run.py:109-345: construct, load the scene, load the
network config, the frame() loop until n_steps, save_snapshot, compute_and_save_marching_cubes_mesh, then the
test-transforms evaluation: black background, pixel-centre sampling, min transmittance 1e-4, fov from
camera_angle_x on axis 0, set_nerf_camera_matrix + render per view, PSNR of clip(srgb) images), written against the
pyngp module API so that tests can drive it through the mirror: tests/test_pyngp_surface.py on the CPU with a
recording stand-in for the C library, tests/test_gpu_drivers.py on the MI355X. Not the reference's script."""
import json
import math
import os

import numpy as np


def run_py_sequence(ngp, scene_json, network, out_dir, n_steps, test_transforms=None, spp=1, mesh_res=32,
                    nerf_compatibility=True, near_distance=0.0):
    res = {"losses": [], "psnr": []}
    testbed = ngp.Testbed(ngp.TestbedMode.Nerf)
    testbed.nerf.sharpen = 0.0
    testbed.load_training_data(scene_json)
    testbed.reload_network_from_file(network)
    testbed.shall_train = True
    testbed.nerf.render_with_camera_distortion = True
    if near_distance >= 0.0:
        testbed.nerf.training.near_distance = near_distance
    if nerf_compatibility:
        testbed.color_space = ngp.ColorSpace.SRGB
        testbed.nerf.cone_angle_constant = 0
    while testbed.frame():
        if testbed.want_repl():
            raise RuntimeError("no REPL")
        if testbed.training_step >= n_steps:
            break
        if testbed.training_step % 2 == 0:
            res["losses"].append((testbed.training_step, testbed.loss, testbed.ek_loss, testbed.mask_loss))
    res["steps"] = testbed.training_step
    snap = os.path.join(out_dir, "checkpoints", f"{n_steps}.msgpack")
    os.makedirs(os.path.dirname(snap), exist_ok=True)
    testbed.save_snapshot(snap, False)
    mesh = os.path.join(out_dir, "mesh", f"{n_steps}.obj")
    os.makedirs(os.path.dirname(mesh), exist_ok=True)
    testbed.compute_and_save_marching_cubes_mesh(mesh, [mesh_res, mesh_res, mesh_res])
    res["snapshot"], res["mesh"] = snap, mesh
    if test_transforms:
        with open(test_transforms) as f:
            tt = json.load(f)
        data_dir = os.path.dirname(test_transforms)
        testbed.background_color = [0.0, 0.0, 0.0, 1.0]
        testbed.snap_to_pixel_centers = True
        testbed.nerf.rendering_min_transmittance = 1e-4
        if "from_na" not in tt:
            testbed.fov_axis = 0
            testbed.fov = tt["camera_angle_x"] * 180 / np.pi
            testbed.shall_train = False
        for frame in tt["frames"]:
            from PIL import Image
            ref = np.asarray(Image.open(os.path.join(data_dir, frame["file_path"])).convert("RGBA"), np.float32) / 255.0
            ref[..., :3] = ngp.srgb_to_linear(ref[..., :3]) * ref[..., 3:4]  # read_image: linear, premultiplied
            if testbed.color_space == ngp.ColorSpace.SRGB:
                a = ref[..., 3:4]
                ref[..., :3] = np.divide(ref[..., :3], a, out=np.zeros_like(ref[..., :3]), where=a != 0)
                ref[..., :3] = ngp.linear_to_srgb(ref[..., :3]) * a
                ref += (1.0 - a) * testbed.background_color
                ref[..., :3] = ngp.srgb_to_linear(ref[..., :3])
            testbed.set_nerf_camera_matrix(np.array(frame["transform_matrix"], np.float32)[:-1, :])
            image = testbed.render(ref.shape[1], ref.shape[0], spp, True)
            A = np.clip(ngp.linear_to_srgb(image[..., :3]), 0.0, 1.0)
            R = np.clip(ngp.linear_to_srgb(ref[..., :3]), 0.0, 1.0)
            res["psnr"].append(float(ngp.mse2psnr(float(np.mean((A - R) ** 2)))))
    res["testbed"] = testbed
    return res


def camera_angle_x(width, fl_x):
    return 2.0 * math.atan(0.5 * width / fl_x)


def run_dynamic_sequence(ngp, scene_dir, network, out_dir):
    """scripts/run_dynamic.py's training loop (:283-340: frame() over all frames; at each frame's last step a
    per-frame snapshot, save_transform, a mesh and the training-view PSNR) followed by its --dynamic_test pass
    (:147-208: a fresh testbed, change_to_frame(0), per frame load_snapshot + prepare_for_test + PSNR, then
    training_network_next_frame)."""
    res = {"train_psnr": [], "test_psnr": [], "transforms": [], "frames_seen": []}
    testbed = ngp.Testbed(ngp.TestbedMode.Nerf)
    testbed.load_training_data(scene_dir)
    testbed.reload_network_from_file(network)
    paths = sorted(p for p in os.listdir(scene_dir) if p.endswith(".json"))
    ck = os.path.join(out_dir, "checkpoints")
    os.makedirs(ck, exist_ok=True)
    os.makedirs(os.path.join(out_dir, "pred_transform"), exist_ok=True)
    while testbed.frame():
        k = testbed.current_training_time_frame
        limit = testbed.first_frame_max_training_step if k == 0 else testbed.next_frame_max_training_step
        if testbed.training_step == limit:
            res["frames_seen"].append(k)
            testbed.save_snapshot(os.path.join(ck, f"frame_{k}.msgpack"), False)
            tp = os.path.join(out_dir, "pred_transform", f"frame_{k}.txt")
            testbed.save_transform(tp)
            res["transforms"].append(open(tp).read())
            testbed.compute_and_save_marching_cubes_mesh(os.path.join(out_dir, f"frame_{k:04}.obj"), [32, 32, 32])
            res["train_psnr"].append(_training_view_psnr(ngp, testbed, 0))
    # --dynamic_test
    tb = ngp.Testbed(ngp.TestbedMode.Nerf)
    tb.load_training_data(scene_dir)
    tb.reload_network_from_file(network)
    tb.change_to_frame(0)
    while True:
        k = tb.current_training_time_frame
        tb.load_snapshot(os.path.join(ck, f"frame_{k}.msgpack"))
        aabb = ngp.BoundingBox(np.array([0, 0.0, 0]), np.array([1.0, 1.0, 1.0]))
        tb.compute_and_save_marching_cubes_mesh(os.path.join(out_dir, f"test_{k:04}.obj"), [32, 32, 32], aabb=aabb)
        res.setdefault("use_delta", []).append(tb.prepare_for_test())
        res["test_psnr"].append(_training_view_psnr(ngp, tb, 0))
        if not tb.training_network_next_frame() and tb.current_training_time_frame >= tb.all_training_time_frame - 1:
            break
    res["n_frames"] = len(paths)
    res["testbed"], res["test_testbed"] = testbed, tb
    return res


def _training_view_psnr(ngp, testbed, view):
    testbed.background_color = [0.0, 0.0, 0.0, 0.0]
    testbed.snap_to_pixel_centers = True
    testbed.set_camera_to_training_view(view)
    gt = testbed._images[view]
    img = testbed.render(gt.shape[1], gt.shape[0], 2, True)
    return float(ngp.eval_psnr(img, gt)[0])
