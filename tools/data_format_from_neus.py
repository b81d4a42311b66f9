"""NeuS/DTU `cameras_sphere.npz` -> NeuS2 `transform_train.json` / `transform_test.json`.

Follows the reference converter tools/data_format_from_neus.py:
  - P = (world_mat_i @ scale_mat_i)[:3, :4]                           (:66-68)
  - load_K_Rt_from_P: P -> K (normalised by K[2,2]), pose = [R^T | C] (:12-33)
  - header {w, h, aabb_scale 1, scale 0.5, offset 0.5, from_na}        (:141-150, :177-186)
  - views 8,13,16,21,26,31,34,56 go to the test split, the rest train (:93, :170-171, :208-209)
  - images: RGB from image/, alpha from mask/ (luminance, as cv2.imread(path, 0)), written as RGBA PNG (:120-135)
The reference decomposes P with cv2.decomposeProjectionMatrix (absent here); this is the same
decomposition restated in numpy: M = K R with R a rotation (det +1), K upper triangular,
K[0,0] > 0 and K[1,1] > 0 (OpenCV's RQDecomp3x3 convention), camera centre C = null(P).
Image IO uses PIL (what neus2_amd.pyngp.load_transforms reads) instead of cv2.
"""
from __future__ import annotations

import argparse
import json
import os

import numpy as np

TEST_VIEWS = (8, 13, 16, 21, 26, 31, 34, 56)


def rq3(M):
    """RQ decomposition of a 3x3 matrix, M = K @ R, with K[0,0], K[1,1] > 0 and det(R) = +1."""
    P = np.eye(3)[::-1]
    q, r = np.linalg.qr((P @ M).T)
    K = P @ r.T @ P
    R = P @ q.T
    s0, s1 = np.sign(K[0, 0]) or 1.0, np.sign(K[1, 1]) or 1.0
    s2 = s0 * s1 * np.sign(np.linalg.det(R))
    D = np.diag([s0, s1, s2])
    return K @ D, D @ R


def load_K_Rt_from_P(P):
    """P (3x4) -> (intrinsics 4x4, pose 4x4 camera-to-world); tools/data_format_from_neus.py:12-33."""
    P = np.asarray(P, np.float64)
    K, R = rq3(P[:, :3])
    K = K / K[2, 2]
    intrinsics = np.eye(4)
    intrinsics[:3, :3] = K
    C = -np.linalg.solve(P[:, :3], P[:, 3])
    pose = np.eye(4, dtype=np.float32)
    pose[:3, :3] = R.T
    pose[:3, 3] = C
    return intrinsics.astype(np.float32), pose


def cameras_from_npz(cams, n_images):
    Ks, poses = [], []
    for i in range(n_images):
        wm = np.asarray(cams["world_mat_%d" % i], np.float32)
        sm = np.asarray(cams["scale_mat_%d" % i], np.float32)
        K, pose = load_K_Rt_from_P((wm @ sm)[:3, :4])
        Ks.append(K)
        poses.append(pose)
    return Ks, poses


def generate(base_dir, output_dir, copy_image=True, wrong_camera=(), test_views=TEST_VIEWS):
    from PIL import Image
    imgs = sorted(os.listdir(os.path.join(base_dir, "image")))
    msks = sorted(os.listdir(os.path.join(base_dir, "mask")))
    assert len(imgs) == len(msks), "image/ and mask/ must hold the same number of files"
    with np.load(os.path.join(base_dir, "cameras_sphere.npz")) as cams:
        Ks, poses = cameras_from_npz(cams, len(imgs))
    out_img = os.path.join(output_dir, "images")
    os.makedirs(out_img, exist_ok=True)
    H, W = 1200, 1600
    for name, mname in zip(imgs, msks):
        if not copy_image:
            break
        rgb = np.asarray(Image.open(os.path.join(base_dir, "image", name)).convert("RGB"))
        # cv2.imread(path, 0) (reference :130) reads the mask as luminance; PIL's "L" is the same ITU-R 601 weighting
        # (integer rounding may differ by one level from OpenCV's, which is not importable here: parity unpinned)
        m = np.asarray(Image.open(os.path.join(base_dir, "mask", mname)).convert("L"))
        Image.fromarray(np.concatenate([rgb, m[..., None]], -1), "RGBA").save(os.path.join(out_img, name))
        H, W = rgb.shape[:2]
    names = sorted(os.listdir(out_img))
    assert len(names) == len(Ks), "The number of cameras should be equal to the number of images!"
    for split, keep in (("train", lambda i: i not in test_views), ("test", lambda i: i in test_views)):
        out = {"w": W, "h": H, "aabb_scale": 1.0, "scale": 0.5, "offset": [0.5, 0.5, 0.5],
               "from_na": True, "frames": []}
        for i, name in enumerate(names):
            if i in wrong_camera or not keep(i):
                continue
            out["frames"].append({"file_path": os.path.join("images", name),
                                  "transform_matrix": poses[i].tolist(),
                                  "intrinsic_matrix": Ks[i].tolist()})
        with open(os.path.join(output_dir, "transform_%s.json" % split), "w") as f:
            json.dump(out, f, indent=4)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--base_dir", required=True, help="DTU scan dir: cameras_sphere.npz, image/, mask/")
    ap.add_argument("--output_dir", required=True)
    ap.add_argument("--copy_image", action="store_true")
    a = ap.parse_args()
    generate(a.base_dir, a.output_dir, a.copy_image)
