"""CPU tests of tools/data_format_from_neus.py (the NeuS cameras_sphere.npz converter, §8(f)).

Parity is pinned by construction: a camera built from a known K, R, C and scale matrix must come
back as the same intrinsics and camera-to-world pose, as cv2.decomposeProjectionMatrix gives in
the reference (tools/data_format_from_neus.py:12-33); cv2 is absent here."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import data_format_from_neus as conv  # noqa: E402


def _rot(rng):
    q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
    return q * np.sign(np.linalg.det(q))


def _camera(rng):
    K = np.array([[1100 + rng.uniform(0, 200), rng.uniform(-1, 1), 800 + rng.uniform(-20, 20)],
                  [0, 1100 + rng.uniform(0, 200), 600 + rng.uniform(-20, 20)], [0, 0, 1]])
    R = _rot(rng)
    C = rng.normal(size=3) * 3
    return K, R, C


def test_decompose_recovers_camera():
    rng = np.random.default_rng(0)
    for _ in range(50):
        K, R, C = _camera(rng)
        lam = rng.uniform(0.5, 2.0)  # projective scale of P
        P = lam * K @ np.hstack([R, -R @ C[:, None]])
        Ki, pose = conv.load_K_Rt_from_P(P)
        np.testing.assert_allclose(Ki[:3, :3], K, rtol=1e-5, atol=1e-3)
        np.testing.assert_allclose(pose[:3, :3], R.T, atol=1e-5)
        np.testing.assert_allclose(pose[:3, 3], C, atol=1e-4)
        assert abs(np.linalg.det(pose[:3, :3]) - 1) < 1e-5


def test_generate_splits_and_header(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(1)
    base = tmp_path / "scan"
    (base / "image").mkdir(parents=True)
    (base / "mask").mkdir()
    n, cams, truth = 10, {}, []
    S = np.diag([2.0, 2.0, 2.0, 1.0]); S[:3, 3] = [0.1, -0.2, 0.3]
    for i in range(n):
        K, R, C = _camera(rng)
        Ccam = np.linalg.inv(S) @ np.append(C, 1)  # world_mat sees scale-normalised coordinates
        P = np.eye(4); P[:3] = K @ np.hstack([R, -R @ C[:, None]])
        cams["world_mat_%d" % i] = (P @ np.linalg.inv(S)).astype(np.float32)
        cams["scale_mat_%d" % i] = S.astype(np.float32)
        truth.append((K, R, C, Ccam))
        Image.fromarray(rng.integers(0, 255, (6, 8, 3), dtype=np.uint8)).save(base / "image" / ("%03d.png" % i))
        Image.fromarray(np.full((6, 8, 3), 255 * (i % 2), np.uint8)).save(base / "mask" / ("%03d.png" % i))
    np.savez(base / "cameras_sphere.npz", **cams)
    out = tmp_path / "out"
    conv.generate(str(base), str(out), copy_image=True, test_views=(2, 5))
    tr = json.load(open(out / "transform_train.json"))
    te = json.load(open(out / "transform_test.json"))
    assert (tr["w"], tr["h"], tr["scale"], tr["offset"], tr["from_na"]) == (8, 6, 0.5, [0.5] * 3, True)
    assert len(tr["frames"]) == 8 and len(te["frames"]) == 2
    assert te["frames"][0]["file_path"] == os.path.join("images", "002.png")
    K, R, C, _ = truth[2]
    np.testing.assert_allclose(np.array(te["frames"][0]["intrinsic_matrix"])[:3, :3], K, rtol=1e-4, atol=1e-2)
    np.testing.assert_allclose(np.array(te["frames"][0]["transform_matrix"])[:3, 3], C, atol=1e-3)
    rgba = np.asarray(Image.open(out / "images" / "003.png"))
    assert rgba.shape == (6, 8, 4) and (rgba[..., 3] == 255).all()
