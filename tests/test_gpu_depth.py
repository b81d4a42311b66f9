"""Depth supervision: the reference loads per-frame depth maps (nerf_loader.cu:599-612)
and its loss kernel reads them when nerf.training.depth_supervision_lambda > 0 (testbed_nerf.cu:1697-1698), but the
term it forms (`depth_supervision`, :1836) is added to no gradient and no loss output, so training is the same as with
lambda = 0. Parity here: a testbed with lambda = 1 and analytic depth maps of the sphere (the distance along each pixel
ray to the surface, scene units) trains bit-identically to lambda = 0 (per-ray composited counts every 10 steps, then
parameters and loss). The lambda = 0 loss / compaction itself is oracle-checked by test_gpu_parity.py
test_loss_compaction_parity; the oracle restates the reference and so has no depth term either."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sphere_depth(sc, i):
    """Analytic depth fixture: distance from the camera centre to the sphere along each pixel-centre ray (0 = miss,
    which the reference treats as no target: target_depth > 0 fails)."""
    from neus2_amd import scenes
    h, w = sc["images"][i].shape[:2]
    M = np.asarray(sc["xforms"][i], np.float64)
    fx, fy = sc["focal"][i]
    px, py = sc["principal"][i]
    X, Y = np.meshgrid((np.arange(w) + 0.5) / w, (np.arange(h) + 0.5) / h)
    d = np.stack([(X - px) * w / fx, (Y - py) * h / fy, np.ones_like(X)], -1) @ M[:, :3].T
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    oc = M[:, 3] - scenes.CENTER
    b = d @ oc
    disc = b * b - (oc @ oc - scenes.RADIUS ** 2)
    t = -b - np.sqrt(np.maximum(disc, 0))
    return np.where((disc > 0) & (t > 0), t, 0.0).astype(np.float32)


def test_depth_supervision_lambda_is_inert(torch_cuda):
    from neus2_amd import pyngp, scenes
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    tbs = []
    for lam in (1.0, 0.0):
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        if lam > 0:
            for i in range(len(sc["images"])):
                tb.set_depth(i, sphere_depth(sc, i))
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
        tb.nerf.training.depth_supervision_lambda = lam
        assert tb.nerf.training.depth_supervision_lambda == lam
        tbs.append(tb)
    a, b = tbs
    assert a.nerf.training.dataset.has_depth and not b.nerf.training.dataset.has_depth
    assert (a.nerf.training.dataset.depth(0) > 0).any()
    for _ in range(3):
        a.train_steps(10)
        b.train_steps(10)
        np.testing.assert_array_equal(a.ray_counts(1 << 12)[1], b.ray_counts(1 << 12)[1])
    np.testing.assert_array_equal(a.get_params().view(np.uint32), b.get_params().view(np.uint32))
    assert a.stats()["loss"] == b.stats()["loss"]
