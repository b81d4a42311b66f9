"""The hash-grid gradient scatter paths (grid.hip) against each other: per-block record regions (k_scatter_bin_r +
k_scatter_accum_r, the default), the wide-block binning (k_scatter_hist_w + k_scatter_bin_w, NEUS_SCATTER=wide) and
the 256-sample binned one (NEUS_SCATTER=binned), at 512- and 1024-sample workgroups: all bin the same fp16x2 corner contributions (first +
second order, grid.h:371-500 and 880-1007) and sum them in int64 fixed point, so the grid gradient must be bitwise equal, for a
backward on perturbed parameters (every level active, dense and hashed levels, the heavy split buckets of the small
dense levels), for a backward at a low progressive level (inactive levels untouched), and over 40 training steps."""
import ctypes as C
import os

import numpy as np
import pytest

from gpu_util import dev, ptr

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _testbed(sc, mode, batch):
    """mode: "regions" (per-block record regions, 512-sample workgroups: the default), "regions1024" (1024-sample
    ones), "seg" (wide-block binning, 512), "seg1024" or "binned" (the 256-sample histogram / scan / bin path)."""
    from neus2_amd import pyngp
    env = {"NEUS_SCATTER": {"binned": "binned", "seg": "wide", "seg1024": "wide"}.get(mode),
           "NEUS_SCATTER_CHUNK": "1024" if mode.endswith("1024") else None}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=batch)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return tb


@pytest.fixture(scope="module")
def scene(torch_cuda):
    from neus2_amd import scenes
    return scenes.small_scene(n_views=8, width=64, height=48)


def test_scatter_paths_bitwise_equal(scene, torch_cuda):
    from neus2_amd._lib import check, lib
    t = torch_cuda
    n = 1 << 14
    modes = ("regions", "regions1024", "seg", "seg1024", "binned")
    tbs = [_testbed(scene, m, n) for m in modes]
    seg = tbs[0]
    lay = seg.layout()
    rng = np.random.default_rng(17)
    p = seg.get_params().copy()
    din, L = lay["density_input_width"], lay["n_levels"]
    w0 = p[: 64 * din].reshape(64, din)
    w0[:, 3:3 + 2 * L] = rng.normal(0, 0.3, (64, 2 * L))
    p[: 64 * din] = w0.reshape(-1)
    p[lay["grid_offset"]:lay["variance_offset"]] = rng.uniform(-0.1, 0.1, lay["variance_offset"] - lay["grid_offset"])
    for tb in tbs:
        tb.set_params(p)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0.02, 0.98, (n, 3))
    # runs of samples along "rays" (consecutive lanes sharing coarse cells: the wave run merge)
    c[n // 2:, :3] = np.repeat(rng.uniform(0.1, 0.9, (n // 64, 3)), 32, axis=0) + np.tile(np.linspace(0, 0.02, 32), n // 64)[:, None]
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c[:, 4:] = (d + 1) * 0.5
    dl = np.zeros((n, 16), np.float32)
    dl[:, :4] = rng.normal(0, 1e-2, (n, 4))
    dl[:, 4:7] = rng.normal(0, 1.0, (n, 3))
    dl[:, 7] = rng.normal(0, 1e-2, n)
    dl16 = dl.astype(np.float16)
    for valid in (L, 3):
        grads = []
        for tb in tbs:
            g = t.zeros(lay["n_params"], dtype=t.float32, device="cuda")
            check(lib().neus_net_backward(tb.handle, None, C.c_uint32(n), ptr(dev(t, c)), C.c_uint32(valid), ptr(dev(t, dl16)),
                                          C.c_uint32(n), ptr(g)))
            t.cuda.synchronize()
            grads.append(g.cpu().numpy())
        b = grads[-1]
        g0, g1 = lay["grid_offset"], lay["variance_offset"]
        assert np.any(b[g0:g1])
        for m, a in zip(modes, grads):
            np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32), err_msg=m)
    # training: 40 steps (progressive levels 3 -> 3, occupancy updates) bitwise equal
    seg2, bin2 = _testbed(scene, "regions", 4096), _testbed(scene, "binned", 4096)
    seg2.train_steps(40)
    bin2.train_steps(40)
    np.testing.assert_array_equal(seg2.get_params().view(np.uint32), bin2.get_params().view(np.uint32))
    np.testing.assert_array_equal(seg2.get_gradients().view(np.uint32), bin2.get_gradients().view(np.uint32))


def test_valid_level_drop_matches_zeroed_reference(scene, torch_cuda, tmp_path):
    """The scatter writes only the grid levels up to the progressive valid level and zeroes the rest of the gradient
    once when the valid level drops (scatter_work_for): train past several level increments, reload a snapshot of an
    early step (the valid level falls back), train on, and compare parameters and gradients bitwise with a testbed that
    zeroes the whole grid gradient before every scatter (NEUS_SCATTER_NOSKIP=1)."""
    from neus2_amd import pyngp
    out = []
    for noskip in (False, True):
        old = os.environ.get("NEUS_SCATTER_NOSKIP")
        if noskip:
            os.environ["NEUS_SCATTER_NOSKIP"] = "1"
        else:
            os.environ.pop("NEUS_SCATTER_NOSKIP", None)
        try:
            tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
            tb.set_dataset(scene["images"], scene["focal"], scene["principal"], scene["xforms"], 1)
            tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
        finally:
            if old is None:
                os.environ.pop("NEUS_SCATTER_NOSKIP", None)
            else:
                os.environ["NEUS_SCATTER_NOSKIP"] = old
        tb.train_steps(20)
        snap = str(tmp_path / f"early_{int(noskip)}.msgpack")
        tb.save_snapshot(snap, include_optimizer_state=True)
        v_early = tb.stats()["valid_level"]
        tb.train_steps(400)
        v_late = tb.stats()["valid_level"]
        assert v_late > v_early
        tb.load_snapshot(snap)
        tb.train_steps(15)
        assert tb.stats()["valid_level"] < v_late
        out.append((tb.get_params(), tb.get_gradients()))
    (p0, g0), (p1, g1) = out
    np.testing.assert_array_equal(p0.view(np.uint32), p1.view(np.uint32))
    np.testing.assert_array_equal(g0.view(np.uint32), g1.view(np.uint32))
