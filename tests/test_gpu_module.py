"""The tcnn-shaped operator modules (include/neus2_hip.h neus_module_*; cpp_api.h:66-110) on the MI355X:
* the NeuS network module: initialize_params = the Trainer's seed_seq init, inference / backward bit-identical to the
  Testbed's kernels on the same parameters, the backward against the oracle (the tolerances of
  test_gpu_parity.test_network_backward_parity), EGradientMode Ignore / Overwrite / Accumulate, dL_dinput;
* the HashGrid encoding module: forward bit-exact against the oracle (enc + dy/dx), backward (dL_dparams,
  dL_dinput) and backward_backward_input (dL_dparams, dL_ddLdoutput) against float64 autograd of
  tests/torch_ref.hash_grid (the scatter rounds each corner contribution to fp16 like the reference's fp16
  atomics: rel-L2 <= 2e-3)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
N = 1024


def _record(test, **metrics):
    import json
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "parity_metrics.jsonl"), "a") as f:
        f.write(json.dumps({"test": test, **{k: float(v) for k, v in metrics.items()}}) + "\n")


def _coords(n, seed=0):
    rng = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0.05, 0.95, (n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c[:, 4:] = (d + 1) * 0.5
    return c


def _rel_cos(x, y):
    x, y = np.asarray(x, np.float64).ravel(), np.asarray(y, np.float64).ravel()
    return np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30), x @ y / max(np.linalg.norm(x) * np.linalg.norm(y), 1e-30)


def test_network_module(torch_cuda):
    import oracle as O
    from neus2_amd import config, pyngp, scenes
    from neus2_amd._lib import check, lib
    from neus2_amd.module import GradientMode, Module
    t = torch_cuda
    cfg_dict = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    sc = scenes.small_scene(n_views=4, width=32, height=24)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_json(cfg_dict, batch_size=4096)
    lay = tb.layout()
    m = Module.create_network(cfg_dict, batch_capacity=4096)
    assert m.n_params == lay["n_params"] and m.n_input_dims == 7 and m.n_output_dims == 16
    assert m.name() == "NerfNetwork" and m.info["grid_offset"] == lay["grid_offset"]
    assert abs(m.info["per_level_scale"] - lay["per_level_scale"]) < 1e-6
    # initialize_params: the Trainer's init (seed 1337); the Testbed replaces the density block by the geometric init
    p0 = m.initialize_params(1337).cpu().numpy()
    tp = tb.get_params()
    nd = lay["n_density"]
    np.testing.assert_array_equal(p0[nd:], tp[nd:])
    # perturbed parameters that exercise every path, shared as fp16 by the module call and the Testbed
    rng = np.random.default_rng(3)
    p = tp.copy()
    din = lay["density_input_width"]
    w0 = p[: 64 * din].reshape(64, din)
    w0[:, 3:31] = rng.normal(0, 0.3, (64, 28))
    p[: 64 * din] = w0.reshape(-1)
    p[lay["grid_offset"]:lay["variance_offset"]] = rng.uniform(-0.1, 0.1, lay["variance_offset"] - lay["grid_offset"])
    tb.set_params(p)
    ph = tb.get_half_params()
    params = t.from_numpy(ph.view(np.int16).copy()).cuda()
    c = _coords(N, 7)
    x = t.from_numpy(c).cuda()
    L = lay["n_levels"]
    out = m.inference(x, params)
    ref = t.zeros((N, 16), dtype=t.int16, device="cuda")
    t.cuda.synchronize()
    check(lib().neus_net_forward(tb.handle, None, C.c_uint32(N), C.c_void_p(x.data_ptr()), C.c_uint32(L), C.c_void_p(ref.data_ptr())))
    t.cuda.synchronize()
    np.testing.assert_array_equal(out.view(t.int16).cpu().numpy(), ref.cpu().numpy())
    ctx, out2 = m.forward(x, params)
    np.testing.assert_array_equal(out2.view(t.int16).cpu().numpy(), ref.cpu().numpy())
    # backward: Overwrite == the Testbed's backward (same kernels), == the oracle within the parity tolerances
    dl = np.zeros((N, 16), np.float32)
    dl[:, :4] = rng.normal(0, 1e-2, (N, 4))
    dl[:, 4:7] = rng.normal(0, 1.0, (N, 3))
    dl[:, 7] = rng.normal(0, 1e-2, N)
    dl[:, 8:11] = rng.normal(0, 1e-2, (N, 3))
    dl16 = dl.astype(np.float16)
    dlt = t.from_numpy(dl16.view(np.int16).copy()).cuda()
    m.set_indeed_batch_size(N)
    g = t.full((m.n_params,), 7.0, dtype=t.float32, device="cuda")
    dx = t.full((N, 7), 3.0, dtype=t.float32, device="cuda")
    m.backward(ctx, x, dlt, params, dL_dparams=g, dL_dinput=dx, mode=GradientMode.Overwrite)
    gt = t.zeros(m.n_params, dtype=t.float32, device="cuda")
    dpos = t.zeros((N, 4), dtype=t.float32, device="cuda")
    t.cuda.synchronize()  # the Testbed runs on its own stream: torch's fills (queued behind the module) must land first
    check(lib().neus_net_backward_pos(tb.handle, None, C.c_uint32(N), C.c_void_p(x.data_ptr()), C.c_uint32(L), C.c_void_p(dlt.data_ptr()),
                                      C.c_uint32(N), C.c_void_p(gt.data_ptr()), C.c_void_p(dpos.data_ptr())))
    t.cuda.synchronize()
    gm = g.cpu().numpy()
    np.testing.assert_array_equal(gm, gt.cpu().numpy())
    dxm = dx.cpu().numpy()
    np.testing.assert_array_equal(dxm[:, :3], dpos.cpu().numpy()[:, :3])
    assert not dxm[:, 3:].any()
    gref = O.network_backward(O.make_cfg(per_level_scale=lay["per_level_scale"]), ph.astype(np.float32), c, L, dl16.view(np.uint16), N)
    for name, (a, b) in {"density": (0, nd), "rgb": (nd, lay["n_matrix"]), "grid": (lay["grid_offset"], lay["variance_offset"]),
                         "variance": (lay["variance_offset"], lay["variance_offset"] + 1)}.items():
        rel, cos = _rel_cos(gm[a:b], gref[a:b])
        _record("module_network_backward_" + name, rel=rel, cos=cos)
        assert rel <= 2e-2 and cos >= 0.999, (name, rel, cos)
    # Accumulate adds the same gradient; Ignore leaves dL_dparams untouched
    m.backward(ctx, x, dlt, params, dL_dparams=g, mode=GradientMode.Accumulate)
    np.testing.assert_array_equal(g.cpu().numpy(), gm * 2)
    m.backward(ctx, x, dlt, params, dL_dparams=g, mode=GradientMode.Ignore)
    np.testing.assert_array_equal(g.cpu().numpy(), gm * 2)
    with pytest.raises(Exception):
        m.backward_backward_input(ctx, x, dx, dlt, params, dL_dparams=g)
    # the module's parameters are the call's: other params -> other outputs
    params2 = t.from_numpy((ph * np.float16(0.5)).view(np.int16).copy()).cuda()
    assert not t.equal(m.inference(x, params2).view(t.int16), ref)


def test_encoding_module(torch_cuda):
    import torch
    import oracle as O
    from torch_ref import grid_tables, hash_grid
    from neus2_amd.module import GradientMode, Module
    t = torch_cuda
    enc_cfg = {"otype": "HashGrid", "n_levels": 8, "n_features_per_level": 2, "log2_hashmap_size": 14, "base_resolution": 16,
               "per_level_scale": 1.5}
    m = Module.create_encoding(enc_cfg, batch_capacity=N)
    L = 8
    off, res = grid_tables(L, 14, 16, 1.5)
    assert m.n_params == 2 * off[-1] and m.n_output_dims == 2 * L and m.name() == "HashGrid"
    p0 = m.initialize_params(1337).cpu().numpy()
    assert np.abs(p0).max() <= 1e-4 and np.abs(p0).max() > 0
    rng = np.random.default_rng(9)
    ph = rng.uniform(-1, 1, m.n_params).astype(np.float16)
    params = t.from_numpy(ph.view(np.int16).copy()).cuda()
    pos = rng.uniform(0.02, 0.98, (N, 3)).astype(np.float32)
    x = t.from_numpy(pos).cuda()
    ctx, y = m.forward(x, params, prepare_input_gradients=True)
    got = y.float().cpu().numpy().transpose(1, 0, 2).reshape(N, 2 * L)
    # oracle: a 8-level config with the same tables, parameters in the grid block
    ocfg = O.make_cfg(n_levels=L, log2_hashmap_size=14, base_resolution=16, per_level_scale=1.5)
    olay = O.layout(ocfg)
    op = np.zeros(olay["n_params"], np.float32)
    op[olay["grid_off"]:olay["grid_off"] + m.n_params] = ph.astype(np.float32)
    renc, _ = O.grid_forward(ocfg, op, pos, L)
    np.testing.assert_array_equal(got.view(np.uint32), renc.astype(np.float32).view(np.uint32))
    # float64 autograd reference
    tab = torch.tensor(ph.astype(np.float64).reshape(-1, 2), requires_grad=True)
    xt = torch.tensor(pos.astype(np.float64), requires_grad=True)
    e = hash_grid(xt, tab, off, res)
    dly = rng.normal(0, 1, (L, N, 2)).astype(np.float16)
    dly_t = torch.tensor(dly.astype(np.float64).transpose(1, 0, 2).reshape(N, 2 * L), requires_grad=True)
    S = (e * dly_t).sum()
    g_tab, g_x = torch.autograd.grad(S, (tab, xt), create_graph=True)
    v = rng.normal(0, 1, (N, 3)).astype(np.float32)
    S2 = (g_x * torch.tensor(v.astype(np.float64))).sum()
    g2_tab, g2_dly = torch.autograd.grad(S2, (tab, dly_t))
    # backward: dL_dparams (Overwrite) and dL_dinput
    dly_dev = t.from_numpy(dly.view(np.int16).copy()).cuda()
    g = t.zeros(m.n_params, dtype=t.float32, device="cuda")
    dx = t.zeros((N, 3), dtype=t.float32, device="cuda")
    m.backward(ctx, x, dly_dev, params, dL_dparams=g, dL_dinput=dx, mode=GradientMode.Overwrite)
    rel_p, cos_p = _rel_cos(g.cpu().numpy(), g_tab.detach().numpy().ravel())
    rel_x, cos_x = _rel_cos(dx.cpu().numpy(), g_x.detach().numpy())
    # backward_backward_input: second-order dL_dparams and dL_ddLdoutput
    g2 = t.zeros(m.n_params, dtype=t.float32, device="cuda")
    ddo = t.zeros((L, N, 2), dtype=t.float16, device="cuda")
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dly_dev, params, dL_dparams=g2, dL_ddLdoutput=ddo)
    rel_p2, cos_p2 = _rel_cos(g2.cpu().numpy(), g2_tab.numpy().ravel())
    ddo_np = ddo.float().cpu().numpy().transpose(1, 0, 2).reshape(N, 2 * L)
    rel_o2, cos_o2 = _rel_cos(ddo_np, g2_dly.numpy())
    _record("module_encoding", rel_params=rel_p, rel_dinput=rel_x, rel_params_2nd=rel_p2, rel_ddLdoutput=rel_o2)
    assert rel_p <= 2e-3 and cos_p >= 0.99999, (rel_p, cos_p)
    assert rel_x <= 1e-4, rel_x
    assert rel_p2 <= 2e-3 and cos_p2 >= 0.99999, (rel_p2, cos_p2)
    assert rel_o2 <= 2e-3, rel_o2  # fp16 output
    # Accumulate: first + second order into one buffer == their sum
    acc = g.clone()
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dly_dev, params, dL_dparams=acc, mode=GradientMode.Accumulate)
    np.testing.assert_allclose(acc.cpu().numpy(), g.cpu().numpy() + g2.cpu().numpy(), rtol=1e-6, atol=1e-6)
    # progressive levels: set_training_step(1) -> ceil(0.2 * 8) = 2 -> levels 0..2 active, the rest 0
    m.set_training_step(1)
    y3 = m.inference(x, params).float().cpu().numpy()
    assert not y3[3:].any() and np.array_equal(y3[:3], y.float().cpu().numpy()[:3])
