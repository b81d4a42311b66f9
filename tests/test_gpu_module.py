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
    m = Module.create_nerf_network(dict(cfg_dict, gradient_precision="fp32"), batch_capacity=4096)
    m16 = Module.create_nerf_network(cfg_dict, batch_capacity=4096)  # default: fp16 dL_dparams (tcnn's param precision)
    assert m.n_params == lay["n_params"] and m.n_input_dims == 7 and m.n_output_dims == 16
    assert m.name() == "NerfNetwork" and m.info["grid_offset"] == lay["grid_offset"]
    assert abs(m.info["per_level_scale"] - lay["per_level_scale"]) < 1e-6
    assert m.gradient_precision == "fp32" and m16.gradient_precision == "fp16"
    # initialize_params: cpp::Module draws from pcg32{seed} (cpp_api.cu:162-165), not the Trainer's seed_seq
    p0 = m.initialize_params(1337).cpu().numpy()
    ocfg = O.make_cfg(per_level_scale=lay["per_level_scale"])
    ref0 = np.zeros(p0.size, np.float32)
    O.lib().or_init_params_pcg(C.byref(ocfg), C.c_uint64(1337), None, O.P(ref0))
    np.testing.assert_array_equal(p0, ref0)
    tp = tb.get_params()
    nd = lay["n_density"]
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
    # fp16 dL_dparams (the default): the fp32 gradient rounded once; Accumulate adds in fp32 and rounds once
    ctx16, _ = m16.forward(x, params)
    m16.set_indeed_batch_size(N)
    g16 = m16.gradient_buffer()
    assert g16.dtype == t.float16
    m16.backward(ctx16, x, dlt, params, dL_dparams=g16, mode=GradientMode.Overwrite)
    h16 = gm.astype(np.float16)
    np.testing.assert_array_equal(g16.cpu().numpy().view(np.uint16), h16.view(np.uint16))
    m16.backward(ctx16, x, dlt, params, dL_dparams=g16, mode=GradientMode.Accumulate)
    np.testing.assert_array_equal(g16.cpu().numpy().view(np.uint16), (h16.astype(np.float32) + gm).astype(np.float16).view(np.uint16))
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


def _to_nf(a, layout, n, L):
    """An encoding-shaped module tensor (host) as [n][2L] (feature 2l + k of level l)."""
    a = np.asarray(a)
    return {"AoS": lambda: a.reshape(n, 2 * L), "SoA": lambda: a.reshape(2 * L, n).T,
            "paired": lambda: a.reshape(L, n, 2).transpose(1, 0, 2).reshape(n, 2 * L)}[layout]()


def _from_nf(a, layout, n, L):
    return np.ascontiguousarray({"AoS": lambda: a, "SoA": lambda: a.T,
                                 "paired": lambda: a.reshape(n, L, 2).transpose(1, 0, 2)}[layout]())


@pytest.mark.parametrize("layout", ["AoS", "SoA", "paired"])
def test_encoding_module(torch_cuda, layout):
    """The HashGrid module in each output layout: AoS [n][2L] (the cpp::Module view, cpp_api.cu:58-70, the default),
    SoA [2L][n] (grid.h:2357-2359), paired [L][n] half2: forward bit-exact vs the oracle, backward and double backward
    vs float64 autograd; pcg32{seed} initialisation (cpp_api.cu:162-165) bit-exact; tcnn's defaults for omitted keys."""
    import torch
    import oracle as O
    from torch_ref import grid_tables, hash_grid
    from neus2_amd.module import GradientMode, Module
    t = torch_cuda
    enc_cfg = {"otype": "HashGrid", "n_levels": 8, "n_features_per_level": 2, "log2_hashmap_size": 14, "base_resolution": 16,
               "per_level_scale": 1.5, "gradient_precision": "fp32"}
    if layout != "AoS":
        enc_cfg["output_layout"] = layout
    m = Module.create_encoding(enc_cfg, batch_capacity=N)
    assert m.output_layout == layout
    L = 8
    off, res = grid_tables(L, 14, 16, 1.5)
    assert m.n_params == 2 * off[-1] and m.n_output_dims == 2 * L and m.name() == "HashGrid"
    hp = m.hyperparams()
    # omitted progressive-level keys take tcnn's create_grid_encoding defaults (grid.h:2518-2525)
    assert hp["valid_level_scale"] == pytest.approx(0.01) and hp["base_valid_level_scale"] == pytest.approx(0.5)
    assert hp["base_training_step"] == 200 and hp["per_level_scale"] == 1.5
    p0 = m.initialize_params(1337).cpu().numpy()
    assert np.abs(p0).max() <= 1e-4 and np.abs(p0).max() > 0
    oinit = np.zeros(m.n_params, np.float32)
    O.lib().or_grid_init_pcg(C.c_uint64(m.n_params), C.c_uint64(1337), O.P(oinit))
    np.testing.assert_array_equal(p0, oinit)
    ocfg = O.make_cfg(n_levels=L, log2_hashmap_size=14, base_resolution=16, per_level_scale=1.5)
    olay = O.layout(ocfg)
    rng = np.random.default_rng(9)
    ph = rng.uniform(-1, 1, m.n_params).astype(np.float16)
    params = t.from_numpy(ph.view(np.int16).copy()).cuda()
    pos = rng.uniform(0.02, 0.98, (N, 3)).astype(np.float32)
    x = t.from_numpy(pos).cuda()
    ctx, y = m.forward(x, params, prepare_input_gradients=True)
    assert tuple(y.shape) == m.output_shape(N)
    got = _to_nf(y.float().cpu().numpy(), layout, N, L)
    # oracle: a 8-level config with the same tables, parameters in the grid block
    op = np.zeros(olay["n_params"], np.float32)
    op[olay["grid_off"]:olay["grid_off"] + m.n_params] = ph.astype(np.float32)
    renc, _ = O.grid_forward(ocfg, op, pos, L)
    np.testing.assert_array_equal(got.view(np.uint32), renc.astype(np.float32).view(np.uint32))
    # float64 autograd reference
    tab = torch.tensor(ph.astype(np.float64).reshape(-1, 2), requires_grad=True)
    xt = torch.tensor(pos.astype(np.float64), requires_grad=True)
    e = hash_grid(xt, tab, off, res)
    dly_nf = rng.normal(0, 1, (N, 2 * L)).astype(np.float16)
    dly = _from_nf(dly_nf, layout, N, L)
    dly_t = torch.tensor(dly_nf.astype(np.float64), requires_grad=True)
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
    ddo = t.zeros(m.output_shape(N), dtype=t.float16, device="cuda")
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dly_dev, params, dL_dparams=g2, dL_ddLdoutput=ddo)
    rel_p2, cos_p2 = _rel_cos(g2.cpu().numpy(), g2_tab.numpy().ravel())
    ddo_np = _to_nf(ddo.float().cpu().numpy(), layout, N, L)
    rel_o2, cos_o2 = _rel_cos(ddo_np, g2_dly.numpy())
    _record("module_encoding_" + layout, rel_params=rel_p, rel_dinput=rel_x, rel_params_2nd=rel_p2, rel_ddLdoutput=rel_o2)
    assert rel_p <= 2e-3 and cos_p >= 0.99999, (rel_p, cos_p)
    assert rel_x <= 1e-4, rel_x
    assert rel_p2 <= 2e-3 and cos_p2 >= 0.99999, (rel_p2, cos_p2)
    assert rel_o2 <= 2e-3, rel_o2  # fp16 output
    # Accumulate: first + second order into one buffer == their sum
    acc = g.clone()
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dly_dev, params, dL_dparams=acc, mode=GradientMode.Accumulate)
    np.testing.assert_allclose(acc.cpu().numpy(), g.cpu().numpy() + g2.cpu().numpy(), rtol=1e-6, atol=1e-6)
    # progressive levels with tcnn's defaults: set_training_step(1) -> valid level ceil(0.5 * 8) = 4 -> levels 0..4 active
    m.set_training_step(1)
    y3 = _to_nf(m.inference(x, params).float().cpu().numpy(), layout, N, L)
    assert not y3[:, 10:].any() and np.array_equal(y3[:, :10], got[:, :10])
    # fp16 dL_dparams (default gradient precision): the fp32 first-order gradient rounded once
    enc16 = dict(enc_cfg)
    del enc16["gradient_precision"]
    m16 = Module.create_encoding(enc16, batch_capacity=N)
    ctx16, _ = m16.forward(x, params, prepare_input_gradients=True)
    g16 = m16.gradient_buffer()
    m16.backward(ctx16, x, dly_dev, params, dL_dparams=g16, mode=GradientMode.Overwrite)
    np.testing.assert_array_equal(g16.cpu().numpy().view(np.uint16), g.cpu().numpy().astype(np.float16).view(np.uint16))


@pytest.mark.parametrize("layout", ["AoS", "SoA"])
def test_encoding_module_fp32(torch_cuda, layout):
    """create_encoding(..., requested_precision=Fp32) (cpp_api.h:110, cpp_api.cu:174-183: GridEncoding<float>): f32 params,
    output, dL_doutput and gradients. Forward, backward (dL_dparams, dL_dinput) and backward_backward_input
    (second-order dL_dparams, dL_ddLdoutput) vs float64 autograd at fp32 tolerance; Overwrite / Accumulate; paired
    layout refused; the fp16 module (Fp16, the default) is unchanged."""
    import torch
    from torch_ref import grid_tables, hash_grid
    from neus2_amd.module import GradientMode, Module, Precision
    t = torch_cuda
    L = 8
    enc_cfg = {"otype": "HashGrid", "n_levels": L, "n_features_per_level": 2, "log2_hashmap_size": 14, "base_resolution": 16,
               "per_level_scale": 1.5, "output_layout": layout}
    m = Module.create_encoding(enc_cfg, batch_capacity=N, requested_precision=Precision.Fp32)
    assert m.info["param_precision"] == 0 and m.info["output_precision"] == 0 and m.hyperparams()["precision"] == "fp32"
    with pytest.raises(Exception):
        Module.create_encoding(dict(enc_cfg, output_layout="paired"), batch_capacity=N, requested_precision=Precision.Fp32)
    off, res = grid_tables(L, 14, 16, 1.5)
    rng = np.random.default_rng(19)
    pf = rng.uniform(-1, 1, m.n_params).astype(np.float32)
    params = t.from_numpy(pf).cuda()
    pos = rng.uniform(0.02, 0.98, (N, 3)).astype(np.float32)
    x = t.from_numpy(pos).cuda()
    ctx, y = m.forward(x, params, prepare_input_gradients=True)
    assert y.dtype == t.float32 and tuple(y.shape) == m.output_shape(N)
    tab = torch.tensor(pf.astype(np.float64).reshape(-1, 2), requires_grad=True)
    xt = torch.tensor(pos.astype(np.float64), requires_grad=True)
    e = hash_grid(xt, tab, off, res)
    rel_f, _ = _rel_cos(_to_nf(y.cpu().numpy(), layout, N, L), e.detach().numpy())
    dly_nf = rng.normal(0, 1, (N, 2 * L)).astype(np.float32)
    dly_t = torch.tensor(dly_nf.astype(np.float64), requires_grad=True)
    S = (e * dly_t).sum()
    g_tab, g_x = torch.autograd.grad(S, (tab, xt), create_graph=True)
    v = rng.normal(0, 1, (N, 3)).astype(np.float32)
    S2 = (g_x * torch.tensor(v.astype(np.float64))).sum()
    g2_tab, g2_dly = torch.autograd.grad(S2, (tab, dly_t))
    dly_dev = t.from_numpy(_from_nf(dly_nf, layout, N, L)).cuda()
    g = t.zeros(m.n_params, dtype=t.float32, device="cuda")
    dx = t.zeros((N, 3), dtype=t.float32, device="cuda")
    m.backward(ctx, x, dly_dev, params, dL_dparams=g, dL_dinput=dx, mode=GradientMode.Overwrite)
    # dL_dinput summed per sample in feature order (kernel_grid_backward_input, grid.h:804-830): bitwise the same on a
    # second call (it was a float-atomic sum over the levels)
    dx2 = t.full((N, 3), 3.0, dtype=t.float32, device="cuda")
    m.backward(ctx, x, dly_dev, params, dL_dinput=dx2, mode=GradientMode.Ignore)
    np.testing.assert_array_equal(dx2.cpu().numpy(), dx.cpu().numpy())
    rel_p, cos_p = _rel_cos(g.cpu().numpy(), g_tab.detach().numpy().ravel())
    rel_x, _ = _rel_cos(dx.cpu().numpy(), g_x.detach().numpy())
    g2 = t.full((m.n_params,), 7.0, dtype=t.float32, device="cuda")  # Overwrite must not read the old contents
    ddo = t.zeros(m.output_shape(N), dtype=t.float32, device="cuda")
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dly_dev, params, dL_dparams=g2, dL_ddLdoutput=ddo)
    rel_p2, cos_p2 = _rel_cos(g2.cpu().numpy(), g2_tab.numpy().ravel())
    rel_o2, _ = _rel_cos(_to_nf(ddo.cpu().numpy(), layout, N, L), g2_dly.numpy())
    _record("module_encoding_fp32_" + layout, rel_forward=rel_f, rel_params=rel_p, rel_dinput=rel_x, rel_params_2nd=rel_p2,
            rel_ddLdoutput=rel_o2)
    # fp32 arithmetic: the level position x * scale + 0.5 (scale up to ~270 here) carries ~2^-24 * 270 of its fraction,
    # the interpolation weights that much (measured 5.5e-6 .. 7.8e-6 rel-L2)
    assert rel_f <= 3e-5, rel_f
    assert rel_p <= 3e-5 and cos_p >= 0.9999999, (rel_p, cos_p)
    assert rel_x <= 3e-5, rel_x
    assert rel_p2 <= 3e-5 and cos_p2 >= 0.9999999, (rel_p2, cos_p2)
    assert rel_o2 <= 3e-5, rel_o2
    acc = g.clone()
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dly_dev, params, dL_dparams=acc, mode=GradientMode.Accumulate)
    # (float atomics, as GridEncoding<float>'s: the summation order varies from call to call)
    np.testing.assert_allclose(acc.cpu().numpy(), g.cpu().numpy() + g2.cpu().numpy(), rtol=1e-5, atol=2e-5)
    # progressive levels: set_training_step(1) -> levels 0..4 (tcnn's defaults), the rest 0
    m.set_training_step(1)
    y3 = _to_nf(m.inference(x, params).cpu().numpy(), layout, N, L)
    assert not y3[:, 10:].any() and np.array_equal(y3[:, :10], _to_nf(y.cpu().numpy(), layout, N, L)[:, :10])


@pytest.mark.parametrize("n_levels,width", [(8, 64), (14, 64), (1, 16)])
def test_network_with_input_encoding_module(torch_cuda, n_levels, width):
    """create_network_with_input_encoding (cpp_api.h:108): HashGrid -> FullyFusedMLP (1 hidden ReLU layer) on the MFMA
    kernel k_dnet, against a float64 autograd restatement (tests/torch_ref.hash_grid + the MLP):
    * forward: the fp16 output within fp16 rounding of the float64 value;
    * backward (network_with_input_encoding.h:113-156): dL_dparams (MLP and grid blocks) and dL_dinput;
    * backward_backward_input (network_with_input_encoding.h:159-250, fully_fused_mlp.cu:1088-1198): the second-order
      parameter gradient = d/dtheta of sum(dL_ddLdinput . dL/dx) (ReLU'' = 0), MLP and grid blocks;
    * Accumulate adds; pcg32{seed} initialisation = xavier(W0), xavier(W1), then the grid (cpp_api.cu:162-165)."""
    import torch
    from torch_ref import grid_tables, hash_grid
    from neus2_amd.module import GradientMode, Module
    t = torch_cuda
    L, W = n_levels, width
    log2t = 14
    enc_cfg = {"otype": "HashGrid", "n_levels": L, "n_features_per_level": 2, "log2_hashmap_size": log2t, "base_resolution": 16,
               "per_level_scale": 1.5}
    net_cfg = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": W, "n_hidden_layers": 1,
               "gradient_precision": "fp32"}
    m = Module.create_network_with_input_encoding(3, 16, enc_cfg, net_cfg, batch_capacity=N)
    DE = (2 * L + 15) // 16 * 16
    off, res = grid_tables(L, log2t, 16, 1.5)
    n_mlp = W * DE + 16 * W
    assert m.n_params == n_mlp + 2 * off[-1] and m.n_output_dims == 16 and m.info["grid_offset"] == n_mlp
    assert m.name() == "NetworkWithInputEncoding"
    # initialisation from pcg32{1337}: the two xavier matrices, then the grid block continues the same generator
    p0 = m.initialize_params(1337).cpu().numpy()
    s0, s1 = np.sqrt(6.0 / (W + DE)), np.sqrt(6.0 / (16 + W))
    assert np.abs(p0[: W * DE]).max() <= s0 and np.abs(p0[W * DE:n_mlp]).max() <= s1 and np.abs(p0[n_mlp:]).max() <= 1e-4
    rng = np.random.default_rng(L)
    ph = np.concatenate([rng.normal(0, 0.3, W * DE), rng.normal(0, 0.3, 16 * W),
                         rng.uniform(-1, 1, 2 * off[-1])]).astype(np.float16)
    params = t.from_numpy(ph.view(np.int16).copy()).cuda()
    pos = rng.uniform(0.02, 0.98, (N, 3)).astype(np.float32)
    x = t.from_numpy(pos).cuda()
    ctx, y = m.forward(x, params, prepare_input_gradients=True)
    # float64 reference
    pd = torch.tensor(ph.astype(np.float64))
    w0 = pd[: W * DE].reshape(W, DE).clone().requires_grad_(True)
    w1 = pd[W * DE:n_mlp].reshape(16, W).clone().requires_grad_(True)
    tab = pd[n_mlp:].reshape(-1, 2).clone().requires_grad_(True)
    xt = torch.tensor(pos.astype(np.float64), requires_grad=True)
    e = hash_grid(xt, tab, off, res)
    ein = torch.nn.functional.pad(e, (0, DE - 2 * L))
    pre = ein @ w0.T
    hid = torch.relu(pre)
    out = hid @ w1.T
    yo = y.float().cpu().numpy()
    ro = out.detach().numpy()
    err = np.abs(yo - ro)
    assert np.mean(err <= 4e-3 + 4e-3 * np.abs(ro)) >= 0.995, np.max(err)
    dlo = rng.normal(0, 1, (N, 16)).astype(np.float16)
    # A pre-activation within fp16 rounding of 0 may take the other ReLU branch on the device (its encoding is fp16):
    # one such flip moves a float64 gradient by ~1% (a whole W1^T dL entry). Those samples get dL = 0, which removes
    # them from every first- and second-order term on both sides.
    ambiguous = (np.abs(pre.detach().numpy()) < 2e-3).any(axis=1)
    assert ambiguous.mean() < 0.5
    dlo[ambiguous] = 0
    dlo_t = torch.tensor(dlo.astype(np.float64))
    S = (out * dlo_t).sum()
    gw0, gw1, gtab, gx = torch.autograd.grad(S, (w0, w1, tab, xt), create_graph=True)
    v = rng.normal(0, 1, (N, 3)).astype(np.float32)
    S2 = (gx * torch.tensor(v.astype(np.float64))).sum()
    g2w0, g2w1, g2tab = torch.autograd.grad(S2, (w0, w1, tab))
    dlo_dev = t.from_numpy(dlo.view(np.int16).copy()).cuda()
    g = t.zeros(m.n_params, dtype=t.float32, device="cuda")
    dx = t.zeros((N, 3), dtype=t.float32, device="cuda")
    m.backward(ctx, x, dlo_dev, params, dL_dparams=g, dL_dinput=dx, mode=GradientMode.Overwrite)
    gm = g.cpu().numpy()
    blocks1 = {"W0": (gm[: W * DE], gw0), "W1": (gm[W * DE:n_mlp], gw1), "grid": (gm[n_mlp:], gtab), "dinput": (dx.cpu().numpy(), gx)}
    g2 = t.zeros(m.n_params, dtype=t.float32, device="cuda")
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dlo_dev, params, dL_dparams=g2, mode=GradientMode.Overwrite)
    g2m = g2.cpu().numpy()
    blocks2 = {"W0_2nd": (g2m[: W * DE], g2w0), "W1_2nd": (g2m[W * DE:n_mlp], g2w1), "grid_2nd": (g2m[n_mlp:], g2tab)}
    res_ = {}
    for name, (a, b) in {**blocks1, **blocks2}.items():
        res_[name] = _rel_cos(a, b.detach().numpy())
    _record(f"module_network_with_input_encoding_L{L}_W{W}", **{f"rel_{k}": v_[0] for k, v_ in res_.items()},
            **{f"cos_{k}": v_[1] for k, v_ in res_.items()})
    for name, (rel, cos) in res_.items():
        assert rel <= 5e-3 and cos >= 0.9999, (name, rel, cos)
    # Accumulate: the second-order gradient added onto the first-order one
    acc = g.clone()
    m.backward_backward_input(ctx, x, t.from_numpy(v).cuda(), dlo_dev, params, dL_dparams=acc, mode=GradientMode.Accumulate)
    np.testing.assert_allclose(acc.cpu().numpy(), gm + g2m, rtol=1e-6, atol=1e-6)
