"""BASELINE.json's configs beyond base.json's 14 levels, through the HIP path against the oracle:
* config 1: the 1-view 64x64 synthetic sphere with a 1-level grid and width-16 MLPs;
* config 2 as BASELINE.json words it: a 16-level hash grid with width-64 MLPs.
Per config: Trainer init bit-exact, grid encode bit-exact (enc, dy/dx), network forward / backward within the
tolerances of test_gpu_parity, and a 16-step free-running training trajectory against oracle/cpu_step.py
(compacted counts within 1 %, parameter-change cosine >= 0.98 per block)."""
import ctypes as C
import os

import numpy as np
import pytest

from gpu_util import dev, host, ptr

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 4096
CONFIGS = {
    "config1_L1_W16": dict(n_levels=1, n_neurons=16, views=1, width=64, height=64),
    "config2_L16_W64": dict(n_levels=16, n_neurons=64, views=8, width=64, height=48),
}


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


@pytest.fixture(scope="module", params=sorted(CONFIGS))
def cfgenv(request, torch_cuda):
    import oracle as O
    from neus2_amd import config, pyngp, scenes
    k = CONFIGS[request.param]
    if k["views"] == 1:
        sc = scenes.sphere_scene(1, k["width"], k["height"], (70.0, 70.0), (0.5, 0.5), distance=1.6)
    else:
        sc = scenes.small_scene(n_views=k["views"], width=k["width"], height=k["height"])
    cfg_dict = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    cfg_dict["encoding"]["n_levels"] = k["n_levels"]
    cfg_dict["network"]["n_neurons"] = k["n_neurons"]
    cfg_dict["rgb_network"]["n_neurons"] = k["n_neurons"]
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_json(cfg_dict, batch_size=BATCH)
    ocfg = O.make_cfg(n_levels=k["n_levels"], width=k["n_neurons"], per_level_scale=tb._net_cfg.per_level_scale)
    return dict(name=request.param, tb=tb, O=O, cfg=ocfg, sc=sc, t=torch_cuda, L=k["n_levels"], W=k["n_neurons"], cfg_dict=cfg_dict)


def test_config_init_encode_forward_backward(cfgenv):
    from neus2_amd._lib import check, lib
    e = cfgenv
    O, tb, t, L, W = e["O"], e["tb"], e["t"], e["L"], e["W"]
    lay = tb.layout()
    assert lay["n_levels"] == L
    ref = np.zeros(O.layout(e["cfg"])["n_params"], np.float32)
    O.lib().or_init_params(C.byref(e["cfg"]), C.c_uint32(1337), O.P(tb._geo), O.P(ref))
    np.testing.assert_array_equal(tb.get_params(), ref)
    # parameters that exercise every path
    rng = np.random.default_rng(5)
    p = tb.get_params().copy()
    din = lay["density_input_width"]
    w0 = p[: W * din].reshape(W, din)
    w0[:, 3:3 + 2 * L] = rng.normal(0, 0.3, (W, 2 * L))
    p[: W * din] = w0.reshape(-1)
    p[lay["grid_offset"]:lay["variance_offset"]] = rng.uniform(-0.1, 0.1, lay["variance_offset"] - lay["grid_offset"])
    tb.set_params(p)
    n = 1024
    c = _coords(n, 1)
    enc = t.zeros((L, n, 2), dtype=t.int16, device="cuda")
    dydx = t.zeros((6 * L, n), dtype=t.float32, device="cuda")
    check(lib().neus_grid_encode(tb.handle, None, C.c_uint32(n), C.c_uint32(n), ptr(dev(t, c)), C.c_uint32(7), C.c_uint32(L), ptr(enc), ptr(dydx)))
    t.cuda.synchronize()
    got = host(enc, np.float16).astype(np.float32).transpose(1, 0, 2).reshape(n, 2 * L)
    gdy = host(dydx, np.float32).reshape(L, 2, 3, n).transpose(3, 0, 1, 2).reshape(n, 2 * L, 3)
    renc, rdy = O.grid_forward(e["cfg"], p, c[:, :3], L)
    np.testing.assert_array_equal(got.view(np.uint32), renc.astype(np.float32).view(np.uint32))
    np.testing.assert_array_equal(gdy.view(np.uint32), rdy.view(np.uint32))
    out = t.zeros((n, 16), dtype=t.int16, device="cuda")
    check(lib().neus_net_forward(tb.handle, None, C.c_uint32(n), ptr(dev(t, c)), C.c_uint32(L), ptr(out)))
    t.cuda.synchronize()
    fo = host(out, np.float16).astype(np.float32)
    ro = O.network_forward(e["cfg"], p, c, L).view(np.float16).astype(np.float32)
    err = np.abs(fo[:, :11] - ro[:, :11])
    ok = np.all(err <= 2e-3 + 4e-3 * np.abs(ro[:, :11]), axis=1)
    dl = np.zeros((n, 16), np.float32)
    dl[:, :4] = rng.normal(0, 1e-2, (n, 4))
    dl[:, 4:7] = rng.normal(0, 1.0, (n, 3))
    dl[:, 7] = rng.normal(0, 1e-2, n)
    dl[:, 8:11] = rng.normal(0, 1e-2, (n, 3))
    dl16 = dl.astype(np.float16)
    g = t.zeros(lay["n_params"], dtype=t.float32, device="cuda")
    check(lib().neus_net_backward(tb.handle, None, C.c_uint32(n), ptr(dev(t, c)), C.c_uint32(L), ptr(dev(t, dl16)), C.c_uint32(n), ptr(g)))
    t.cuda.synchronize()
    gg = g.cpu().numpy()
    gr = O.network_backward(e["cfg"], p, c, L, dl16.view(np.uint16), n)
    res = {}
    for name, (a, b) in {"density": (0, lay["n_density"]), "rgb": (lay["n_density"], lay["n_matrix"]),
                         "grid": (lay["grid_offset"], lay["variance_offset"]),
                         "variance": (lay["variance_offset"], lay["variance_offset"] + 1)}.items():
        x, y = gg[a:b].astype(np.float64), gr[a:b].astype(np.float64)
        res[name] = (np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30), x @ y / max(np.linalg.norm(x) * np.linalg.norm(y), 1e-30))
    _record(e["name"] + "_net", forward_frac_within_tol=ok.mean(), forward_median_err=np.median(err),
            **{f"rel_{k}": v[0] for k, v in res.items()}, **{f"cos_{k}": v[1] for k, v in res.items()})
    assert ok.mean() >= 0.995 and np.median(err) < 1e-3, ok.mean()
    for name, (rel, cos) in res.items():
        assert rel <= 2e-2 and cos >= 0.999, (name, rel, cos)


def test_config_train_trajectory(cfgenv):
    import oracle as O
    from cpu_step import CpuTrainer
    from neus2_amd import pyngp
    e = cfgenv
    sc = e["sc"]
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_json(e["cfg_dict"], batch_size=BATCH)
    lay = tb.layout()
    p0 = tb.get_params()
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    tr = CpuTrainer(e["cfg"], ds, p0, batch=BATCH, rays_per_batch=BATCH)
    gc, cc = [], []
    for _ in range(16):
        tb.train_steps(1)
        tr.step()
        gc.append(tb.stats()["measured_batch_size"])
        cc.append(tr.last["compacted"])
    gc, cc = np.array(gc, np.float64), np.array(cc, np.float64)
    rel_c = np.abs(gc - cc) / np.maximum(cc, 1)
    pg, pc = tb.get_params().astype(np.float64), tr.params.astype(np.float64)
    res = {}
    for name, (a, b) in {"density": (0, lay["n_density"]), "rgb": (lay["n_density"], lay["n_matrix"]),
                         "grid": (lay["grid_offset"], lay["variance_offset"])}.items():
        x, y = pg[a:b] - p0[a:b], pc[a:b] - p0[a:b]
        res[name] = (x @ y / max(np.linalg.norm(x) * np.linalg.norm(y), 1e-30), np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30))
    _record(e["name"] + "_trajectory", max_rel_compacted=rel_c.max(), **{f"cos_{k}": v[0] for k, v in res.items()},
            **{f"rel_{k}": v[1] for k, v in res.items()})
    assert cc.min() > 0 and rel_c.max() <= 0.01, (gc, cc)
    for name, (cos, rel) in res.items():
        assert cos >= 0.98 and rel <= 0.25, (name, cos, rel)


def test_config_occupancy_update(cfgenv):
    """update_density_grid_nerf at step 0 (all 128^3 cells, uniform samples) on the config's network against
    or_density_grid_update (tolerances of test_gpu_train_parity.test_occupancy_update_parity)."""
    import oracle as O
    from neus2_amd import pyngp
    from neus2_amd._lib import check, lib
    e = cfgenv
    sc = e["sc"]
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_json(e["cfg_dict"], batch_size=BATCH)
    G3 = 128 ** 3
    rs, ri = tb.get_rng()[2:4]
    params = tb.get_params()
    check(lib().neus_occ_update(tb.handle, None, C.c_uint32(G3), C.c_uint32(0)))
    g, bf = tb.get_density_grid()
    rg = np.zeros(G3, np.float32)
    rbf = np.zeros(G3 // 8 * 8, np.uint8)
    O.density_grid_update(e["cfg"], params, e["L"], G3, 0, 0, rs, ri, rg, rbf)
    err = np.abs(g - rg)
    ok = err <= 2e-2 * np.abs(rg) + 2e-3
    bits = np.unpackbits(bf) != np.unpackbits(rbf)
    _record(e["name"] + "_occupancy", frac_within_tol=ok.mean(), bit_mismatch=bits.mean(), occ_gpu=np.unpackbits(bf[: G3 // 8]).mean(),
            occ_ref=np.unpackbits(rbf[: G3 // 8]).mean(), mean_gpu=float(g.mean()), mean_ref=float(rg.mean()))
    assert ok.mean() >= 0.999 and bits.mean() <= 2e-3, (ok.mean(), bits.mean())
