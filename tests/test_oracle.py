"""CPU tests of the oracle (oracle/neus_oracle.cpp): known-answer vectors, the pinned parameter layout,
autograd cross-checks of the analytic first/second-order derivatives, and the committed golden fixtures."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _float(u):
    """pcg32::next_float (pcg32.h:98-106): 23 mantissa bits of next_uint."""
    return ((np.asarray(u, np.uint32) >> 9) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1)


def test_pcg32_published_kat():
    """PCG32 (O'Neill, pcg-c demo): pcg32_srandom(42, 54) -> 0xa15c02b7 0x7b47f409 0xba1d3330 ..."""
    got = O.pcg32(42, 54, 0, 6)
    want = [0xA15C02B7, 0x7B47F409, 0xBA1D3330, 0x83D2F293, 0xBFA4784B, 0xCBED606E]
    assert list(map(int, got)) == want


def test_pcg32_survey_probe():
    """the reference's pcg32.h probe gave {2023056239, 634364130} for pcg32{1337}
    (printed with two draws in one printf: the argument evaluation order of that probe is
    unspecified, so the pair is compared as a set; the first draw is fixed by the KAT above) and
    next_float() == 0.741770506 after advance(40)."""
    got = O.pcg32(1337, 1, 0, 2)
    assert sorted(map(int, got)) == sorted([2023056239, 634364130])
    f = _float(O.pcg32(1337, 1, 40, 1))[0]
    assert abs(float(f) - 0.741770506) < 1e-8


def test_pcg32_advance_is_skip():
    a = O.pcg32(7, 3, 0, 100)
    for k in (1, 17, 64, 99):
        assert int(O.pcg32(7, 3, k, 1)[0]) == int(a[k])


def test_param_layout_pinned_by_survey():
    """P = 10,559,396 (L=14) and 12,208,532 (L=16) for base.json; the matrix
    (L2-regularised) prefix is the 11,264 MLP weights at L=14."""
    l14 = O.layout(O.make_cfg(n_levels=14))
    l16 = O.layout(O.make_cfg(n_levels=16))
    assert l14["n_params"] == 10559396 and l14["n_matrix"] == 11264
    assert l16["n_params"] == 12208532


def test_f2h_matches_numpy_float16():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-1e-4, 1e-4, 50000), rng.uniform(-0.1, 0.1, 50000),
                        rng.standard_normal(50000) * np.exp2(rng.integers(-30, 20, 50000)),
                        [6.1e-5, 5.96e-8, 2.98e-8, 2.99e-8, 65504, 65519, 65520, 1e5, -0.0, np.inf, -np.inf]]).astype(np.float32)
    got = np.zeros(x.size, np.uint16)
    O.lib().or_f2h(O.P(x), O.P(got), C.c_uint64(x.size))
    with np.errstate(over="ignore"):
        np.testing.assert_array_equal(got, x.astype(np.float16).view(np.uint16))


def test_det_expf_accuracy():
    """det_expf: the fixed-operation-sequence expf both the oracle and the HIP march/loss kernels use."""
    xs = np.linspace(-80, 80, 20001).astype(np.float32)
    got = np.array([O.det_expf(float(v)) for v in xs], np.float32)
    ref = np.exp(xs.astype(np.float64))
    ok = ref < 3e38
    rel = np.abs(got[ok] - ref[ok]) / ref[ok]
    assert rel.max() < 4e-7


# ------------------------------------------------------------------ autograd cross-check (float64 torch)
def _small_net():
    torch = pytest.importorskip("torch")
    from torch_ref import Net
    cfg = O.make_cfg(n_levels=4, log2_hashmap_size=12, base_resolution=8, per_level_scale=2.0)
    net = Net(4, 12, 8, 2.0)
    lay = O.layout(cfg)
    assert net.n_params == lay["n_params"]
    rng = np.random.default_rng(3)
    p = O.init_params(cfg)
    din = cfg.density_in
    w0 = p[: 64 * din].reshape(64, din)
    w0[:, 3:3 + 8] = rng.normal(0, 0.3, (64, 8))
    p[lay["grid_off"]:lay["var_off"]] = rng.uniform(-0.1, 0.1, lay["n_grid_params"])
    # the oracle computes with fp16-rounded weights; give both sides the same values
    ph = p.astype(np.float16).astype(np.float32)
    ph[lay["var_off"]] = 0.3
    return torch, cfg, net, lay, ph


def _coords(n, seed=0):
    rng = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0.1, 0.9, (n, 3))
    c[:, 3] = 0.01
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c[:, 4:] = (d + 1) * 0.5
    return c


def test_oracle_forward_vs_autograd():
    torch, cfg, net, lay, p = _small_net()
    c = _coords(256)
    out = O.network_forward(cfg, p, c, 4).view(np.float16).astype(np.float64)
    f = net.forward(torch.tensor(p, dtype=torch.float64), torch.tensor(c, dtype=torch.float64))
    ref_rgb = f["rout"][:, :3].detach().numpy()
    ref_sdf = f["sdf"].detach().numpy()
    ref_g = f["gsdf"].detach().numpy()
    # fp16 storage of every activation (the reference's rounding points) vs exact float64: a ReLU whose
    # pre-activation is within fp16 noise of 0 can flip, so >= 99% of elements within tolerance and a
    # small median error
    def close(got, ref, tol):
        err = np.abs(got - ref)
        assert np.mean(err <= tol * (1 + np.abs(ref))) >= 0.99 and np.median(err) < tol / 10, (err.max(), np.median(err))
    close(out[:, :3], ref_rgb, 2e-2)
    close(out[:, 3], ref_sdf, 5e-3)
    close(out[:, 4:7] / np.abs(ref_g).max(), ref_g / np.abs(ref_g).max(), 2e-2)
    np.testing.assert_allclose(out[:, 7], 0.3, rtol=1e-3)
    np.testing.assert_array_equal(out[:, 8:11], c[:, 4:7].astype(np.float16).astype(np.float64))


@pytest.mark.parametrize("which", ["rgb", "sdf", "eikonal", "bentdir", "all"])
def test_oracle_backward_vs_autograd(which):
    """First- and second-order parameter gradients: per block cosine >= 0.998 and rel-L2 <= 7e-2
    (the oracle replicates the reference's fp16 rounding points; torch is exact float64; measured
    worst case 0.9990 / 4.6e-2 on d0 through the rgb path, dominated by the fp16-accumulated hash-grid features). Blocks the case does not reach must be
    exactly zero in both."""
    torch, cfg, net, lay, p = _small_net()
    n = 256
    c = _coords(n, 1)
    rng = np.random.default_rng({"rgb": 5, "sdf": 6, "eikonal": 7, "bentdir": 8, "all": 9}[which])
    d = np.zeros((n, 16), np.float32)
    if which in ("rgb", "all"):
        d[:, 0:3] = rng.normal(0, 1e-2, (n, 3))
    if which in ("sdf", "all"):
        d[:, 3] = rng.normal(0, 1e-2, n)
    if which in ("eikonal", "all"):
        d[:, 4:7] = rng.normal(0, 1.0, (n, 3))
        d[:, 7] = rng.normal(0, 1e-2, n)
    if which in ("bentdir", "all"):
        d[:, 8:11] = rng.normal(0, 1e-2, (n, 3))
    d16 = d.astype(np.float16)
    g_or = O.network_backward(cfg, p, c, 4, d16.view(np.uint16), n)
    g_t = net.backward(torch.tensor(p, dtype=torch.float64), torch.tensor(c, dtype=torch.float64),
                       torch.tensor(d16.astype(np.float64)), float(n)).numpy()
    checked = 0
    for k, (a, b, _) in net.slices.items():
        x, y = g_or[a:b].astype(np.float64), g_t[a:b]
        ny = np.linalg.norm(y)
        if ny < 1e-12:
            assert np.linalg.norm(x) < 1e-9, k
            continue
        cos = float(x @ y / (np.linalg.norm(x) * ny + 1e-300))
        rel = float(np.linalg.norm(x - y) / ny)
        assert cos >= 0.998 and rel <= 7e-2, (k, cos, rel)
        checked += 1
    assert checked >= 3


def test_grid_dydx_is_derivative():
    """dy/dx from the grid kernel equals the central finite difference of the fp32 interpolation."""
    torch, cfg, net, lay, p = _small_net()
    c = _coords(64, 2)[:, :3].astype(np.float64)
    tab = torch.tensor(p[lay["grid_off"]:lay["var_off"]].reshape(-1, 2), dtype=torch.float64)
    from torch_ref import hash_grid
    _, dydx = O.grid_forward(cfg, p, c.astype(np.float32), 4)
    x = torch.tensor(c, requires_grad=True)
    enc = hash_grid(x, tab, net.off, net.res)
    J = np.stack([torch.autograd.grad(enc[:, k].sum(), x, retain_graph=True)[0].numpy() for k in range(enc.shape[1])], 1)
    np.testing.assert_allclose(dydx, J, rtol=1e-4, atol=1e-4 * np.abs(J).max())


# ------------------------------------------------------------------ golden fixtures (tests/golden/make_golden.py)
def _golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} missing (run tests/golden/make_golden.py)")
    return np.load(path)


def test_golden_sampling_fixture():
    from make_golden import sampling_case
    g = _golden("sampling_small.npz")
    got = sampling_case()
    for k in ("rays", "numsteps", "coords"):
        np.testing.assert_array_equal(got[k].view(np.uint32), g[k].view(np.uint32), err_msg=k)
    assert int(got["counter"]) == int(g["counter"])


def test_golden_loss_fixture():
    from make_golden import loss_case
    g = _golden("loss_small.npz")
    got = loss_case()
    np.testing.assert_array_equal(got["numsteps"], g["numsteps"])
    np.testing.assert_array_equal(got["coords"].view(np.uint32), g["coords"].view(np.uint32))
    np.testing.assert_array_equal(got["dL_dout"], g["dL_dout"])
    assert int(got["counter"]) == int(g["counter"])


def test_golden_network_fixture():
    from make_golden import network_case
    g = _golden("network_small.npz")
    got = network_case()
    np.testing.assert_array_equal(got["out"], g["out"])
    # double-precision atomics under OpenMP: summation order varies run to run below fp32 resolution
    np.testing.assert_allclose(got["grads"], g["grads"], rtol=1e-6, atol=1e-7 * np.abs(g["grads"]).max())


def test_neus_loss_gradient_vs_autograd():
    """dL/d(network output) of the oracle's NeuS composite (rows 0..3 rgb/sdf, 7 variance, 8..10
    bent-dir, 4..6 eikonal) against float64 autograd of the same composite, per compacted sample:
    rows 0..3, 7, 8..10 within 2e-2 relative of each ray's largest gradient (fp16 network outputs,
    fp16-stored dL/dout, the reference's 1e-5 regularisers in its closed-form dalpha; rays with a
    sample of 1 - alpha < 1e-3 are skipped because that regulariser dominates there)."""
    torch = pytest.importorskip("torch")
    from make_golden import SAMPLE_RAYS, SAMPLE_RNG, loss_case, small_dataset
    from torch_ref import huber_sum, neus_ray_loss_grad
    sc, ds = small_dataset()
    g = loss_case()
    out = g["net_out"]
    ns = g["numsteps"]
    from neus2_amd import scenes
    bf = scenes.shell_bitfield(thickness=4.0 / 128)
    rays, ns0, co, counter, nr = O.generate_samples(ds, bf, SAMPLE_RAYS, 0, SAMPLE_RNG[0], SAMPLE_RNG[1], 1 << 14)
    ls = 128.0 / SAMPLE_RAYS
    n_checked = 0
    for i in range(SAMPLE_RAYS):
        comp, cb = int(ns[i, 0]), int(ns[i, 1])
        n_pre, base = int(ns0[i, 0]), int(ns0[i, 1])
        if comp < 2:
            continue
        lo = torch.tensor(out[base:base + n_pre].view(np.float16).astype(np.float64))
        dt = torch.tensor(co[base:base + n_pre, 3].astype(np.float64) * (1.7320508 / 1024 * (1 << 7) - 1.7320508 / 1024) + 1.7320508 / 1024)
        target, bg = O.ray_target(ds, i, SAMPLE_RAYS, 0, SAMPLE_RNG[0], SAMPLE_RNG[1])
        # the composite runs over the samples before transmittance drops below 1e-4 (cn); the gradient
        # is emitted for the first `comp` of them (the compaction cap can cut a ray short)
        _, _, _, a_all = neus_ray_loss_grad(lo, dt, None, None, SAMPLE_RAYS)
        T_before = np.concatenate([[1.0], np.cumprod(1 - a_all.numpy())[:-1]])
        cn = int(np.argmax(T_before < 1e-4)) if np.any(T_before < 1e-4) else n_pre
        lo, dt = lo[:cn], dt[:cn]
        lo_t, rgb, T_end, alpha = neus_ray_loss_grad(lo, dt, torch.tensor(target, dtype=torch.float64), None, SAMPLE_RAYS)
        if float((1 - alpha).min()) < 1e-3:
            # the reference's closed-form dalpha divides by (1 - alpha + 1e-5): more than 1% off the
            # exact derivative here, by design of the reference; such rays are not comparable
            continue
        if cn == n_pre:  # ran to its end before T < 1e-4: the background shows through
            rgb = rgb + T_end * torch.tensor(bg, dtype=torch.float64)
        S = huber_sum(rgb, torch.tensor(target, dtype=torch.float64)) * ls
        gt, = torch.autograd.grad(S, lo_t)
        gt = gt.numpy()[:comp]
        go = g["dL_dout"][cb:cb + comp].view(np.float16).astype(np.float64)
        # the composite's dL/d(grad sdf) (through cos = dir . grad_sdf) travels in rows 8..10; rows 4..6
        # carry only the eikonal term (nerf_network.h:478-504 adds both into dL/d(grad sdf))
        want = np.concatenate([gt[:, 0:4], gt[:, 7:8], gt[:, 4:7]], 1)
        got = np.concatenate([go[:, 0:4], go[:, 7:8], go[:, 8:11]], 1)
        scale = np.abs(want).max()
        if scale < 1e-6:
            continue
        np.testing.assert_allclose(got, want, atol=2e-2 * scale, rtol=2e-2, err_msg=f"ray {i}")
        # eikonal rows: ek_w * 2 * 128 * (1 - 1/|g|) g with |g| = sqrt(g.g + 1e-6)
        pg = lo.numpy()[:comp, 4:7]
        gn = np.sqrt((pg * pg).sum(1) + 1e-6)
        ek = 0.01 * 2 * 128.0 * (1 - 1 / gn)[:, None] * pg
        np.testing.assert_allclose(go[:, 4:7], ek, rtol=2e-3, atol=1e-3 * np.abs(ek).max())
        n_checked += 1
    assert n_checked >= 10, n_checked


def test_sobol_direction_numbers_match_reference_table():
    """random_val.cuh:160-200: dimension 0 is the bit reversal; the first 16 dimension-1 direction
    numbers of the reference's table (sobol(2^b, 1) = directions[1][b])."""
    dim1 = [0x80000000, 0xc0000000, 0xa0000000, 0xf0000000, 0x88000000, 0xcc000000, 0xaa000000, 0xff000000,
            0x80800000, 0xc0c00000, 0xa0a00000, 0xf0f00000, 0x88880000, 0xcccc0000, 0xaaaa0000, 0xffff0000]
    for b in range(32):
        assert O.sobol(1 << b, 0) == 1 << (31 - b)
    for b, want in enumerate(dim1):
        assert O.sobol(1 << b, 1) == want
    # XOR-linearity of a digital sequence
    assert O.sobol(0b1011, 1) == dim1[0] ^ dim1[1] ^ dim1[3]


def test_ld_random_val_properties():
    """ld_random_val (random_val.cuh:284-288): values in [0,1), and the 2-D variant's dimension 0 equals
    the 1-D value (both scramble index, then sobol dim 0 with hash_combine(seed, 0))."""
    vals = [O.ld_random_val(i, 786433 * 7) for i in range(64)]
    assert all(0.0 <= v < 1.0 for v in vals)
    assert len(set(vals)) == 64
    for i in range(8):
        assert O.ld_random_val_2d(i, 0xdeadbeef)[0] == np.float32(O.ld_random_val(i, 0xdeadbeef))


def test_oracle_render_small_scene():
    """Oracle render (render_to_cpu restatement) of the small sphere scene with geometric-init weights:
    finite, premultiplied colour <= alpha <= 1, more coverage at the image centre than in the corners
    (the geometric init is a sphere SDF around the aabb centre), deterministic."""
    from neus2_amd import scenes
    sc = scenes.small_scene(n_views=2, width=32, height=24)
    cfg = O.make_cfg(n_levels=4, per_level_scale=1.5)
    params = O.init_params(cfg, 1337, geo=True)
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    bf = np.full(128 ** 3 // 8 * 8, 0xff, np.uint8)
    args = (cfg, params, 4, ds, bf, sc["xforms"][0], np.asarray(sc["focal"][0]) * 24 / 48, sc["principal"][0], 32, 24)
    img, iters = O.render(*args, spp=1)
    img2, _ = O.render(*args, spp=1)
    assert iters > 0
    assert np.isfinite(img).all()
    np.testing.assert_array_equal(img, img2)
    a = img[..., 3]
    assert (a >= 0).all() and (a <= 1 + 1e-6).all()
    assert a[8:16, 12:20].mean() > a[:4, :4].mean()


def _sphere_sdf(res, r=0.3):
    ax = (np.arange(res) / res).astype(np.float32)
    z, y, x = np.meshgrid(ax, ax, ax, indexing="ij")
    return (np.sqrt((x - .5) ** 2 + (y - .5) ** 2 + (z - .5) ** 2) - r).astype(np.float32)


def test_mc_oracle_cpp_matches_python_restatement():
    """or_marching_cubes (C++, fma vertices) and mc_table.marching_cubes (numpy) agree on a random field."""
    import mc_table
    d = np.random.default_rng(0).normal(size=(9, 10, 11)).astype(np.float32)
    V, F = O.marching_cubes(d, 0.1)
    V2, F2 = mc_table.marching_cubes(d, 0.1)
    np.testing.assert_array_equal(F, F2)
    np.testing.assert_allclose(V, V2, rtol=0, atol=1e-6)


def test_mc_oracle_sphere_is_closed_and_accurate():
    """The generated case table gives a closed, consistently oriented surface (every directed edge once,
    its reverse once), outward normals, area and radius of the analytic sphere within grid error."""
    import collections
    d = _sphere_sdf(48)
    V, F = O.marching_cubes(d, 0.0)
    E = collections.Counter()
    for a, b, c in F:
        for u, v in ((a, b), (b, c), (c, a)):
            E[(int(u), int(v))] += 1
    assert max(E.values()) == 1
    assert all((v, u) in E for (u, v) in E)
    P = V[F.astype(np.int64)]
    n = np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0])
    area = 0.5 * np.linalg.norm(n, axis=1)
    out = ((n * (P.mean(1) - 0.5)).sum(1) > 0)
    assert area[out].sum() / area.sum() > 0.999
    assert abs(area.sum() - 4 * np.pi * 0.09) / (4 * np.pi * 0.09) < 0.01
    assert np.abs(np.linalg.norm(V - 0.5, axis=1) - 0.3).max() < 2.0 / 48


def _moved_params():
    p = np.zeros(12, np.float32)
    p[:3] = [0.01, -0.02, 0.005]
    p[4:10] = [0.99, 0.05, -0.02, -0.04, 1.01, 0.03]
    return p


def test_motion_restatement_identity_and_gradient():
    """oracle/motion.py (DeltaNetwork restatement): identity parameters move nothing (bit-exact), the rotation is
    orthonormal, and the reference's closed-form gradient (add_loss_to_rotation_6d_each +
    gradient_rotation_matrix_to_6d) agrees with central finite differences of the forward."""
    import motion as M
    rng = np.random.default_rng(0)
    p = np.zeros(12, np.float32); p[4] = 1; p[8] = 1
    c = rng.uniform(0, 1, (16, 7)).astype(np.float32)
    moved = M.delta_apply(p, c)
    np.testing.assert_array_equal(moved[:, :4], c[:, :4])  # positions and dt untouched
    np.testing.assert_allclose(moved[:, 4:], c[:, 4:], atol=1.2e-7)  # dir: (2d - 1 + 1) / 2 rounds
    p2 = _moved_params()
    R = M.rot6d_to_matrix([M.rh(v) for v in p2[4:10]]).reshape(3, 3).astype(np.float64)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-6)
    g = rng.normal(size=(6, 4)).astype(np.float32)
    x = rng.uniform(0, 1, (6, 3)).astype(np.float32)
    an = M.delta_grad(p2, x, g)

    def L(pp):
        return float((M.delta_apply(pp, x).astype(np.float64) * g[:, :3]).sum())
    for k in list(range(3)) + list(range(4, 10)):
        e = np.zeros(12, np.float32); e[k] = 1e-2
        num = (L(p2 + e) - L(p2 - e)) / 2e-2
        assert abs(an[k] - num) <= 5e-3 + 5e-3 * abs(num), (k, an[k], num)
    assert an[3] == 0 and an[10] == 0 and an[11] == 0


def test_motion_accumulation():
    """accumulate_global_movement: identity local movement keeps the accumulated transform; a pure translation t
    adds R_local (t_acc + t) = t_acc + t."""
    import motion as M
    Rt = np.concatenate([np.eye(3, dtype=np.float32), np.float32([[0.1], [0.2], [0.3]])], 1)
    p = np.zeros(12, np.float32); p[4] = 1; p[8] = 1
    np.testing.assert_array_equal(M.accumulate_movement(p, Rt), np.float16(Rt).astype(np.float32))
    p[:3] = [0.01, 0.02, -0.03]
    out = M.accumulate_movement(p, Rt)
    np.testing.assert_allclose(out[:, 3], [0.11, 0.22, 0.27], atol=2e-4)


def test_mc_edge_cases():
    """Empty / full grids give no mesh; a single set corner gives one triangle; res 2 is one cube."""
    for v in (-1.0, 1.0):
        V, F = O.marching_cubes(np.full((4, 5, 6), v, np.float32), 0.0)
        assert len(V) == 0 and len(F) == 0
    d = np.full((2, 2, 2), -1.0, np.float32)
    d[0, 0, 0] = 1.0
    V, F = O.marching_cubes(d, 0.0)
    assert len(V) == 3 and len(F) == 1
    np.testing.assert_allclose(sorted(map(tuple, V)), sorted([(0.25, 0, 0), (0, 0.25, 0), (0, 0, 0.25)]), atol=1e-7)


def test_oracle_sum_order_switch():
    """or_set_sum_order (the all-levels parity test's noise floor): the reversed summation order moves the fp16 outputs
    by at most a few ulps, and switching back restores the index-order results bit for bit."""
    cfg = O.make_cfg(n_levels=4, log2_hashmap_size=12, base_resolution=8, per_level_scale=2.0)
    lay = O.layout(cfg)
    rng = np.random.default_rng(5)
    p = O.init_params(cfg)
    p[lay["grid_off"]:lay["var_off"]] = rng.uniform(-0.1, 0.1, lay["n_grid_params"])
    c = _coords(512, seed=2)
    a = O.network_forward(cfg, p, c, 4)
    try:
        O.set_sum_order(True)
        b = O.network_forward(cfg, p, c, 4)
    finally:
        O.set_sum_order(False)
    a2 = O.network_forward(cfg, p, c, 4)
    np.testing.assert_array_equal(a, a2)
    fa, fb = a.view(np.float16).astype(np.float64), b.view(np.float16).astype(np.float64)
    assert np.abs(fa - fb).max() <= 1e-2 * max(1.0, np.abs(fa).max())


def test_oracle_grid_grad_modes():
    """or_set_grid_grad_mode (round 6): the reference's fp16 atomic operand (grid.h:418-421) and fp16 accumulator
    (grid.h:1433) against the exact sum. At a unit loss scale the fp16 operand stays within ~1e-3 of the exact grid
    gradient. Scaled down until the contributions fall below fp16's normal range (the bench runs at a loss scale of
    128 / 2^18 = 2^-11, testbed_nerf.cu:1765, with a converged network's small dL/denc), the operand alone moves a level by
    up to several percent - the effect that the device's scaled scatter records (grid.hip, record format) avoid. The MLP blocks are untouched by the mode, and "exact" is restored
    bit for bit."""
    cfg = O.make_cfg(n_levels=6, log2_hashmap_size=12, base_resolution=8, per_level_scale=2.0)
    lay = O.layout(cfg)
    off, _, _, _ = O.grid_tables(cfg)
    rng = np.random.default_rng(11)
    p = O.init_params(cfg, geo=False)  # the geometric init zeroes the density MLP's grid-feature columns
    p[lay["grid_off"]:lay["var_off"]] = rng.uniform(-0.1, 0.1, lay["n_grid_params"])
    c = _coords(2048, seed=3)
    g0, g1 = lay["grid_off"], lay["var_off"]

    def grads(scale, mode):
        d = (rng_d.standard_normal((c.shape[0], 16)) * scale).astype(np.float16).view(np.uint16)
        O.set_grid_grad_mode(mode)
        try:
            return O.network_backward(cfg, p, c, 6, d, c.shape[0]).astype(np.float64)
        finally:
            O.set_grid_grad_mode("exact")

    def level_rel(a, b):
        out = []
        for l in range(cfg.n_levels):
            s, e = g0 + 2 * int(off[l]), g0 + 2 * int(off[l + 1])
            out.append(np.linalg.norm(a[s:e] - b[s:e]) / max(np.linalg.norm(b[s:e]), 1e-30))
        return np.array(out)

    for scale, lo, hi in ((1.0, 0.0, 2e-3), (2.0 ** -18, 5e-3, 1.0)):
        rng_d = np.random.default_rng(7)
        ex = grads(scale, "exact")
        rng_d = np.random.default_rng(7)
        op = grads(scale, "ref_operand")
        rng_d = np.random.default_rng(7)
        hf = grads(scale, "ref_half")
        np.testing.assert_array_equal(ex[:g0], op[:g0])
        np.testing.assert_array_equal(ex[:g0], hf[:g0])
        r_op, r_hf = level_rel(op, ex), level_rel(hf, ex)
        assert r_op.max() <= hi and r_op.max() >= lo, (scale, r_op)
        assert r_hf.max() >= r_op.max() * 0.5, (scale, r_hf, r_op)
        rng_d = np.random.default_rng(7)
        np.testing.assert_array_equal(grads(scale, "exact"), ex)
