"""tcnn::cpp::create_network (cpp_api.h:109; cpp_api.cu:170-172): an Identity encoding (inputs padded to 16 with ones,
identity.h:44-70) in front of a FullyFusedMLP (fully_fused_mlp.cu), on the gfx950 MFMA kernels (ffmlp.hip), against a
float64 torch restatement on the same fp16 parameters:
* initialize_params: pcg32{seed} xavier-uniform per matrix in order (fully_fused_mlp.cu:1229-1256), bit-exact;
* forward (hidden activation on every layer, output activation on the last; fp16 storage): within fp16 tolerance;
* backward: dL_dparams (fp32 precision mode) and dL_dinput vs autograd; Accumulate adds, fp16 mode rounds;
* backward_backward_input (ReLU networks, linear output: tcnn's fronts / backs chain is exact there, relu'' = 0):
  dL_dparams vs the autograd gradient of <dL_ddLdinput, d<dL_doutput, y>/dx>.
Tolerances: rel-L2 <= 2e-2 and cosine >= 0.999 per weight matrix (fp16 storage of activations and deltas)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [
    dict(n_in=32, n_out=3, W=64, N=2, act="ReLU", out_act="None"),
    dict(n_in=3, n_out=16, W=16, N=1, act="ReLU", out_act="None"),
    dict(n_in=40, n_out=4, W=128, N=3, act="ReLU", out_act="Sigmoid"),
    dict(n_in=20, n_out=1, W=32, N=2, act="Softplus", out_act="Exponential"),
    dict(n_in=8, n_out=5, W=64, N=1, act="Sigmoid", out_act="None"),
]


def _record(test, **metrics):
    import json
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "parity_metrics.jsonl"), "a") as f:
        f.write(json.dumps({"test": test, **{k: float(v) for k, v in metrics.items()}}) + "\n")


def _act(name, x, torch):
    if name == "ReLU":
        return torch.relu(x)
    if name == "Exponential":
        return torch.exp(x)
    if name == "Sigmoid":
        return torch.sigmoid(x)
    if name == "Softplus":
        return torch.log(torch.exp(x * 10.0) + 1.0) / 10.0
    return x


def _shapes(c):
    in_pad, out_pad = (c["n_in"] + 15) // 16 * 16, (c["n_out"] + 15) // 16 * 16
    return [(c["W"], in_pad)] + [(c["W"], c["W"])] * (c["N"] - 1) + [(out_pad, c["W"])], in_pad, out_pad


def _mats(c, p):
    shapes, _, _ = _shapes(c)
    out, off = [], 0
    for r, k in shapes:
        out.append(p[off: off + r * k].reshape(r, k))
        off += r * k
    return out


def _r16_fn(torch):
    class R16(torch.autograd.Function):
        """fp16 storage of a value and of the gradient flowing back through it (the kernels store activations and
        deltas in fp16); differentiable, so double backward works."""

        @staticmethod
        def forward(ctx, v):
            return v.to(torch.float16).to(torch.float64)

        @staticmethod
        def backward(ctx, g):
            return R16.apply(g)
    return R16.apply


def _ref_forward(c, mats, x, torch):
    """float64 restatement on the fp16 parameters and fp16-rounded input; every layer's sum and output, and the deltas
    flowing back through them, are rounded to fp16 as the kernels store them."""
    _, in_pad, _ = _shapes(c)
    n = x.shape[0]
    r16 = _r16_fn(torch)

    h = torch.cat([x, torch.ones(n, in_pad - c["n_in"], dtype=torch.float64)], 1)
    for l, Wm in enumerate(mats):
        z = r16(h @ Wm.T)
        h = r16(_act(c["out_act"] if l == len(mats) - 1 else c["act"], z, torch))
    return h


def _net(c, precision="fp32"):
    from neus2_amd.module import Module
    return Module.create_network(c["n_in"], c["n_out"], {"otype": "FullyFusedMLP", "n_neurons": c["W"], "n_hidden_layers": c["N"],
                                                          "activation": c["act"], "output_activation": c["out_act"],
                                                          "gradient_precision": precision}, batch_capacity=1024)


def _rel_cos(x, y):
    x, y = np.asarray(x, np.float64).ravel(), np.asarray(y, np.float64).ravel()
    return np.linalg.norm(x - y) / max(np.linalg.norm(y), 1e-30), x @ y / max(np.linalg.norm(x) * np.linalg.norm(y), 1e-30)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_ffmlp_module(torch_cuda, case):
    import oracle as O
    from neus2_amd.module import GradientMode
    t = torch_cuda
    c = CASES[case]
    shapes, in_pad, out_pad = _shapes(c)
    m = _net(c)
    P = sum(r * k for r, k in shapes)
    assert m.n_params == P and m.n_input_dims == c["n_in"] and m.n_output_dims == out_pad
    assert m.hyperparams()["network"]["n_hidden_layers"] == c["N"]
    # initialize_params: pcg32{seed} xavier per matrix (gpu_matrix.h:292-306), bit-exact
    p32 = m.initialize_params(seed=7).cpu().numpy()
    u = O.pcg32(7, 1, 0, P)
    f = ((u >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1)
    ref, off = np.zeros(P, np.float32), 0
    for r, k in shapes:
        sc = np.float32(np.sqrt(np.float32(6.0) / np.float32(r + k)))
        ref[off: off + r * k] = f[off: off + r * k] * np.float32(2) * sc - sc
        off += r * k
    np.testing.assert_array_equal(p32, ref)
    # moderate weights so every activation stays in its interesting range
    p16 = (p32 * 0.8).astype(np.float16)
    params = t.from_numpy(p16.view(np.int16)).cuda()
    n = 512
    rng = np.random.default_rng(case)
    x = rng.uniform(-1, 1, (n, c["n_in"])).astype(np.float32)
    xd = t.from_numpy(x).cuda()
    ctx, y = m.forward(xd, params)
    t.cuda.synchronize()
    got = y.cpu().numpy().astype(np.float32)
    mats = [t.tensor(a.astype(np.float64), requires_grad=True) for a in _mats(c, p16.astype(np.float32))]
    xr = t.tensor(x.astype(np.float16).astype(np.float64), requires_grad=True)
    yr = _ref_forward(c, mats, xr, t)
    err = np.abs(got - yr.detach().numpy())
    tol = 2e-2 * np.abs(yr.detach().numpy()) + 5e-3
    _record(f"ffmlp_forward_{case}", frac_within=(err <= tol).mean(), max_err=err.max())
    assert (err <= tol).mean() >= 0.995, (err.max(), (err <= tol).mean())
    # backward: dL_dparams (fp32 mode) and dL_dinput vs autograd
    dL = rng.normal(0, 1, (n, out_pad)).astype(np.float16)
    dLd = t.from_numpy(dL.view(np.int16)).cuda()
    g = t.zeros(P, dtype=t.float32, device="cuda")
    dx = t.zeros((n, c["n_in"]), dtype=t.float32, device="cuda")
    m.backward(ctx, xd, dLd, params, dL_dparams=g, dL_dinput=dx, output=y)
    (yr * t.from_numpy(dL.astype(np.float64))).sum().backward()
    gref = np.concatenate([a.grad.numpy().ravel() for a in mats])
    off = 0
    for l, (r, k) in enumerate(shapes):
        rel, cos = _rel_cos(g.cpu().numpy()[off: off + r * k], gref[off: off + r * k])
        _record(f"ffmlp_backward_{case}_W{l}", rel=rel, cos=cos)
        assert rel <= 2e-2 and cos >= 0.999, (l, rel, cos)
        off += r * k
    rel, cos = _rel_cos(dx.cpu().numpy(), xr.grad.numpy())
    _record(f"ffmlp_dinput_{case}", rel=rel, cos=cos)
    assert rel <= 2e-2 and cos >= 0.999, (rel, cos)
    # Accumulate adds to the caller's buffer; fp16 gradients are the fp32 ones rounded
    g2 = g.clone()
    m.backward(ctx, xd, dLd, params, dL_dparams=g2, mode=GradientMode.Accumulate, output=y)
    np.testing.assert_allclose(g2.cpu().numpy(), 2 * g.cpu().numpy(), rtol=1e-6, atol=1e-30)
    m16 = _net(c, "fp16")
    ctx16, y16 = m16.forward(xd, params)
    g16 = m16.gradient_buffer()
    m16.backward(ctx16, xd, dLd, params, dL_dparams=g16, output=y16)
    np.testing.assert_array_equal(g16.cpu().numpy(), g.cpu().numpy().astype(np.float16))


@pytest.mark.parametrize("case", [0, 1])
def test_ffmlp_backward_backward_input(torch_cuda, case):
    t = torch_cuda
    c = CASES[case]
    shapes, in_pad, out_pad = _shapes(c)
    m = _net(c)
    P = sum(r * k for r, k in shapes)
    p16 = (m.initialize_params(seed=3).cpu().numpy() * 0.8).astype(np.float16)
    params = t.from_numpy(p16.view(np.int16)).cuda()
    n = 512
    rng = np.random.default_rng(10 + case)
    x = rng.uniform(-1, 1, (n, c["n_in"])).astype(np.float32)
    xd = t.from_numpy(x).cuda()
    ctx, y = m.forward(xd, params)
    dL = rng.normal(0, 1, (n, out_pad)).astype(np.float16)
    u = rng.normal(0, 1, (n, c["n_in"])).astype(np.float32)
    g = t.zeros(P, dtype=t.float32, device="cuda")
    m.backward_backward_input(ctx, xd, t.from_numpy(u).cuda(), t.from_numpy(dL.view(np.int16)).cuda(), params, dL_dparams=g)
    mats = [t.tensor(a.astype(np.float64), requires_grad=True) for a in _mats(c, p16.astype(np.float32))]
    xr = t.tensor(x.astype(np.float16).astype(np.float64), requires_grad=True)
    yr = _ref_forward(c, mats, xr, t)
    (gx,) = t.autograd.grad((yr * t.from_numpy(dL.astype(np.float64))).sum(), xr, create_graph=True)
    S = (gx * t.from_numpy(u.astype(np.float16).astype(np.float64))).sum()
    grads = t.autograd.grad(S, mats)
    gref = np.concatenate([a.numpy().ravel() for a in grads])
    off = 0
    for l, (r, k) in enumerate(shapes):
        rel, cos = _rel_cos(g.cpu().numpy()[off: off + r * k], gref[off: off + r * k])
        _record(f"ffmlp_bwdbwd_{case}_W{l}", rel=rel, cos=cos)
        assert rel <= 2e-2 and cos >= 0.999, (l, rel, cos)
        off += r * k
