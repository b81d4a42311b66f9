"""Float64 PyTorch (CPU) restatement of the NeuS2 network — TEST INFRASTRUCTURE ONLY.

Used to validate the oracle's analytic first- and second-order derivatives (oracle/neus_oracle.cpp
net_backward_one / grid_scatter_one) by autograd double-backward, as SURVEY.md §8(c).3 prescribes.
It is written from the network definition, not from the oracle:

  enc   = multiresolution hash-grid trilinear interpolation    (my_tcnn grid.h:174-369)
  din   = [x - 0.5, enc, 0...]                                 (nerf_network.h:206-212)
  dout  = W1 relu(W0 din);  sdf = dout[0] + sdf_bias          (fully_fused_mlp.cu:678-812)
  gsdf  = d dout[0] / dx   (autograd, create_graph)           (nerf_network.h:228-253)
  rin   = [dout(16), SH4(dir)(16), x(3), gsdf(3), 0...]        (nerf_network.h:262-280)
  rout  = R2 relu(R1 relu(R0 rin))                             (rgb MLP, 2 hidden layers)

The reference's backward (nerf_network.h:330-601) is the gradient of the scalar
  S = sum_i [ dLo[0:3].rout[0:3] + dLo[3] sdf + (dLo[4:7]/Nb + dLo[8:11]) . gsdf + dLo[7] var ]
with respect to all parameters (Nb = indeed batch size); ReLU'' = 0 as in autograd.
"""
from __future__ import annotations

import numpy as np
import torch

PRIMES = (1, 2654435761, 805459861)


def grid_tables(n_levels, log2_hashmap_size, base_resolution, per_level_scale):
    """Level offsets/resolutions (grid.h:1441-1510), float32 like the reference."""
    off, res = [0], []
    for l in range(n_levels):
        s = np.float32(np.exp2(np.float32(l) * np.float32(np.log2(np.float64(per_level_scale))))) * np.float32(base_resolution) - np.float32(1)
        r = int(np.ceil(s)) + 1
        p = min((r ** 3 + 7) // 8 * 8, 1 << log2_hashmap_size)
        res.append(r)
        off.append(off[-1] + p)
    return off, res


def _index(hsize, res, g):
    """grid_index (grid.h:118-153): dense while res^d fits, else the xor-prime hash."""
    stride, idx, dense = 1, torch.zeros_like(g[..., 0]), True
    for d in range(3):
        if stride > hsize:
            dense = False
            break
        idx = idx + g[..., d] * stride
        stride *= res
    if hsize < stride:
        dense = False
    if not dense:
        h = torch.zeros_like(g[..., 0])
        for d in range(3):
            h = h ^ ((g[..., d] * PRIMES[d]) & 0xFFFFFFFF)
        idx = h
    return idx % hsize


def hash_grid(x, table, off, res, valid_level=None):
    """x: [N,3] float64 in [0,1]; table: [n_entries, 2] float64. Returns [N, 2L]."""
    outs = []
    L = len(res)
    for l in range(L):
        if valid_level is not None and l > valid_level:
            outs.append(torch.zeros(x.shape[0], 2, dtype=x.dtype))
            continue
        scale = float(res[l] - 1)
        p = x * scale + 0.5
        g = torch.floor(p.detach()).to(torch.int64)
        f = p - g.to(x.dtype)
        acc = 0
        for c in range(8):
            bits = [(c >> d) & 1 for d in range(3)]
            w = 1
            for d in range(3):
                w = w * (f[:, d] if bits[d] else 1 - f[:, d])
            gc = g + torch.tensor(bits, dtype=torch.int64)
            e = _index(off[l + 1] - off[l], res[l], gc) + off[l]
            acc = acc + w[:, None] * table[e]
        outs.append(acc)
    return torch.cat(outs, dim=1)


def sh4(wd):
    x, y, z = (wd[:, 0] * 2 - 1), (wd[:, 1] * 2 - 1), (wd[:, 2] * 2 - 1)
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    one = torch.ones_like(x)
    return torch.stack([
        0.28209479177387814 * one, -0.48860251190291987 * y, 0.48860251190291987 * z, -0.48860251190291987 * x,
        1.0925484305920792 * xy, -1.0925484305920792 * yz, 0.94617469575755997 * z2 - 0.31539156525251999,
        -1.0925484305920792 * xz, 0.54627421529603959 * x2 - 0.54627421529603959 * y2,
        0.59004358992664352 * y * (-3.0 * x2 + y2), 2.8906114426405538 * xy * z, 0.45704579946446572 * y * (1.0 - 5.0 * z2),
        0.3731763325901154 * z * (5.0 * z2 - 3.0), 0.45704579946446572 * x * (1.0 - 5.0 * z2), 1.4453057213202769 * z * (x2 - y2),
        0.59004358992664352 * x * (-x2 + 3.0 * y2)], dim=1)


class Net:
    """Parameter views over one flat float64 tensor, in the reference layout
    density | rgb | grid | variance(4) (nerf_network.h:741-785)."""

    def __init__(self, n_levels, log2_hashmap_size, base_resolution, per_level_scale, width=64, sdf_bias=-0.1):
        self.L, self.W = n_levels, width
        self.din = ((3 + 2 * n_levels) + 15) // 16 * 16
        self.rin = 48
        self.off, self.res = grid_tables(n_levels, log2_hashmap_size, base_resolution, per_level_scale)
        W = width
        shapes = [("d0", (W, self.din)), ("d1", (16, W)), ("r0", (W, self.rin)), ("r1", (W, W)), ("r2", (16, W)),
                  ("grid", (self.off[-1], 2)), ("var", (4,))]
        self.slices, o = {}, 0
        for k, s in shapes:
            n = int(np.prod(s))
            self.slices[k] = (o, o + n, s)
            o += n
        self.n_params = o
        self.sdf_bias = sdf_bias

    def view(self, p, k):
        a, b, s = self.slices[k]
        return p[a:b].view(*s)

    def forward(self, p, coords, valid_level=None):
        """coords: [N,7] (x, dt, warped dir). Returns dict of rout, sdf, gsdf, var (float64, autograd-connected)."""
        x = coords[:, :3].clone().requires_grad_(True)
        enc = hash_grid(x, self.view(p, "grid"), self.off, self.res, valid_level)
        n = x.shape[0]
        din = torch.zeros(n, self.din, dtype=p.dtype)
        din = torch.cat([x - 0.5, enc, din[:, 3 + 2 * self.L:]], dim=1)
        h = torch.relu(din @ self.view(p, "d0").T)
        dout = h @ self.view(p, "d1").T
        gsdf, = torch.autograd.grad(dout[:, 0].sum(), x, create_graph=True)
        rin = torch.cat([dout, sh4(coords[:, 4:7]), x, gsdf, torch.zeros(n, self.rin - 38, dtype=p.dtype)], dim=1)
        h1 = torch.relu(rin @ self.view(p, "r0").T)
        h2 = torch.relu(h1 @ self.view(p, "r1").T)
        rout = h2 @ self.view(p, "r2").T
        return dict(rout=rout, sdf=dout[:, 0] + self.sdf_bias, gsdf=gsdf, var=self.view(p, "var")[0], dout=dout)

    def backward(self, p, coords, dLo, indeed_batch, valid_level=None):
        """Gradient of S (module docstring) w.r.t. all parameters."""
        p = p.detach().clone().requires_grad_(True)
        f = self.forward(p, coords, valid_level)
        S = (dLo[:, 0:3] * f["rout"][:, 0:3]).sum() + (dLo[:, 3] * f["sdf"]).sum()
        S = S + ((dLo[:, 4:7] / indeed_batch + dLo[:, 8:11]) * f["gsdf"]).sum() + dLo[:, 7].sum() * f["var"]
        g, = torch.autograd.grad(S, p)
        return g


def neus_ray_loss_grad(lo, dt, target, bg, n_rays_global, loss_scale=128.0, ek_w=0.01, cos_anneal=1.0):
    """Float64 NeuS composite of one ray's first `len(lo)` samples (all of them contribute; the caller
    passes the compacted samples) and autograd dL/d(network output) rows, in the reference's scaling.

    lo: [n,16] float64 network output rows; dt: [n] step sizes; target/bg: sRGB (3,).
    Follows compute_loss_kernel_train_nerf (testbed_nerf.cu:1475-1997) semantically:
      inv_s = exp(10 var); cos = dir.grad_sdf; iter_cos = -(relu(.5-.5cos)(1-a) + relu(-cos) a)
      alpha = clamp((cdf(prev) - cdf(next) + 1e-5) / (cdf(prev) + 1e-5), 0, 1)
      rgb_ray = sum w_j sigmoid(raw_j) (+ T bg when the ray ran to its end: `with_bg`)
    The reference differentiates the channel SUM of Huber(0.1)/5 (its reported loss is the mean,
    its gradient the sum) scaled by loss_scale / n_rays_global; rows 4..6 carry the eikonal term
    ek_w * 2 * loss_scale * (1 - 1/|g|) g (not divided by n_rays)."""
    lo = lo.clone().requires_grad_(True)
    raw, sdf, pg, var = lo[:, 0:3], lo[:, 3], lo[:, 4:7], lo[:, 7]
    u = lo[0, 8:11].detach() * 2 - 1
    d = u / torch.linalg.norm(u)
    inv_s = torch.exp(10 * var)
    tc = pg @ d
    ic = -(torch.relu(-tc * 0.5 + 0.5) * (1 - cos_anneal) + torch.relu(-tc) * cos_anneal)
    nxt = sdf + ic * dt * 0.5
    prv = sdf - ic * dt * 0.5
    ncdf, pcdf = torch.sigmoid(nxt * inv_s), torch.sigmoid(prv * inv_s)
    alpha = torch.clamp((pcdf - ncdf + 1e-5) / (pcdf + 1e-5), 0.0, 1.0)
    T = torch.cumprod(torch.cat([torch.ones(1, dtype=lo.dtype), 1 - alpha[:-1]]), 0)
    w = alpha * T
    rgb = (w[:, None] * torch.sigmoid(raw)).sum(0)
    return lo, rgb, T[-1] * (1 - alpha[-1]), alpha.detach()


def huber_sum(rgb, target):
    diff = rgb - target
    ad = diff.abs()
    return torch.where(ad > 0.1, ad - 0.05, 5.0 * diff * diff).sum() / 5.0
