"""Generates the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no golden vectors for this path; the oracle is pinned by the
PCG32 KAT, the survey's pcg32.h probe values and the survey's parameter count (tests/test_oracle.py),
and cross-checked against float64 autograd. These fixtures freeze the oracle's outputs on small
seeded inputs so that (a) CPU tests detect any drift of the oracle and (b) the GPU tests compare
the HIP path with the same bytes. Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402

SAMPLE_RAYS = 512
SAMPLE_RNG = (0x853C49E6748FEA9B, 0xDA3E39CB94B95BDB)  # pcg32 default state/inc
MAX_SAMPLES = 1 << 14
MAX_COMPACTED = 2048


def small_dataset():
    from neus2_amd import scenes
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    return sc, O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])


def small_cfg():
    return O.make_cfg(n_levels=4, log2_hashmap_size=12, base_resolution=8, per_level_scale=2.0)


def small_params(seed=3):
    cfg = small_cfg()
    lay = O.layout(cfg)
    rng = np.random.default_rng(seed)
    p = O.init_params(cfg)
    din = cfg.density_in
    w0 = p[: 64 * din].reshape(64, din)
    w0[:, 3:11] = rng.normal(0, 0.3, (64, 8))
    p[lay["grid_off"]:lay["var_off"]] = rng.uniform(-0.1, 0.1, lay["n_grid_params"])
    return cfg, p


def sampling_case():
    from neus2_amd import scenes
    sc, ds = small_dataset()
    bf = scenes.shell_bitfield(thickness=4.0 / 128)
    rays, ns, co, counter, nr = O.generate_samples(ds, bf, SAMPLE_RAYS, 0, SAMPLE_RNG[0], SAMPLE_RNG[1], MAX_SAMPLES)
    nk = int(ns[:, 0].sum())
    return dict(rays=rays, numsteps=ns, coords=co[:nk], counter=np.uint32(counter), n_rays_with_samples=np.uint32(nr))


def loss_case():
    from neus2_amd import scenes
    sc, ds = small_dataset()
    bf = scenes.shell_bitfield(thickness=4.0 / 128)
    rays, ns, co, counter, nr = O.generate_samples(ds, bf, SAMPLE_RAYS, 0, SAMPLE_RNG[0], SAMPLE_RNG[1], MAX_SAMPLES)
    nk = int(ns[:, 0].sum())
    cfg, p = small_params()
    out = np.zeros((max(nk, 1), 16), np.uint16)
    out[:nk] = O.network_forward(cfg, p, co[:nk], cfg.n_levels)
    res = O.compute_loss(ds, SAMPLE_RAYS, 0, SAMPLE_RNG[0], SAMPLE_RNG[1], MAX_COMPACTED, rays, ns, co, out)
    m = min(res["counter"], MAX_COMPACTED)
    return dict(net_out=out[:nk], numsteps=res["numsteps"], coords=res["coords"][:m], dL_dout=res["dL_dout"][:m],
                loss=res["loss"], counter=np.uint32(res["counter"]))


def network_case():
    cfg, p = small_params()
    rng = np.random.default_rng(9)
    n = 256
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.uniform(0.05, 0.95, (n, 3))
    c[:, 3] = 0.01
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c[:, 4:] = (d + 1) * 0.5
    out = O.network_forward(cfg, p, c, cfg.n_levels)
    dl = np.zeros((n, 16), np.float32)
    dl[:, 0:4] = rng.normal(0, 1e-2, (n, 4))
    dl[:, 4:7] = rng.normal(0, 1, (n, 3))
    dl[:, 7:11] = rng.normal(0, 1e-2, (n, 4))
    dl16 = dl.astype(np.float16).view(np.uint16)
    grads = O.network_backward(cfg, p, c, cfg.n_levels, dl16, n)
    return dict(coords=c, dL_dout=dl16, out=out, grads=grads)


def main():
    np.savez_compressed(os.path.join(HERE, "sampling_small.npz"), **sampling_case())
    np.savez_compressed(os.path.join(HERE, "loss_small.npz"), **loss_case())
    np.savez_compressed(os.path.join(HERE, "network_small.npz"), **network_case())
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
