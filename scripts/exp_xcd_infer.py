"""Experiment: does an XCD-aware, spatially partitioned work order raise k_nerf_infer's L2 hit rate and speed?

Samples are laid out like the training step's inference lists (runs of consecutive samples along rays, around a
sphere-shell surface, rays in random order). Orders:
  random  - rays in random order (what the step's lists look like)
  morton  - rays sorted by the Morton code of their surface point (8 equal contiguous parts = 8 compact regions)
Run once with NEUS_INFER_XCD_PARTS=1 (part x of the list on XCD x) and once without; prints ms per launch.
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def morton3(q):
    def spread(v):
        v = v.astype(np.uint64) & 0x3FF
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        v = (v | (v << 2)) & 0x09249249
        return v
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def main():
    import torch as t
    from neus2_amd import config, pyngp, scenes
    from neus2_amd._lib import check, lib
    run, n_rays = 64, 1 << 15
    n = run * n_rays
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    cfg = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_json(cfg, batch_size=1 << 18)
    lay = tb.layout()
    rng = np.random.default_rng(0)
    p = tb.get_params().copy()
    p[lay["grid_offset"]:lay["variance_offset"]] = rng.uniform(-0.1, 0.1, lay["variance_offset"] - lay["grid_offset"])
    tb.set_params(p)
    u = rng.normal(size=(n_rays, 3)); u /= np.linalg.norm(u, axis=1, keepdims=True)
    hit = 0.5 + 0.25 * u
    d = rng.normal(size=(n_rays, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = np.where((d * u).sum(1, keepdims=True) > 0, -d, d)  # into the sphere
    dt = 1.7e-3
    offs = (np.arange(run) - run // 2) * dt
    orders = {"random": rng.permutation(n_rays),
              "morton": np.argsort(morton3(np.clip(hit * 1024, 0, 1023).astype(np.int64)), kind="stable")}
    only = os.environ.get("EXP_ORDERS")
    if only:
        orders = {k: v for k, v in orders.items() if k in only.split(",")}
    out = t.zeros((n, 16), dtype=t.int16, device="cuda")
    xcd = os.environ.get("NEUS_INFER_XCD_PARTS", "0")
    for name, order in orders.items():
        h, dd = hit[order], d[order]
        pos = (h[:, None, :] + offs[None, :, None] * dd[:, None, :]).reshape(n, 3)
        c = np.zeros((n, 7), np.float32)
        c[:, :3] = np.clip(pos, 0.0, 1.0)
        c[:, 3] = dt
        c[:, 4:] = np.repeat((dd + 1) * 0.5, run, axis=0)
        ct = t.from_numpy(c).cuda()
        f = lambda: check(lib().neus_net_forward(tb.handle, None, C.c_uint32(n), C.c_void_p(ct.data_ptr()), C.c_uint32(14),
                                                 C.c_void_p(out.data_ptr())))
        for _ in range(5):
            f()
        t.cuda.synchronize()
        reps = 40
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        t.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"xcd_parts={xcd} order={name} n={n} ms_per_launch={ms:.4f} ns_per_sample={ms * 1e6 / n:.2f}", flush=True)


if __name__ == "__main__":
    main()
