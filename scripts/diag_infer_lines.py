"""Compulsory memory traffic of the inference's hash-grid gathers (development tool): at the bench state
(Config S, base.json L=14, R = Nc = 2^18, trained --warm steps), the first progressive round's samples (the first e
samples of every kept ray, e from the step's own rule), ordered and split as the step does (Morton order of the 8^3 cell
of each ray's first sample, the list cut into 8 contiguous eighths, eighth x on XCD x). Per level it counts the distinct
128-B lines the gathers touch: per sample with no reuse at all, per XCD (an infinite L2 per XCD: the compulsory misses of
the step's partition) and over the whole device. The measured memory-side traffic of the launch (PMC, traffic.json) is
set against these bounds.

Level geometry as tcnn's GridEncoding (grid.h: scale = 2^(l log2 s) base - 1, pos = x scale + 0.5, res = ceil(scale) + 1,
the index of common.h grid_index), the level offsets and scales from the CPU oracle's tables (oracle/, test
infrastructure, used here only as a reference for the layout)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ctypes as C  # noqa: E402

import torch  # noqa: E402

import oracle as O  # noqa: E402
from neus2_amd import pyngp, scenes  # noqa: E402
from neus2_amd._lib import check, lib  # noqa: E402

LINE = 128


def morton8(c):
    k = np.zeros(len(c), np.int64)
    for b in range(3):
        for d in range(3):
            k |= ((c[:, d] >> b) & 1).astype(np.int64) << (3 * b + d)
    return k


def main():
    warm = int(os.environ.get("WARM", "800"))
    torch.cuda.set_device(0)
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
    tb.train_steps(warm)
    tb.synchronize()
    R = 1 << 18
    nreq, cc, _ = tb.ray_counts(R)
    base = np.zeros(R, np.uint32)  # the march's exclusive scan of the requested counts (the pre-compaction layout)
    check(lib().neus_debug_get_buffer(tb.handle, 11, C.c_uint64(0), C.c_uint64(base.nbytes), base.ctypes.data_as(C.c_void_p)))
    extent = int(tb.stats()["kept_ray_extent"])
    cnt = np.where(np.arange(R) < extent, nreq, 0).astype(np.int64)
    base = base.astype(np.int64)
    n_kept = int(cnt.sum())
    co = np.zeros(n_kept * 7, np.float32)
    check(lib().neus_debug_get_buffer(tb.handle, 10, C.c_uint64(0), C.c_uint64(co.nbytes), co.ctypes.data_as(C.c_void_p)))
    co = co.reshape(-1, 7)
    m = cnt > 0
    mc = float(cc[m].mean())
    e = int(min(128, max(24, round((0.5 * mc + 12) / 8) * 8)))
    # round 0: the first min(n, e) samples of every kept ray, rays in Morton order of their first sample's 8^3 cell
    rays = np.nonzero(m)[0]
    first = co[base[rays], :3]
    key = morton8(np.clip((first * 8).astype(np.int64), 0, 7))
    order = rays[np.argsort(key, kind="stable")]
    take = np.minimum(cnt[order], e)
    idx = np.concatenate([np.arange(b, b + t) for b, t in zip(base[order], take)])
    pos = co[idx, :3].astype(np.float32)
    n = len(pos)
    xcd = (np.arange(n) * 8) // n
    cfg = O.make_cfg()
    off, res, scale, _ = O.grid_tables(cfg)
    lay = O.layout(cfg)
    grid_byte0 = 2 * lay["grid_off"]
    out = {"warm": warm, "chunk_end": e, "samples": n, "kept": n_kept, "levels": []}
    tot = {"per_sample": 0, "per_xcd": 0, "device": 0}
    for l in range(cfg.n_levels):
        hsize = int(off[l + 1] - off[l])
        r = int(res[l])
        p = pos * np.float32(scale[l]) + np.float32(0.5)
        g = np.floor(p).astype(np.int64)
        dense = r ** 3 <= hsize
        lines_l = []
        for cidx in range(8):
            x, y, z = (g[:, 0] + (cidx & 1)), (g[:, 1] + ((cidx >> 1) & 1)), (g[:, 2] + ((cidx >> 2) & 1))
            if dense:
                ix = (x + y * r + z * r * r) % hsize
            else:
                ix = ((x.astype(np.uint32) ^ (y.astype(np.uint32) * np.uint32(2654435761)) ^ (z.astype(np.uint32) * np.uint32(805459861)))
                      % np.uint32(hsize)).astype(np.int64)
            lines_l.append((grid_byte0 + 4 * (int(off[l]) + ix)) // LINE)
        L8 = np.stack(lines_l, 1)
        per_sample = sum(len(np.unique(row)) for row in np.sort(L8, 1)[:: max(1, n // 20000)]) * max(1, n // 20000)
        per_xcd = sum(len(np.unique(L8[xcd == k])) for k in range(8))
        device = len(np.unique(L8))
        table_lines = (4 * hsize + LINE - 1) // LINE
        out["levels"].append({"level": l, "dense": bool(dense), "res": r, "table_kb": 4 * hsize // 1024, "lines_per_sample_no_reuse": per_sample / n,
                              "lines_per_xcd_infinite": per_xcd, "lines_device": device, "table_lines": table_lines})
        tot["per_sample"] += per_sample
        tot["per_xcd"] += per_xcd
        tot["device"] += device
        print(json.dumps(out["levels"][-1]), flush=True)
    io = n * (28 + 32)
    out["bytes"] = {"algorithmic_gathers": n * 8 * 4 * cfg.n_levels, "coords_and_outputs": io,
                    "no_reuse_lines": tot["per_sample"] * LINE + io, "per_xcd_compulsory": tot["per_xcd"] * LINE + io,
                    "device_compulsory": tot["device"] * LINE + io}
    print(json.dumps(out["bytes"]), flush=True)
    print(json.dumps({k: v for k, v in out.items() if k != "levels"}))


if __name__ == "__main__":
    main()
