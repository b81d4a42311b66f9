"""Why the pre-compaction inference costs more per sample at later training states (development tool).

At the bench's shape (Config S, base.json L=14, R = Nc = 2^18) the one-pass replay of k_nerf_infer over the kept samples
took 0.826 ms at step 800 and 1.088 ms at step 1020 for the same 4.19 M samples (profiles/r05_infer_state_ab.txt). This
trains one testbed through the states in STATES and at each one records, for the kept samples in the step's own layout
(the march's pre-compaction order: a ray's samples consecutive, rays in slot order):
  * the one-pass replay's duration (neus_testbed_time_kernel id 3) and the kept-sample count;
  * the rays per 32-sample wave group and the samples per ray with samples;
  * per level, the distinct 128-B lines one gather instruction touches: k_nerf_infer holds a sample on two lanes (lane half
    h gathers the levels 2m + h), so one instruction of a wave gathers corner c of level 2m for its 32 samples on half 0
    and of level 2m + 1 on half 1 - the lines it touches are what the texture path serves for it;
  * the same for the first progressive round's list (the spatially sorted order the step runs at those states).
Output: one JSON line per state (and gpurun_out/diag_infer_state.json)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402

import oracle as O  # noqa: E402  (the level tables only: offsets, resolutions, scales)
from neus2_amd import pyngp, scenes  # noqa: E402
from neus2_amd._lib import check, lib  # noqa: E402

LINE = 128
GROUPS = int(os.environ.get("GROUPS", "4096"))


def morton8(c):
    k = np.zeros(len(c), np.int64)
    for b in range(3):
        for d in range(3):
            k |= ((c[:, d] >> b) & 1).astype(np.int64) << (3 * b + d)
    return k


def line_ids(pos, l, off, res, scale, grid_byte0):
    """[n, 8] 128-B line of corner c of level l for each position (tcnn GridEncoding geometry, common.h grid_index)."""
    hsize = int(off[l + 1] - off[l])
    r = int(res[l])
    g = np.floor(pos * np.float32(scale[l]) + np.float32(0.5)).astype(np.int64)
    dense = r ** 3 <= hsize
    out = np.empty((len(pos), 8), np.int64)
    for c in range(8):
        x, y, z = g[:, 0] + (c & 1), g[:, 1] + ((c >> 1) & 1), g[:, 2] + ((c >> 2) & 1)
        if dense:
            ix = (x + y * r + z * r * r) % hsize
        else:
            ix = ((x.astype(np.uint32) ^ (y.astype(np.uint32) * np.uint32(2654435761)) ^ (z.astype(np.uint32) * np.uint32(805459861)))
                  % np.uint32(hsize)).astype(np.int64)
        out[:, c] = (grid_byte0 + 4 * (int(off[l]) + ix)) // LINE
    return out


def group_stats(pos, ray, n_levels, off, res, scale, grid_byte0, rng):
    """Distinct lines per gather instruction (per level pair, averaged over corners and a sample of 32-sample groups) and
    distinct rays per group."""
    n = len(pos) // 32 * 32
    gsel = np.sort(rng.choice(n // 32, size=min(GROUPS, n // 32), replace=False))
    idx = (gsel[:, None] * 32 + np.arange(32)[None, :]).ravel()
    p = pos[idx]
    rays_per_group = float(np.mean([len(np.unique(ray[idx[k * 32:(k + 1) * 32]])) for k in range(len(gsel))]))
    per_level = []
    lines = [line_ids(p, l, off, res, scale, grid_byte0).reshape(len(gsel), 32, 8) for l in range(n_levels)]
    for l in range(n_levels):
        a = np.sort(lines[l].transpose(0, 2, 1), axis=2)  # [group, corner, 32]
        per_level.append(float(((np.diff(a, axis=2) != 0).sum(axis=2) + 1).mean()))
    pairs = []
    for m in range((n_levels + 1) // 2):
        h0 = lines[2 * m].transpose(0, 2, 1)
        h1 = lines[2 * m + 1].transpose(0, 2, 1) if 2 * m + 1 < n_levels else h0
        a = np.sort(np.concatenate([h0, h1], axis=2), axis=2)  # [group, corner, 64 lanes]
        pairs.append(float(((np.diff(a, axis=2) != 0).sum(axis=2) + 1).mean()))
    return {"rays_per_32_samples": round(rays_per_group, 2), "lines_per_gather_by_level": [round(v, 2) for v in per_level],
            "lines_per_gather_instruction_by_pair": [round(v, 2) for v in pairs], "lines_per_gather_instruction": round(float(np.mean(pairs)), 2)}


def kept_views(step_n_rays_total, extent, n_img, xforms, R=1 << 18):
    """The training views of the kept ray prefix: image_idx (march_common.h, the reference's uint32 arithmetic,
    testbed_nerf.cu:1291) of the slots [0, extent), with each view's forward direction (-z column of its camera-to-world)."""
    i = np.arange(extent, dtype=np.uint64)
    v = ((((i + np.uint64(step_n_rays_total)) * np.uint64(n_img)) & np.uint64(0xFFFFFFFF)) // np.uint64(R) % np.uint64(n_img)).astype(int)
    ims, cnt = np.unique(v, return_counts=True)
    X = np.asarray(xforms, np.float64).reshape(n_img, 3, 4)
    return [{"view": int(k), "rays": int(c), "forward": (-X[k][:, 2]).round(3).tolist()} for k, c in zip(ims, cnt)]


def state(tb, cfg, off, res, scale, grid_byte0, rng, sc=None):
    R = 1 << 18
    st = tb.stats()
    nreq, cc, _ = tb.ray_counts(R)
    base = np.zeros(R, np.uint32)
    check(lib().neus_debug_get_buffer(tb.handle, 11, C.c_uint64(0), C.c_uint64(base.nbytes), base.ctypes.data_as(C.c_void_p)))
    extent = int(st["kept_ray_extent"])
    cnt = np.where(np.arange(R) < extent, nreq, 0).astype(np.int64)
    base = base.astype(np.int64)
    n_kept = int(cnt.sum())
    co = np.zeros(n_kept * 7, np.float32)
    check(lib().neus_debug_get_buffer(tb.handle, 10, C.c_uint64(0), C.c_uint64(co.nbytes), co.ctypes.data_as(C.c_void_p)))
    co = co.reshape(-1, 7)
    ray = np.repeat(np.arange(R), cnt)
    ms = C.c_float()
    check(lib().neus_debug_time_kernel(tb.handle, 3, 0, 5, C.byref(ms)))
    m = cnt > 0
    out = {"step": st["training_step"], "one_pass_replay_ms": round(ms.value, 4), "kept": n_kept, "rays_with_samples": int(m.sum()),
           "samples_per_ray": {"mean": round(float(cnt[m].mean()), 2), "median": float(np.median(cnt[m])),
                               "p90": float(np.percentile(cnt[m], 90))},
           "composited_per_ray_mean": round(float(cc[m].mean()), 2), "progressive_chunk_end": st["progressive_chunk_end"],
           "aabb_of_kept": [co[:, :3].min(0).round(4).tolist(), co[:, :3].max(0).round(4).tolist()]}
    # consecutive samples of one ray: a constant step (sqrt(3) / 1024 at cone angle 0) inside a run of occupied cells,
    # a jump across skipped empty cells between runs
    same = ray[1:] == ray[:-1]
    d = np.linalg.norm(co[1:, :3] - co[:-1, :3], axis=1)[same]
    dt = np.sqrt(3.0) / 1024
    step = d < 1.5 * dt
    out["consecutive"] = {"frac_constant_step": round(float(step.mean()), 4), "runs_per_ray": round(float((~step).sum() + m.sum()) / max(1, m.sum()), 2),
                          "mean_run_samples": round(n_kept / float((~step).sum() + m.sum()), 2),
                          "median_jump": round(float(np.median(d[~step])) if (~step).any() else 0.0, 5),
                          "step_over_dt_percentiles_1_10_50_90": [round(float(v), 4) for v in np.percentile(d[step] / dt, [1, 10, 50, 90])],
                          "frac_step_below_half_dt": round(float((d[step] < 0.5 * dt).mean()), 4),
                          "frac_zero_step": round(float((d == 0).mean()), 4),
                          # the grid axis the rays step along (mean |delta| per axis of a constant step, warped coordinates):
                          # the hash's x prime is 1, so steps along x stay inside a 128-B line of a hashed table
                          "mean_abs_step_xyz_over_dt": (np.abs(co[1:, :3] - co[:-1, :3])[same][step].mean(0) / dt).round(3).tolist()}
    if sc is not None:  # the last step's views (its n_rays_total: the counter before that step's update)
        out["kept_views"] = kept_views(int(st["n_rays_total"]) - R, extent, len(sc["xforms"]), sc["xforms"])
    out["march_order"] = group_stats(co[:, :3], ray, cfg.n_levels, off, res, scale, grid_byte0, rng)
    # round 0 of the progressive rounds: the first e samples of every kept ray, rays by the Morton key of the 8^3 cell of
    # their first sample (k_ray_hist / k_ray_sort_place)
    e = int(st["progressive_chunk_end"]) or 64
    rays = np.nonzero(m)[0]
    key = morton8(np.clip((co[base[rays], :3] * 8).astype(np.int64), 0, 7))
    order = rays[np.argsort(key, kind="stable")]
    take = np.minimum(cnt[order], e)
    idx = np.concatenate([np.arange(b, b + t) for b, t in zip(base[order], take)])
    out["round0_sorted"] = group_stats(co[idx, :3], np.repeat(order, take), cfg.n_levels, off, res, scale, grid_byte0, rng)
    out["round0_sorted"]["samples"] = int(len(idx))
    return out


def main():
    states = [int(x) for x in os.environ.get("STATES", "800,1020").split(",")]
    torch.cuda.set_device(0)
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
    cfg = O.make_cfg(per_level_scale=tb._net_cfg.per_level_scale)
    off, res, scale, _ = O.grid_tables(cfg)
    grid_byte0 = 2 * O.layout(cfg)["grid_off"]
    rng = np.random.default_rng(0)
    res_all = []
    done = 0
    for s in states:
        tb.train_steps(s - done)
        tb.synchronize()
        done = s
        r = state(tb, cfg, off, res, scale, grid_byte0, rng, sc)
        res_all.append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "diag_infer_state.json"), "w") as f:
        json.dump(res_all, f, indent=1)


if __name__ == "__main__":
    main()
