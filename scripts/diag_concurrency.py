"""Diagnostic: two testbeds trained at the same time from two host threads on one GPU against one trained alone
(tests/test_gpu_determinism.py found them different at the bench shape). Per step: checksums of the parameters,
gradients and density grid of every testbed; prints the first step at which a concurrent testbed leaves the reference
and which block differs first. Options select the subsystems (env switches are read by the library at creation).
Usage: python scripts/diag_concurrency.py [--steps 816] [--batch 262144] [--progressive -1|0|1|2] [--scene s|small]"""
import argparse
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=816)
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--progressive", type=int, default=-1, help="-1: library default (auto)")
    ap.add_argument("--scene", default="s")
    ap.add_argument("--sync-every", type=int, default=1)
    args = ap.parse_args()
    from neus2_amd import pyngp, scenes
    if args.scene == "s":
        sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    else:
        sc = scenes.small_scene(n_views=8, width=64, height=48)

    def make():
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=args.batch, fixed_rays_per_batch=args.batch)
        if args.progressive >= 0:
            tb.set_progressive_inference(args.progressive)
        return tb

    lay = None

    def sums(tb):
        nonlocal lay
        if lay is None:
            lay = tb.layout()
        p, g = tb.get_params().view(np.uint32), tb.get_gradients().view(np.uint32)
        grid = tb.get_density_grid()[0].view(np.uint32)
        bl = {"density": (0, lay["n_density"]), "rgb": (lay["n_density"], lay["n_matrix"]), "grid": (lay["grid_offset"], lay["variance_offset"]),
              "var": (lay["variance_offset"], lay["n_params"])}
        out = {}
        for k, (a, b) in bl.items():
            out["p_" + k] = int(p[a:b].astype(np.uint64).sum())
            out["g_" + k] = int(g[a:b].astype(np.uint64).sum())
        out["occ"] = int(grid.astype(np.uint64).sum())
        st = tb.stats()
        out["n_kept"] = st["measured_batch_size_before_compaction"]
        out["nc"] = st["measured_batch_size"]
        out["prog"] = st["progressive_steps"]
        return out

    def run(tb, rec):
        done = 0
        while done < args.steps:
            k = min(args.sync_every, args.steps - done)
            tb.train_steps(k)
            done += k
            rec.append((done, sums(tb)))

    ref = make()
    rr = []
    run(ref, rr)
    del ref
    pair = [make(), make()]
    recs = [[], []]
    ts = [threading.Thread(target=run, args=(pair[i], recs[i])) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    res = {"args": vars(args), "env": {k: v for k, v in os.environ.items() if k.startswith("NEUS_")}}
    for i in range(2):
        first = None
        for (s0, a), (s1, b) in zip(rr, recs[i]):
            assert s0 == s1
            diff = [k for k in a if a[k] != b[k]]
            if diff:
                first = {"step": s0, "differs": diff, "ref": {k: a[k] for k in diff}, "got": {k: b[k] for k in diff}}
                break
        res[f"testbed{i}"] = first or "identical"
    res["final_prog_steps"] = rr[-1][1]["prog"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
