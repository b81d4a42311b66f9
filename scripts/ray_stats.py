"""Per-ray sample statistics of the bench workload (config 2, base.json, R = Nc = 2^18) at a few training steps:
requested samples ns and composited samples cn (the transmittance cut) of every kept ray, saved to an npz for
offline study of the progressive-inference schedule (evaluated samples of a chunk schedule E: per ray
min(ns, the first chunk end >= cn)). Run from the repo root on the GPU box:
    python scripts/ray_stats.py gpurun_out/ray_stats.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "ray_stats.npz")
    sys.argv = [sys.argv[0]]
    import bench
    from neus2_amd import scenes
    args = bench.parse()
    import torch
    torch.cuda.set_device(0)
    sc = scenes.sphere_scene(args.views, args.width, args.height, principal=(823.2 / 1600, 619.1 / 1200))
    tb = bench.make_testbed(sc, bench.Group(0, 1), 0, args)
    res = {}
    done = 0
    for step in (200, 820, 2000):
        tb.train_steps(step - done)
        done = step
        tb.synchronize()
        nreq, cn, comp = tb.ray_counts()
        kept = cn > 0
        res[f"ns_{step}"] = nreq[kept].astype(np.uint16)
        res[f"cn_{step}"] = cn[kept].astype(np.uint16)
        g, bf = tb.get_density_grid()
        res[f"bf0_{step}"] = np.asarray(bf)[: 128 ** 3 // 8].copy()  # mip-0 occupancy bits (Morton order)
        res[f"grid_{step}"] = np.asarray(g)[: 128 ** 3].astype(np.float16)
        print(step, "kept rays", int(kept.sum()), "samples", int(nreq[kept].sum()), "composited", int(cn[kept].sum()), flush=True)
    np.savez_compressed(out, **res)


if __name__ == "__main__":
    main()
