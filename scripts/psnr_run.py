"""Quality half of BASELINE.json's metric: PSNR after N training steps (default 20k) on the DTU-scan24-shaped
synthetic scene (Config S), with the wall-clock time of the training run.

Protocol of the reference's evaluation (scripts/render_utils.py:252-359): test view 0, spp 8, black
background, snap_to_pixel_centers, rendering_min_transmittance 1e-4, EMA (inference) weights,
PSNR = mse2psnr(mean((clip(srgb(pred)) - clip(srgb(gt)))^2)). Training is the reference's: adaptive rays
per batch, 2^18 compacted samples per step, base.json.

Usage: python scripts/psnr_run.py [--steps 20000] [--checkpoints 1000,5000,20000] [--width 1600 --height 1200]
Prints one JSON line per checkpoint and a final summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--checkpoints", type=str, default="")
    ap.add_argument("--width", type=int, default=1600)
    ap.add_argument("--height", type=int, default=1200)
    ap.add_argument("--views", type=int, default=49)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--config", type=str, default=os.path.join(ROOT, "configs", "nerf", "base.json"))
    args = ap.parse_args()

    import numpy as np
    from neus2_amd import pyngp, scenes

    sc = scenes.sphere_scene(n_views=args.views, width=args.width, height=args.height)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(args.config)
    cps = sorted({int(c) for c in args.checkpoints.split(",") if c} | {args.steps})
    tb.background_color = [0.0, 0.0, 0.0, 0.0]
    tb.snap_to_pixel_centers = True
    tb.nerf.rendering_min_transmittance = 1e-4
    gt = sc["images"][0]
    train_s = 0.0
    done = 0
    res = []
    for cp in cps:
        t0 = time.perf_counter()
        while done < cp:
            k = min(500, cp - done)
            tb.train_steps(k)
            done += k
            if done % 2000 == 0 or done == cp:
                tb.synchronize()
                print(json.dumps({"step": done, "train_s": round(train_s + time.perf_counter() - t0, 3), "loss": tb.loss}), flush=True)
        tb.synchronize()
        train_s += time.perf_counter() - t0
        t1 = time.perf_counter()
        tb.set_camera_to_training_view(0)
        img = tb.render(gt.shape[1], gt.shape[0], spp=args.spp)
        render_s = time.perf_counter() - t1
        psnr, mse = pyngp.eval_psnr(img, gt)
        st = tb.stats()
        r = {"step": cp, "psnr": round(float(psnr), 3), "mse": mse, "train_wall_s": round(train_s, 3), "render_s": round(render_s, 3),
             "render_iterations": tb.last_render_iterations, "loss": st["loss"], "rays_per_batch": st["rays_per_batch"],
             "measured_batch_size": st["measured_batch_size"]}
        res.append(r)
        print(json.dumps(r), flush=True)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.save(os.path.join(ROOT, "gpurun_out", f"psnr_view0_{cp}.npy"), (np.clip(pyngp.linear_to_srgb(img[..., :3]), 0, 1) * 255).astype(np.uint8))
    print(json.dumps({"metric": "PSNR (test view 0, spp 8, black bg)", "scene": f"Config S {args.views}x{args.width}x{args.height}",
                      "steps": args.steps, "psnr": res[-1]["psnr"], "train_wall_s": res[-1]["train_wall_s"], "checkpoints": res}))


if __name__ == "__main__":
    main()
