"""Row Q's anchor (SURVEY.md §8(d) "reference PSNR"): the same reduced Config S training run on the CPU oracle
(oracle/cpu_step.py, the reference's algorithm restated; test infrastructure) and on the MI355X build, both evaluated
with the protocol of render_utils.py:252-359 (test view 0, spp 8, black background, snap_to_pixel_centers, min
transmittance 1e-4, EMA weights; PSNR of clip(srgb(pred)) vs clip(srgb(gt)), scripts/common.py:46).

Reduced Config S: 8 views of the Config S sphere at 200x150 (DTU-scan24 intrinsics scaled by 1/8), base.json (L=14),
the reference's adaptive rays per batch with a compacted batch of --batch samples (default 4096; the reference's 2^18
is out of reach for the CPU), --steps steps, geometric init. Same seed, same data, same schedule on both sides.
--fixed-rays R freezes the rays per batch at R on both sides (round 5): the adaptation follows the compacted counts, which
fp16 network noise moves, so with it on the two runs drift onto different ray sets; frozen, they see identical rays at
every step and differ only by the network arithmetic.

Usage:
  python scripts/psnr_anchor.py --side cpu [--steps 2000] [--checkpoints 250,500,1000] > profiles/rNN_psnr_anchor_cpu.jsonl
  python scripts/psnr_anchor.py --side gpu [...]   (on the GPU box)
Prints one JSON line per checkpoint.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def scene(args):
    from neus2_amd import scenes
    s = args.width / 1600.0
    return scenes.sphere_scene(n_views=args.views, width=args.width, height=args.height, focal=(2892.0 * s, 2892.0 * s),
                               principal=(823.2 / 1600, 619.1 / 1200))


def psnr_of(img, gt):
    from neus2_amd import pyngp
    psnr, mse = pyngp.eval_psnr(img, gt)
    return round(float(psnr), 3), mse


def run_cpu(args, sc, cps):
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from cpu_step import CpuTrainer
    from neus2_amd.pyngp import geometric_init_weights
    cfg = O.make_cfg()
    if args.sum_order != "index":
        O.set_sum_order(args.sum_order)
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    p = O.init_params(cfg, geo=False)
    geo = geometric_init_weights(14, 64)
    p[: geo.size] = geo
    tr = CpuTrainer(cfg, ds, p, batch=args.batch, rays_per_batch=args.fixed_rays or args.batch, fixed_rays=bool(args.fixed_rays))
    gt = sc["images"][0]
    t0 = time.perf_counter()
    done = 0
    for cp in cps:
        while done < cp:
            tr.step()
            done += 1
            if done % 50 == 0:
                print(json.dumps({"side": "cpu", "step": done, "s": round(time.perf_counter() - t0, 1), "R": tr.R,
                                  "compacted": tr.last["compacted"]}), file=sys.stderr, flush=True)
        # the EMA (inference) weights as the kernels read them: fp16 copies (Ema::custom_weights)
        ema = tr.ema_tmp.astype(np.float16).astype(np.float32)
        img, _ = O.render(cfg, ema, tr.valid_level(tr.training_step), ds, tr.bitfield, sc["xforms"][0], sc["focal"][0],
                          sc["principal"][0], gt.shape[1], gt.shape[0], spp=args.spp, snap=True, min_transmittance=1e-4, cos_anneal=1.0)
        psnr, mse = psnr_of(img, gt)
        print(json.dumps({"side": "cpu", "sum_order": args.sum_order, "step": cp, "psnr": psnr, "mse": mse, "wall_s": round(time.perf_counter() - t0, 1),
                          "rays_per_batch": int(tr.R), "compacted": int(tr.last["compacted"]), "threads": O.num_threads()}), flush=True)


def run_gpu(args, sc, cps):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    kw = dict(fixed_rays_per_batch=args.fixed_rays) if args.fixed_rays else {}
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=args.batch, **kw)
    if args.perturb:
        # ensemble member: the lowest mantissa bit of a random 1 % of the initial fp32 parameters flipped (a change far
        # below the fp16 rounding the network computes with), to measure how far fp16-level noise alone moves the PSNR
        import numpy as np
        p = tb.get_params().copy()
        rng = np.random.default_rng(args.perturb)
        idx = rng.choice(p.size, p.size // 100, replace=False)
        p.view(np.uint32)[idx] ^= np.uint32(1)
        tb.set_params(p)
    tb.background_color = [0.0, 0.0, 0.0, 0.0]
    tb.snap_to_pixel_centers = True
    tb.nerf.rendering_min_transmittance = 1e-4
    gt = sc["images"][0]
    done = 0
    t0 = time.perf_counter()
    for cp in cps:
        tb.train_steps(cp - done)
        done = cp
        tb.synchronize()
        tb.set_camera_to_training_view(0)
        img = tb.render(gt.shape[1], gt.shape[0], spp=args.spp)
        psnr, mse = psnr_of(img, gt)
        st = tb.stats()
        print(json.dumps({"side": "gpu", "perturb": args.perturb, "step": cp, "psnr": psnr, "mse": mse, "wall_s": round(time.perf_counter() - t0, 2),
                          "rays_per_batch": st["rays_per_batch"], "compacted": st["measured_batch_size"]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", choices=("cpu", "gpu"), required=True)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--checkpoints", type=str, default="250,500,1000")
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--width", type=int, default=200)
    ap.add_argument("--height", type=int, default=150)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--fixed-rays", type=int, default=0, help="rays per batch frozen at this many on both sides (0: adaptive)")
    ap.add_argument("--sum-order", default="index", help="cpu: the oracle's fp32 summation order (oracle.SUM_ORDERS)")
    ap.add_argument("--perturb", type=int, default=0, help="gpu: seed of a 1-ulp flip of 1 %% of the initial parameters (0: none)")
    ap.add_argument("--ensemble", type=int, default=0, help="gpu: also run perturb seeds 1..N")
    args = ap.parse_args()
    cps = sorted({int(c) for c in args.checkpoints.split(",") if c and int(c) < args.steps} | {args.steps})
    sc = scene(args)
    if args.side == "cpu":
        run_cpu(args, sc, cps)
        return
    run_gpu(args, sc, cps)
    for k in range(1, args.ensemble + 1):
        args.perturb = k
        run_gpu(args, sc, cps)


if __name__ == "__main__":
    main()
