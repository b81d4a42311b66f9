"""Row Q's anchor, segment by segment: the reference's algorithm (the CPU oracle's train step, oracle/cpu_step.py, test
infrastructure) and the MI355X build continue the SAME training state for one segment, and both are evaluated with the
protocol of render_utils.py:252-359 (as scripts/psnr_anchor.py). Free-running trajectories of an fp16 network drift
apart after a few hundred steps whatever the implementation (the GPU ensemble and the oracle's own summation orders in
profiles/r05_psnr_anchor_*), so a long single-trajectory comparison measures that drift; here each segment starts from
the device's state at its first step (parameters, Adam moments and per-parameter steps, the fp32 EMA, occupancy grid
and bitfield, both RNG streams, the step and ray counters), which the oracle takes over.

Reduced Config S as scripts/psnr_anchor.py (8 views of 200x150, base.json, geometric init, 4096-sample batch), rays per
batch frozen at --fixed-rays. Prints one JSON line per segment end (and progress lines on stderr).
Usage (GPU box): python scripts/psnr_anchor_segments.py [--starts 500,1000,1500] [--length 500]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--starts", default="500,1000,1500")
    ap.add_argument("--length", type=int, default=500)
    ap.add_argument("--fixed-rays", type=int, default=512)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--alt-order", default="reversed", help="also continue the oracle in this summation order ('' : no)")
    args = ap.parse_args()
    import oracle as O
    from cpu_step import CpuTrainer
    from neus2_amd import pyngp, scenes
    s = 200 / 1600.0
    sc = scenes.sphere_scene(n_views=8, width=200, height=150, focal=(2892.0 * s, 2892.0 * s), principal=(823.2 / 1600, 619.1 / 1200))
    gt = sc["images"][0]

    def make_tb():
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=args.batch,
                                    fixed_rays_per_batch=args.fixed_rays)
        tb.background_color = [0.0, 0.0, 0.0, 0.0]
        tb.snap_to_pixel_centers = True
        tb.nerf.rendering_min_transmittance = 1e-4
        return tb

    def gpu_psnr(tb):
        tb.synchronize()
        tb.set_camera_to_training_view(0)
        img = tb.render(gt.shape[1], gt.shape[0], spp=args.spp)
        return float(pyngp.eval_psnr(img, gt)[0])

    cfg = O.make_cfg()
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])

    def cpu_from(tb):
        st, opt = tb.stats(), tb.get_optimizer_state()
        tr = CpuTrainer(cfg, ds, tb.get_params(), batch=args.batch, rays_per_batch=args.fixed_rays, fixed_rays=True)
        tr.m1[:] = opt["m1"]; tr.m2[:] = opt["m2"]; tr.steps[:] = opt["param_steps"]
        tr.ema_tmp[:] = tb.get_ema_params()
        tr.adam_step = int(opt["current_step"])
        tr.training_step = int(st["training_step"])
        tr.n_rays_total = int(st["n_rays_total"])
        rng = tb.get_rng()
        tr.rng_state, tr.rng_inc, tr.dg_state, tr.dg_inc = rng[0], rng[1], rng[2], rng[3]
        grid, bf = tb.get_density_grid()
        tr.density_grid[:] = grid
        tr.bitfield[:] = bf
        tr.ema_step = int(st["occ_updates"])
        before = int(st["measured_batch_size_before_compaction"])
        tr.max_inference = (min(before, tr.max_samples) + 127) // 128 * 128 if before else tr.max_samples
        return tr

    def cpu_psnr(tr):
        ema = tr.ema_tmp.astype(np.float16).astype(np.float32)
        img, _ = O.render(cfg, ema, tr.valid_level(tr.training_step), ds, tr.bitfield, sc["xforms"][0], sc["focal"][0], sc["principal"][0],
                          gt.shape[1], gt.shape[0], spp=args.spp, snap=True, min_transmittance=1e-4, cos_anneal=1.0)
        return float(pyngp.eval_psnr(img, gt)[0])

    tb = make_tb()
    done = 0
    for start in sorted(int(v) for v in args.starts.split(",")):
        tb.train_steps(start - done)
        done = start
        tb.synchronize()
        p_start = gpu_psnr(tb)
        # the oracle's own spread over the segment: the same state continued with its layer products summed in reversed
        # order (the noise floor any fp32 accumulation order adds to an fp16 network)
        p_cpu_alt = None
        if args.alt_order:
            tr2 = cpu_from(tb)
            O.set_sum_order(args.alt_order)
            try:
                for _ in range(args.length):
                    tr2.step()
            finally:
                O.set_sum_order("index")
            p_cpu_alt = cpu_psnr(tr2)
            del tr2
        tr = cpu_from(tb)
        t0 = time.perf_counter()
        lock = []
        for k in range(args.length):
            tr.step()
            if k < 2:  # the first steps in lockstep: the same state must give the same compacted count (sanity)
                tb.train_steps(1)
                lock.append([int(tb.stats()["measured_batch_size"]), int(tr.last["compacted"])])
            if (k + 1) % 50 == 0:
                print(json.dumps({"segment": start, "cpu_step": tr.training_step, "s": round(time.perf_counter() - t0, 1)}), file=sys.stderr, flush=True)
        p_cpu = cpu_psnr(tr)
        # the device continues from the same state (its own trajectory: the next segment starts from it)
        tb.train_steps(args.length - min(2, args.length))
        done += args.length
        p_gpu = gpu_psnr(tb)
        print(json.dumps({"segment_start": start, "segment_end": start + args.length, "psnr_start": round(p_start, 3),
                          "psnr_cpu_oracle": round(p_cpu, 3), "psnr_gpu": round(p_gpu, 3), "delta_db": round(p_gpu - p_cpu, 3),
                          "psnr_cpu_alt_order": None if p_cpu_alt is None else round(p_cpu_alt, 3),
                          "delta_cpu_alt_db": None if p_cpu_alt is None else round(p_cpu_alt - p_cpu, 3),
                          "cpu_s": round(time.perf_counter() - t0, 1), "threads": O.num_threads(),
                          "rays_per_batch": args.fixed_rays, "batch": args.batch, "lockstep_compacted_gpu_cpu": lock}), flush=True)


if __name__ == "__main__":
    main()
