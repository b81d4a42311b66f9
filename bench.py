"""NeuS2 training throughput on MI355X (BASELINE.json metric: training samples/sec).

Workload (BASELINE.md §3 / SURVEY.md §8(d) "Config S"): DTU-scan24-shaped synthetic scene, 49 views of
1600x1200 RGBA8 (analytic sphere; DTU itself is not reachable here), configs/nerf/base.json
(14-level hash grid, width-64 MLPs), batch Nc = 2^18 compacted samples per GPU per step, R = 2^18
rays per GPU per step (adaptation frozen), occupancy-grid updates at the reference cadence.
A step = Testbed::train: occupancy update (when due) + sampling + pre-compaction forward + NeuS
loss/compaction + forward/backward (1st + 2nd order) + RCCL gradient all-reduce + Ema(Adam).

Usage: python bench.py --gpus N --steps K --warmup W  (N>1 via torch.distributed.run, one rank/GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# Memory-side bytes per launch, measured by rocprofv3 PMC passes at HEAD (scripts/gpu_traffic.sh ->
# profiles/traffic.json): reads = 128 B x TCC_EA0_RDREQ_128B + 64 B x the other read requests (FETCH_SIZE
# tallies 128-B requests at 64 B, the gfx950 half-count), writes = WRITE_SIZE; L2-to-fabric traffic, so
# Infinity Cache hits are included (an upper bound on DRAM bytes). Keyed by kernel and the number of
# active hash-grid levels of the replayed state; `traffic` is null when no measurement of that state exists.
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def measured_traffic(kernel, levels):
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    e = t.get(f"{kernel}@L{levels}")
    return None if e is None else e.get("bytes_per_launch")


def line_traffic(traffic, ms, algorithmic):
    if not traffic or not ms:
        return None
    gbs = traffic / (ms * 1e-3) / 1e9
    return {"GBs": round(gbs, 1), "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4),
            "traffic_over_algorithmic": round(traffic / algorithmic, 2) if algorithmic else None}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=800)  # past step ~660 every hash-grid level is active (valid_level schedule)
    p.add_argument("--views", type=int, default=49)
    p.add_argument("--width", type=int, default=1600)
    p.add_argument("--height", type=int, default=1200)
    p.add_argument("--batch", type=int, default=1 << 18)
    p.add_argument("--rays", type=int, default=1 << 18)
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-steps", type=int, default=8)
    # quality half of the metric: PSNR after this many steps of the reference's (adaptive-R) training, N=1 only
    p.add_argument("--psnr-steps", type=int, default=20000)
    # config 5: marching cubes at mc_res^3 over the PSNR leg's trained model (0 = skip)
    p.add_argument("--mc-res", type=int, default=1024)
    # BASELINE.json words config 2 as a 16-level grid (the reference's base.json has 14): the same step at L=16
    p.add_argument("--l16", type=int, default=1)
    return p.parse_args()


# Algorithmic work per unit, split over this build's kernels. F = 2, fp16
# grid: a hash-grid gather is 8 corners x L_active x 4 B per sample (448 B with all 14 levels active), the
# fused first+second order grid-gradient RMW 2 x that per compacted sample. L_active = valid_level + 1 of the
# replayed state (progressive levels, grid.h:2427-2440): levels beyond it are neither read nor written.
#   unit "ray"   : 40 B (ray record + indices + pixel)                       -> march (ray gen + march)
#   unit "pre"   : 596 B = 28 coords write (coord write pass) + 28 coords read + 448 gather + 32 output
#                  write (fused inference: 508 B) + 60 loss reads (loss kernels)
#   unit "train" : 1496 B = 60 compacted coords + dL/dout write (loss) + 28 coords + 448 gather (training
#                  encode: 476 B) + 32 output + 32 dL/dout (training MLP kernels: 32 B each) + 896 grid RMW (scatter)
# The SURVEY's figures count the gathers as HBM bytes; the 21 MB table mostly hits L2 / Infinity Cache,
# so `traffic` (PMC) is reported next to them. MFMA flops (SURVEY: 28,672 per pre-compaction sample,
# 92,160 per compacted sample) are reported alongside for the MLP kernels.
def kernel_table(levels):
    g = 8 * levels * 4
    return {
        # name: (kernel id of neus_testbed_time_kernel, algorithmic bytes per unit, flops per unit)
        "march": (0, 40, 0),
        "march_write": (1, 28, 0),
        "inference": (3, 28 + g + 32, 28672),
        "loss_alpha": (4, 60, 0),
        "train_encode": (8, 28 + g, 0),
        # the two training-MLP kernels (fwd recompute + 1st / 2nd-order backward; SURVEY: 92,160 - 28,672 flops per
        # compacted sample between them): dL/dout read by the colour kernel, the output-side operands by the density one
        "mlp_train_rgb": (9, 32, 0),
        "mlp_train_density": (10, 32, 0),
        "grid_scatter": (7, 2 * g, 0),
    }
MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 (MI355X_MICROARCH.md)


def kernel_rooflines(tb, levels, iters=9):
    """Per-kernel median launch duration (hipEvents on the testbed stream between `iters` back-to-back
    launches replayed on the final training state, neus_testbed_time_kernel) and the algorithmic HBM
    roofline of each launch with `levels` active hash-grid levels."""
    out = {}
    for name, (kid, bpu, fpu) in kernel_table(levels).items():
        ms, units = tb.time_kernel(kid, iters)
        b = bpu * units
        r = {"ms": round(ms, 4), "units": units, "bytes": b, "achieved": round(b / (ms * 1e-3) / 1e9, 1), "unit": "GB/s",
             "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if fpu:
            r["tflops"] = round(fpu * units / (ms * 1e-3) / 1e12, 1)
            r["mfma_frac"] = round(r["tflops"] / MFMA_PEAK_TFLOPS, 4)
        out[name] = r
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(local)
    from neus2_amd import pyngp, scenes
    sc = scenes.sphere_scene(args.views, args.width, args.height, principal=(823.2 / 1600, 619.1 / 1200))
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf, device=local)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=args.batch,
                                fixed_rays_per_batch=args.rays)
    if world > 1:
        import torch.distributed as dist
        obj = [pyngp.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        tb.init_data_parallel(rank, world, obj[0])

    def barrier():
        tb.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    t0 = time.time()
    tb.train_steps(args.warmup)
    barrier()
    warm_s = time.time() - t0
    # timed region
    tb.set_profiling(False)
    barrier()
    trained0 = tb.stats()["trained_samples_total"]
    t1 = time.perf_counter()
    tb.train_steps(args.steps)
    barrier()
    elapsed = time.perf_counter() - t1
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = tb.stats()
    batch = args.batch
    # every step trains on Nc = batch samples per GPU (the reference's m_training_batch_size; a short compaction
    # is rollover-padded, fill_rollover_and_rescale); the non-rollover share is reported next to it
    samples = batch * world * args.steps
    value = samples / elapsed
    real = (st["trained_samples_total"] - trained0) / max(1, batch * args.steps)
    levels = min(st["valid_level"] + 1, tb.layout()["n_levels"])
    # per-kernel timing after the timed region, on its final state (hipEvents on the testbed stream)
    kern = kernel_rooflines(tb, levels)
    dom = max(kern, key=lambda k: kern[k]["ms"])
    d = kern[dom]
    out = {
        "metric": "training samples/sec (compacted NeuS2 training samples, DTU-scan24-shaped synthetic, base.json)",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16 MFMA (fp32 accumulate) / fp32 optimizer",
        "data": "synthetic (analytic sphere, 49 x 1600x1200 RGBA8 views; DTU scan24 unavailable offline)",
        "config": {"workload": "NeuS2 train step, Config S, base.json L=14 T=2^19 W=64, Nc=2^18/GPU, R=2^18/GPU fixed",
                   "global_batch": batch * world, "rays_per_gpu": args.rays, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": d["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": d["frac"], "traffic": measured_traffic(dom, levels), "bytes_per_launch": d["bytes"],
                     "units_per_launch": d["units"], "launch_ms": d["ms"], "levels_active": levels},
        # memory-side line traffic (PMC, profiles/traffic.json) over the same launch: the hashed levels' 4-B corner
        # gathers each move a 128-B line from the Infinity Cache, so this, not the algorithmic rate, is what binds
        "line_traffic": line_traffic(measured_traffic(dom, levels), d["ms"], d["bytes"]),
        "non_rollover_fraction": round(real, 4),
        "kernels": kern,
        "loss": st["ray_loss"],
        "warmup_s": warm_s,
    }
    if world == 1 and args.l16:
        out["levels16"] = l16_leg(sc, args)
    if world == 1 and args.psnr_steps > 0:
        del tb
        out["psnr"], tb2 = psnr_leg(sc, args.psnr_steps)
        if args.mc_res > 0:
            out["marching_cubes"] = marching_cubes_leg(tb2, args.mc_res)
        del tb2
    if rank == 0 and args.cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(sc, args.cpu_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def l16_leg(sc, args):
    """The timed step of the main measurement with a 16-level hash grid (base.json otherwise): same data, batch,
    rays and warmup / steps, wall clock between synchronised points."""
    from neus2_amd import config, pyngp
    cfg = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    cfg["encoding"]["n_levels"] = 16
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_json(cfg, batch_size=args.batch, fixed_rays_per_batch=args.rays)
    tb.train_steps(args.warmup)
    tb.synchronize()
    t = time.perf_counter()
    tb.train_steps(args.steps)
    tb.synchronize()
    dt = time.perf_counter() - t
    st = tb.stats()
    levels = min(st["valid_level"] + 1, 16)
    inf_ms, inf_units = tb.time_kernel(3, 9)
    g = 8 * levels * 4
    del tb
    return {"value": args.batch * args.steps / dt, "unit": "samples/s", "ms_per_step": dt / args.steps * 1e3,
            "levels_active": levels,
            "inference": {"ms": round(inf_ms, 4), "units": inf_units,
                          "achieved_GBs": round((28 + g + 32) * inf_units / (inf_ms * 1e-3) / 1e9, 1)}}


def psnr_leg(sc, n_steps):
    """PSNR@n_steps (BASELINE.json metric, second half) with the reference's training (adaptive rays per
    batch, Nc = 2^18) and evaluation protocol (render_utils.py:252-359: view 0, spp 8, black background,
    pixel centres, min transmittance 1e-4, EMA weights); scripts/psnr_run.py is the standalone version."""
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"))
    t0 = time.perf_counter()
    done = 0
    while done < n_steps:
        k = min(2000, n_steps - done)
        tb.train_steps(k)
        done += k
        tb.synchronize()  # also a progress point for long runs
    train_s = time.perf_counter() - t0
    tb.background_color = [0.0, 0.0, 0.0, 0.0]
    tb.snap_to_pixel_centers = True
    tb.nerf.rendering_min_transmittance = 1e-4
    tb.set_camera_to_training_view(0)
    gt = sc["images"][0]
    t1 = time.perf_counter()
    img = tb.render(gt.shape[1], gt.shape[0], spp=8)
    render_s = time.perf_counter() - t1
    psnr, _ = pyngp.eval_psnr(img, gt)
    out = {"value": round(float(psnr), 3), "unit": "dB", "steps": n_steps, "train_wall_s": round(train_s, 2),
           "render_s": round(render_s, 3), "protocol": "view 0, spp 8, black bg, snap_to_pixel_centers, min_T 1e-4, EMA weights",
           "training": "reference schedule: adaptive rays/batch, Nc=2^18, base.json"}
    return out, tb


def marching_cubes_leg(tb, res=1024, reps=3):
    """BASELINE.json config 5: Testbed::marching_cubes at res^3 over the trained model (SDF of every grid point
    through the fused encode + density MLP, then the count / scan / emit mesh kernels). Voxels/s of the whole
    call (host sync at its end), best of `reps`; the mesh stays on the device."""
    import ctypes as C
    from neus2_amd._lib import check, lib
    r = (C.c_int32 * 3)(res, res, res)
    lo, hi = (C.c_float * 3)(0.0, 0.0, 0.0), (C.c_float * 3)(1.0, 1.0, 1.0)
    nv, nt = C.c_uint32(), C.c_uint32()
    best = None
    for _ in range(reps):
        tb.synchronize()
        t0 = time.perf_counter()
        check(lib().neus_testbed_marching_cubes(tb.handle, r, lo, hi, C.c_float(0.0), None, C.byref(nv), C.byref(nt)))
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    n = res ** 3
    # algorithmic bytes per voxel: 448 B gather + 4 B density write + 2 x 16 B MC passes
    return {"value": n / best, "unit": "voxels/s", "res": res, "ms": round(best * 1e3, 2), "n_verts": nv.value, "n_tris": nt.value,
            "achieved_GBs": round(n * (448 + 4 + 32) / best / 1e9, 1)}


def cpu_baseline(sc, n_steps):
    """The CPU oracle's train step (oracle/cpu_step.py) on the same Config S data at R = Nc = 4096
    (BASELINE.md §2 'CS-small'), all host threads via OpenMP."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from cpu_step import CpuTrainer
    from neus2_amd.pyngp import geometric_init_weights
    cfg = O.make_cfg()
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    p = O.init_params(cfg, geo=False)
    geo = geometric_init_weights(14, 64)
    p[: geo.size] = geo
    tr = CpuTrainer(cfg, ds, p, batch=4096, rays_per_batch=4096, fixed_rays=True)
    tr.step()  # step 0 includes the 2M-sample occupancy bootstrap; not timed
    t = time.perf_counter()
    for _ in range(n_steps):
        tr.step()
    dt = time.perf_counter() - t
    import platform
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": 4096 * n_steps / dt, "unit": "samples/s", "cores": O.num_threads(), "kind": "port",
            "sample": f"{n_steps} CPU-oracle train steps (incl. occupancy updates at cadence), Config S, R=Nc=4096; cpu={cpu}",
            "ms_per_step": dt / n_steps * 1e3, "host": platform.node()}


if __name__ == "__main__":
    main()
