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
# HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE/WRITE_SIZE, gfx950-corrected; see
# profiles/README.md). Filled from the committed profile of this round; None where not collected.
TRAFFIC = {}


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
    return p.parse_args()


# Algorithmic work per unit for the single-kernel phases. HBM bytes count compulsory
# streams only: the hash-grid table (21 MB fp16) and the fp32 grid gradient (42 MB) stay resident in the
# 256 MB Infinity Cache, so 8-corner gathers and atomics are not HBM traffic; grid_scatter adds one
# read-modify-write pass over the fp32 grid gradient per launch. The fused inference kernel moves only
# 60 B/sample through HBM, so its bound is the MFMA work (dense fp16 flops of the six layers).
COORD_B = 7 * 4          # NerfCoordinate AoS (pos, dt, dir)
OUT_B = 16 * 2           # network output / dL/dout rows, fp16 x 16
MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 (MI355X_MICROARCH.md)


def flops_per_sample(L=14, W=64):
    din = ((3 + 2 * L) + 15) // 16 * 16
    # density L0, L1, dSDF/d(din) through W1 row 0 and W0^T, rgb L0 (48 in), L1, L2
    return 2 * (din * W + W * 16 + W + W * din + 48 * W + W * W + W * 16)


def bytes_per_sample(L=14, W=64, din=32):
    enc = 2 * 2 * L                     # fp16 features, 2 per level
    dydx = 6 * 4 * L                    # f32 d(feature)/d(xyz)
    soa = 2 * 2 * (W + din + 16 + W) + 2 * (W + 48 + W + W + 16 + W)   # weight-grad operands, fp16
    return {
        "inference": COORD_B + OUT_B,
        "train_encode": COORD_B + enc + dydx,
        "mlp_train": COORD_B + enc + dydx + OUT_B + soa + 2 * enc + 16,
        "wgrad": soa,
        "grid_scatter": COORD_B + 2 * enc + 16,
    }


def roofline(name, ms, npre, ntrain, grid_params, L=14):
    """(bound, achieved, peak, unit, work per launch) of one single-kernel phase."""
    if name == "inference":
        fl = flops_per_sample(L) * npre
        return "mfma", fl / (ms * 1e-3) / 1e12, MFMA_PEAK_TFLOPS, "TFLOP/s", fl
    b = bytes_per_sample(L)[name] * ntrain + (8 * grid_params if name == "grid_scatter" else 0)
    return "hbm", b / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s", b


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
    # per-kernel timing with hipEvents recorded on the testbed's own stream (the stream every kernel of the
    # step is launched on), over a separate profiled pass of the same workload
    n_prof = max(4, min(32, args.steps // 4))
    tb.set_profiling(True)
    tb.train_steps(n_prof)
    phases, pinfo = tb.phase_times()
    tb.set_profiling(False)
    batch = args.batch
    samples = batch * world * args.steps
    value = samples / elapsed
    lay = tb.layout()
    single = ("inference", "train_encode", "mlp_train", "wgrad", "grid_scatter")
    dom = max(single, key=lambda k: phases[k])
    bound, achieved, peak, unit, work = roofline(dom, phases[dom], pinfo["npre"], pinfo["ntrain"], lay["n_grid_params"])
    rl_all = {}
    for k in single:
        if phases[k] > 0:
            bd, ac, pk, un, _ = roofline(k, phases[k], pinfo["npre"], pinfo["ntrain"], lay["n_grid_params"])
            rl_all[k] = {"ms": round(phases[k], 4), "bound": bd, "achieved": round(ac, 2), "unit": un, "frac": round(ac / pk, 4)}
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
        "roofline": {"bound": bound, "kernel": dom, "achieved": achieved, "peak": peak, "unit": unit,
                     "frac": achieved / peak, "traffic": TRAFFIC.get(dom), "work_per_launch": work,
                     "launch_ms": phases[dom]},
        "kernels": rl_all,
        "phase_ms": {k: round(v, 4) for k, v in phases.items()},
        "npre_per_step": pinfo["npre"], "ntrain_per_step": pinfo["ntrain"],
        "loss": st["ray_loss"],
        "warmup_s": warm_s,
    }
    if rank == 0 and args.cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(sc, args.cpu_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


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
