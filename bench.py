"""NeuS2 training throughput on MI355X (BASELINE.json metric: training samples/sec + PSNR@20k).

Workload (BASELINE.md §3 / SURVEY.md §8(d) "Config S"): DTU-scan24-shaped synthetic scene, 49 views of
1600x1200 RGBA8 (analytic sphere; DTU itself is not reachable here), configs/nerf/base.json
(14-level hash grid, width-64 MLPs), batch Nc = 2^18 compacted samples per GPU per step, R = 2^18
rays per GPU per step (adaptation frozen), occupancy-grid updates at the reference cadence.
A step = Testbed::train: occupancy update (when due) + sampling + pre-compaction forward + NeuS
loss/compaction + forward/backward (1st + 2nd order) + RCCL gradient all-reduce + Ema(Adam).

The timed state is config 2 as labelled: before the W warm-up steps the network is trained `--prepare` steps
(default 800) so that every hash-grid level is active (the progressive schedule of grid.h:2427-2440 enables the
last level at step 660). The fresh-network number (W warm-up + K timed steps from step 0, 4 active levels) is
reported beside it as the `early_steps` leg.

Usage: python bench.py --gpus N --steps K --warmup W
  N > 1: run under `torch.distributed.run` (one rank per GPU; WORLD_SIZE must equal N), or plainly, in which
  case this process starts `torch.distributed.run` itself as a child (before touching the GPU) and exits with
  its status.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 MFMA (MI355X_MICROARCH.md)
# Memory-side bytes per launch, measured by rocprofv3 PMC passes (scripts/gpu_traffic.sh -> profiles/traffic.json):
# reads = 128 B x TCC_EA0_RDREQ_128B + 64 B x the other read requests (FETCH_SIZE tallies 128-B requests at 64 B,
# the gfx950 half-count), writes = WRITE_SIZE; L2-to-fabric traffic, so Infinity Cache hits are included (an upper
# bound on DRAM bytes). Keyed by kernel and the number of active hash-grid levels of the replayed state; `traffic`
# is null when no measurement of that state exists. The file records the commit its passes ran at.
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def traffic_table():
    try:
        with open(TRAFFIC_FILE) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def measured_traffic(kernel, levels):
    e = traffic_table().get(f"{kernel}@L{levels}")
    return None if e is None else e.get("bytes_per_launch")


def traffic_source(tr, kernel, levels):
    """Where `roofline.traffic` comes from: a builder-run PMC pass (not this run), its summary file and commit."""
    e = tr.get(f"{kernel}@L{levels}")
    if e is None:
        return None
    return f"builder-run rocprofv3 PMC pass, profiles/{e.get('source')} at commit {e.get('commit')}"


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
    p.add_argument("--warmup", type=int, default=20)
    # training steps before the warm-up: the all-levels state of config 2 (every level active from step 660)
    p.add_argument("--prepare", type=int, default=800)
    p.add_argument("--views", type=int, default=49)
    p.add_argument("--width", type=int, default=1600)
    p.add_argument("--height", type=int, default=1200)
    p.add_argument("--batch", type=int, default=1 << 18)
    p.add_argument("--rays", type=int, default=1 << 18)
    p.add_argument("--cpu-baseline", type=int, default=1)
    p.add_argument("--cpu-steps", type=int, default=20)
    p.add_argument("--cpu-config1-steps", type=int, default=100)
    # quality half of the metric: PSNR after this many steps of the reference's (adaptive-R) training
    p.add_argument("--psnr-steps", type=int, default=20000)
    # config 5: marching cubes at mc_res^3 over the PSNR leg's trained model (0 = skip), N = 1
    p.add_argument("--mc-res", type=int, default=1024)
    # BASELINE.json words config 2 as a 16-level grid (the reference's base.json has 14): the same step at L=16
    p.add_argument("--l16", type=int, default=1)
    p.add_argument("--early", type=int, default=1)
    # data-parallel backend: "rccl" (one rank per GPU over xGMI, the production path) or "host" (the host-staged TCP
    # group, include/neus2_hip.h neus_host_group_create: ranks that cannot form an RCCL communicator, e.g. several on
    # one GPU with --same-device; a bring-up / test path whose exchange runs through host memory, not a scaling number)
    p.add_argument("--dp-backend", choices=("rccl", "host"), default="rccl")
    p.add_argument("--same-device", type=int, default=0, help="every rank on GPU 0 (with --dp-backend host)")
    p.add_argument("--rccl-info", type=int, default=1, help="N > 1 over RCCL: record RCCL's setup and algorithm / protocol "
                                                            "choices (NCCL_DEBUG=INFO into a file) in the bench line")
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
# MFMA flops per unit (SURVEY: 28,672 per pre-compaction sample, 92,160 per compacted sample), split over the
# kernels that carry them (W = 64, DIN = 32):
#   inference          : density fwd 6,144 + grad-SDF backward 6,144 + rgb fwd 16,384 = 28,672
#   mlp_train_rgb      : density fwd 6,144 + grad SDF 6,144 + rgb hidden fwd 14,336 + rgb dL/dinput 16,384 = 43,008
#   mlp_train_density  : density dL/dinput 6,144 + second-order front W0 u 4,096 = 10,240 (+ its recomputed
#                        density forward, not algorithmic)
#   weight gradients   : every layer's dW, first and second order = 28,672 (inside the training kernels, or k_wgrad)
def kernel_table(levels):
    g = 8 * levels * 4
    return {
        # name: (kernel id of neus_testbed_time_kernel, algorithmic bytes per unit, flops per unit)
        "march": (0, 40, 0),
        "march_write": (1, 28, 0),
        "inference": (3, 28 + g + 32, 28672),
        "train_encode": (8, 28 + g, 0),
        "mlp_train_rgb": (9, 32, 43008),
        "mlp_train_density": (10, 32, 10240),
        "grid_scatter": (7, 2 * g, 0),
        # Adam + EMA: 14 B per parameter + 34 B per stepped parameter (adam_bytes); the replay advances the optimizer
        # (after the timed steps)
        "adam_ema": (12, 48, 0),
        # the march of a cut step (the march cut: the slots below the compaction cut's estimate); last, it leaves a cut
        # march's state behind
        "march_cut": (13, 40, 0),
    }


INFER_STEPS = 10


def step_inference(it, levels):
    """The pre-compaction network pass as the training step runs it (progressive rounds of k_nerf_infer over their
    work lists): bytes = (28 coords + 32 L gather + 32 output) per evaluated sample, time = the launches' summed
    kernel durations (start/stop hipEvents given to hipExtLaunchKernelGGL); reported per launch (the rocprofv3 kernel-trace average of k_nerf_infer over the same steps)."""
    g = 8 * levels * 4
    n = max(1, it["launches"])
    ms = it["ms"] / n
    b = (28 + g + 32) * it["evaluated"] / n
    return {"ms": round(ms, 4), "units": round(it["evaluated"] / n), "bytes": round(b), "achieved": round(b / (ms * 1e-3) / 1e9, 1),
            "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "launches_per_step": round(it["launches"] / max(1, it["steps"]), 2),
            "evaluated_per_step": round(it["evaluated"] / max(1, it["steps"])), "ms_per_step": round(it["ms"] / max(1, it["steps"]), 4),
            "steps": it["steps"], "tflops": round(28672 * it["evaluated"] / (it["ms"] * 1e-3) / 1e12, 1),
            "note": "the step's own k_nerf_infer launches (progressive rounds), each launched with start/stop hipEvents (hipExtLaunchKernelGGL), timed over the steps after the timed region"}


def adam_bytes(tb):
    """The bytes the reference's optimizer step moves over the last step's gradient (adam.h:51-160 + ema.h:45-110):
    every parameter reads its fp16 gradient (2 B) and takes the EMA step (fp16 weight read, fp32 EMA read + write, fp16
    EMA write: 12 B); a parameter that steps (every matrix weight; the others only with a nonzero gradient, adam.h:
    107-110) also reads and writes its fp32 master weight, both moments and its step count and writes its fp16 weight
    (34 B): 14 P + 34 P_stepped. Returns (bytes, P, P_stepped)."""
    import numpy as np
    g = tb.get_gradients()
    n_matrix = tb.layout()["n_matrix"]
    stepped = n_matrix + int(np.count_nonzero(g[n_matrix:]))
    return 14 * g.size + 34 * stepped, int(g.size), stepped


def kernel_rooflines(tb, levels, iters=9):
    """Per-kernel median launch duration (hipEvents on the testbed stream between `iters` back-to-back
    launches replayed on the final training state, neus_testbed_time_kernel) and the algorithmic HBM
    roofline of each launch with `levels` active hash-grid levels."""
    out = {}
    ab = adam_bytes(tb)  # (the gradient the Adam replays run on)
    for name, (kid, bpu, fpu) in kernel_table(levels).items():
        ms, units = tb.time_kernel(kid, iters)
        b = bpu * units if name != "adam_ema" else ab[0]
        r = {"ms": round(ms, 4), "units": units, "bytes": b, "achieved": round(b / (ms * 1e-3) / 1e9, 1), "unit": "GB/s",
             "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if fpu:
            r["tflops"] = round(fpu * units / (ms * 1e-3) / 1e12, 1)
            r["mfma_frac"] = round(r["tflops"] / MFMA_PEAK_TFLOPS, 4)
        if name == "adam_ema":
            r["params_stepped"] = ab[2]
            r["note"] = ("bytes: what the reference's adam_step + Ema move for this gradient: 14 B per parameter (fp16 gradient "
                         "read and early-out, EMA step) + 34 B per stepped parameter (fp32 master weight, moments, step count, "
                         "fp16 weight); a parameter steps when it is a matrix weight or its gradient is nonzero (adam.h:107-110)")
        out[name] = r
    return out


def step_roofline(d, levels, n_params, ms_per_step, steps, adam_b=None):
    """Whole-step roofline: B_step = 40 R + 28 Npre + 568 Nev + 1496 Nc + 48 P + B_occ,
    with the gather terms at L_active levels, from the counters of the timed steps (this rank): every kept sample's
    coordinates are written (28 B), the pre-compaction network pass reads, gathers and writes only the samples it
    evaluates (Nev <= Npre: progressive inference skips samples past the transmittance cut-off) and the loss reads their
    outputs (28 + 32 L + 32 + 60 B). B_occ = (96 + 32 L) bytes per occupancy sample + a 32 MB grid pass per update.
    The optimizer term is adam_bytes of the last step (14 P + 34 P_stepped), or the upper bound 48 P without it.
    F_step = 28,672 Nev + 92,160 Nc."""
    g = 8 * levels * 4
    R, npre, nev, nc = d["rays"] / steps, d["pre"] / steps, d["evaluated"] / steps, d["train"] / steps
    occ = (d["occ_samples"] * (96 + g) + d["occ_updates"] * 32e6) / steps
    b = 40 * R + 28 * npre + (28 + g + 32 + 60) * nev + (60 + 28 + g + 32 + 32 + 2 * g) * nc + (adam_b or 48 * n_params) + occ
    f = 28672 * nev + 92160 * nc
    t = ms_per_step * 1e-3
    return {"bound": "hbm", "achieved": round(b / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(b / t / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_step": round(b), "flops_per_step": round(f),
            "mfma_tflops": round(f / t / 1e12, 1), "mfma_frac": round(f / t / 1e12 / MFMA_PEAK_TFLOPS, 4),
            "per_step": {"rays": round(R), "pre_samples": round(npre), "evaluated_samples": round(nev), "train_samples": round(nc),
                         "occ_samples": round(d["occ_samples"] / steps), "params": n_params}}


def work_counters(st):
    return {"rays": st["rays_total"], "pre": st["pre_samples_total"], "evaluated": st["evaluated_samples_total"],
            "occ_samples": st["occ_samples_total"], "occ_updates": st["occ_updates"], "progressive": st["progressive_steps"],
            "cut": st["cut_steps"], "mcut": st["march_cut_steps"], "mcut_reruns": st["march_cut_reruns"]}


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """One rank per GPU as fresh child processes (this process has not touched the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


RCCL_LOG = "/tmp/neus_bench_rccl.%h.%p.log"


def rccl_env(args, world):
    """RCCL's own report of its setup (NCCL_DEBUG=INFO, subsystems INIT / GRAPH / TUNING) into a per-process file, read
    back by rccl_info; never to stdout, which carries the bench line. Set before the communicator exists; a caller's own
    NCCL_DEBUG wins."""
    if world > 1 and args.dp_backend == "rccl" and args.rccl_info and "NCCL_DEBUG" not in os.environ:
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,GRAPH,TUNING", NCCL_DEBUG_FILE=RCCL_LOG)
        return True
    return False


def rccl_info(args, rank):
    """What RCCL reported about this rank's communicator (rccl_env): the channel / ring / tree setup lines of init and
    the algorithm / protocol it chose per message size (its TUNING lines), summarised; {} without a log."""
    import glob
    import re
    if os.environ.get("NCCL_DEBUG_FILE") != RCCL_LOG:
        return {}
    try:
        paths = [p for p in glob.glob(RCCL_LOG.replace("%h", "*").replace("%p", str(os.getpid())))]
        if not paths:
            return {"rccl_log": "missing"}
        init, choices = [], {}
        with open(paths[0], errors="replace") as f:
            for line in f:
                m = re.search(r"(\d+) Bytes -> Algo (\w+) proto (\w+)", line)
                if m:
                    choices.setdefault(f"algo {m.group(2)} proto {m.group(3)}", []).append(int(m.group(1)))
                elif len(init) < 24 and re.search(r"Init COMPLETE|nchannels|Channel 00|Trees|Pattern|NCCL_ALGO|NCCL_PROTO|Using", line):
                    init.append(line.strip()[-160:])
        return {"rccl": {"rank": rank, "init": init,
                         "choices": {k: {"calls": len(v), "min_bytes": min(v), "max_bytes": max(v)} for k, v in choices.items()}}}
    except Exception as e:  # the report is informational: never fail the bench over it
        return {"rccl_log_error": repr(e)[:200]}


class Group:
    """The gloo control plane of the ranks (RCCL communicators are created inside each C++ Testbed)."""

    def __init__(self, rank, world, backend="rccl"):
        self.rank, self.world, self.backend = rank, world, backend
        self.hgroups = []  # host groups outlive their testbeds' training (kept until close)
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo", init_method="env://")

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def max(self, v):
        if self.world == 1:
            return v
        import torch
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def attach(self, tb):
        """Data-parallel Testbed: a fresh RCCL unique id from rank 0, broadcast over gloo (or, with the host backend, rank
        0's TCP port for a fresh host group)."""
        if self.world == 1:
            return
        import torch.distributed as dist
        from neus2_amd import pyngp
        if self.backend == "host":
            obj = [(free_port(), int.from_bytes(os.urandom(8), "little")) if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            g = pyngp.HostGroup(self.rank, self.world, "127.0.0.1", obj[0][0], token=obj[0][1])
            g.join(tb)
            self.hgroups.append(g)
            return
        obj = [pyngp.nccl_unique_id() if self.rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        tb.init_data_parallel(self.rank, self.world, obj[0])

    def close(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


def make_testbed(sc, grp, device, args, cfg=None, fixed_rays=True):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf, device=device)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    kw = dict(batch_size=args.batch, fixed_rays_per_batch=args.rays) if fixed_rays else {}
    if cfg is None:
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), **kw)
    else:
        tb.reload_network_from_json(cfg, **kw)
    grp.attach(tb)
    return tb


def timed_steps(tb, grp, warmup, steps, batch):
    """W untimed warm-up steps, then exactly K steps bracketed by a barrier + device synchronisation on both
    sides; the max over ranks. Returns (seconds, work counters of the timed steps)."""
    import torch

    def barrier():
        tb.synchronize()
        torch.cuda.synchronize()
        grp.barrier()

    tb.train_steps(warmup)
    barrier()
    st0 = tb.stats()
    if grp.world > 1:  # per step: the join before Adam waiting for the collectives (events, no host wait per step)
        tb.set_exchange_timing(True)
    t1 = time.perf_counter()
    tb.train_steps(steps)
    barrier()
    elapsed = grp.max(time.perf_counter() - t1)
    st1 = tb.stats()
    w0, w1 = work_counters(st0), work_counters(st1)
    d = {k: w1[k] - w0[k] for k in w0}
    if grp.world > 1:
        x = tb.exchange_timing()
        tb.set_exchange_timing(False)
        info = tb.data_parallel_info()
        k = max(1, x["steps"])
        d["exchange"] = {"exposed_us_per_step": round(grp.max(x["exposed_ms"] / k) * 1e3, 1),
                         "span_us_per_step": round(grp.max(x["span_ms"] / k) * 1e3, 1), "steps": x["steps"],
                         "allreduce_bytes_last_step": int(info["last_step_allreduce_bytes"]),
                         "note": "exposed = max over ranks of the mean per-step wait of the join before Adam for the "
                                 "collectives (end of the last collective - end of the backward, hipEvents); span = end of "
                                 "the last collective - end of the loss (the counters' all-reduce starts there)"}
    d["train"] = steps * batch
    d["trained_real"] = st1["trained_samples_total"] - st0["trained_samples_total"]
    return elapsed, d, st1


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        if args.dp_backend != "host" and world > 1:
            print("bench.py: --same-device needs --dp-backend host (RCCL refuses two ranks on one GPU)", file=sys.stderr)
            sys.exit(2)
        local = 0
    rccl_env(args, world)
    import torch
    grp = Group(rank, world, args.dp_backend)
    torch.cuda.set_device(local)
    from neus2_amd import scenes
    sc = scenes.sphere_scene(args.views, args.width, args.height, principal=(823.2 / 1600, 619.1 / 1200))
    tb = make_testbed(sc, grp, local, args)
    t0 = time.time()
    tb.train_steps(args.prepare)
    tb.synchronize()
    prepare_s = time.time() - t0
    tb.set_profiling(False)
    elapsed, d, st = timed_steps(tb, grp, args.warmup, args.steps, args.batch)
    batch = args.batch
    # every step trains on Nc = batch samples per GPU (the reference's m_training_batch_size; a short compaction
    # is rollover-padded, fill_rollover_and_rescale); the non-rollover share is reported next to it
    value = batch * world * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3
    lay = tb.layout()
    levels = min(st["valid_level"] + 1, lay["n_levels"])
    # the dominant kernel as the training step runs it: after the timed region, INFER_STEPS more steps with hipEvents
    # around each pre-compaction network launch (the progressive rounds' k_nerf_infer), the samples they evaluated
    # from the device counter
    it = tb.infer_timing(INFER_STEPS)
    inf = step_inference(it, levels)
    # per-kernel timing of the other kernels after that, on the final state (hipEvents on the testbed stream)
    kern = kernel_rooflines(tb, levels)
    per_step = {k: v["ms"] for k, v in kern.items() if k not in ("inference", "march_cut")}
    per_step["inference_step"] = inf["ms_per_step"]
    # the step's march: the cut march on the steps that cut it, the full march on the others (the replays time both)
    fcut = d["mcut"] / max(1, args.steps)
    per_step["march"] = round(fcut * kern["march_cut"]["ms"] + (1 - fcut) * kern["march"]["ms"], 4)
    dom = max(per_step, key=per_step.get)
    dk = inf if dom == "inference_step" else kern[dom]
    mlp = ("mlp_train_rgb", "mlp_train_density")
    mlp_ms = sum(kern[k]["ms"] for k in mlp)
    tr = traffic_table()
    out = {
        "metric": "training samples/sec (compacted NeuS2 training samples, DTU-scan24-shaped synthetic, base.json)",
        "value": value,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16 MFMA (fp32 accumulate) / fp32 optimizer",
        "data": "synthetic (analytic sphere, 49 x 1600x1200 RGBA8 views; DTU scan24 unavailable offline)",
        "config": {"workload": "NeuS2 train step, Config S, base.json L=14 T=2^19 W=64, Nc=2^18/GPU, R=2^18/GPU fixed, "
                               f"all {levels} levels active (network trained {args.prepare} steps before the warm-up)",
                   "global_batch": batch * world, "rays_per_gpu": args.rays, "parallelism": f"dp{world}",
                   "dp_backend": args.dp_backend if world > 1 else None,
                   **({"same_device": True} if args.same_device and world > 1 else {}),
                   "prepare_steps": args.prepare, "levels_active": levels},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": dk["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": dk["frac"], "traffic": measured_traffic(dom, levels), "bytes_per_launch": dk["bytes"],
                     "units_per_launch": dk["units"], "launch_ms": dk["ms"], "levels_active": levels,
                     "traffic_source": traffic_source(tr, dom, levels),
                     **({k: inf[k] for k in ("launches_per_step", "evaluated_per_step", "ms_per_step", "steps", "note")}
                        if dom == "inference_step" else {})},
        # the whole step against the HBM roofline and its MFMA rate
        "roofline_step": step_roofline(d, levels, lay["n_params"], ms_step, args.steps, kern["adam_ema"]["bytes"]),
        # the training MLP kernels (fwd recompute + 1st / 2nd-order backward + weight gradients) against the MFMA peak
        "mfma_mlp_train": {"flops_per_sample": 43008 + 10240 + 28672, "ms": round(mlp_ms, 4),
                           "tflops": round((43008 + 10240 + 28672) * batch / (mlp_ms * 1e-3) / 1e12, 1),
                           "frac": round((43008 + 10240 + 28672) * batch / (mlp_ms * 1e-3) / 1e12 / MFMA_PEAK_TFLOPS, 4)},
        # memory-side line traffic (PMC, profiles/traffic.json) over the same launch: the hashed levels' 4-B corner
        # gathers each move a 128-B line from the Infinity Cache, so this, not the algorithmic rate, is what binds
        "line_traffic": line_traffic(measured_traffic(dom, levels), dk["ms"], dk["bytes"]),
        "progressive_steps_timed": d["progressive"],
        # steps whose later progressive rounds skipped the rays past the compaction cut (their network outputs
        # feed no training sample; the trained parameters are bitwise those without the cut, NEUS_PROG_CUT=0)
        "compaction_cut_steps_timed": d["cut"],
        # steps whose sampling marched only the slots below the cut's estimate, and steps run again with the full march
        # because the cut march's witness failed (nothing of the first run is applied)
        "march_cut_steps_timed": d["mcut"], "march_cut_reruns_timed": d["mcut_reruns"],
        "progressive_chunk_end": st["progressive_chunk_end"],
        "non_rollover_fraction": round(d["trained_real"] / max(1, batch * args.steps), 4),
        **({"exchange": {**d["exchange"], **rccl_info(args, rank)}} if "exchange" in d else {}),
        "kernels": kern,
        "loss": st["ray_loss"],
        "prepare_s": round(prepare_s, 3),
    }
    del tb
    if args.early:
        out["early_steps"] = early_leg(sc, grp, local, args)
    if world == 1 and args.l16:
        out["levels16"] = l16_leg(sc, grp, local, args)
    if args.psnr_steps > 0:
        out["psnr"], tb2 = psnr_leg(sc, grp, local, args)
        if world == 1 and args.mc_res > 0:
            out["marching_cubes"] = marching_cubes_leg(tb2, args.mc_res)
        del tb2
    if rank == 0 and args.cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(sc, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    grp.close()


def early_leg(sc, grp, device, args):
    """The same step on a fresh network: W warm-up + K timed steps from step 0 (the first progressive levels,
    occupancy updates every step): the driver-shaped transient."""
    tb = make_testbed(sc, grp, device, args)
    elapsed, d, st = timed_steps(tb, grp, args.warmup, args.steps, args.batch)
    levels = min(st["valid_level"] + 1, tb.layout()["n_levels"])
    del tb
    return {"value": args.batch * grp.world * args.steps / elapsed, "unit": "samples/s", "ms_per_step": elapsed / args.steps * 1e3,
            "steps": f"{args.warmup}..{args.warmup + args.steps}", "levels_active_at_end": levels}


def l16_leg(sc, grp, device, args):
    """The timed step of the main measurement with a 16-level hash grid (base.json otherwise): same data, batch,
    rays, preparation and warmup / steps."""
    from neus2_amd import config
    cfg = config.load_json(os.path.join(ROOT, "configs", "nerf", "base.json"))
    cfg["encoding"]["n_levels"] = 16
    tb = make_testbed(sc, grp, device, args, cfg=cfg)
    tb.train_steps(args.prepare)
    elapsed, d, st = timed_steps(tb, grp, args.warmup, args.steps, args.batch)
    levels = min(st["valid_level"] + 1, 16)
    ms_step = elapsed / args.steps * 1e3
    inf_ms, inf_units = tb.time_kernel(3, 9)
    g = 8 * levels * 4
    n_params = tb.layout()["n_params"]
    del tb
    return {"value": args.batch * grp.world * args.steps / elapsed, "unit": "samples/s", "ms_per_step": ms_step,
            "levels_active": levels, "roofline_step": step_roofline(d, levels, n_params, ms_step, args.steps),
            "inference": {"ms": round(inf_ms, 4), "units": inf_units,
                          "achieved_GBs": round((28 + g + 32) * inf_units / (inf_ms * 1e-3) / 1e9, 1)}}


def psnr_leg(sc, grp, device, args):
    """PSNR@n_steps (BASELINE.json metric, second half) with the reference's training (adaptive rays per
    batch, Nc = 2^18 per GPU) and evaluation protocol (render_utils.py:252-359: view 0, spp 8, black background,
    pixel centres, min transmittance 1e-4, EMA weights); at N > 1 every rank trains its ray shard (the global batch
    is N x 2^18) and rank 0 renders. scripts/psnr_run.py is the standalone version."""
    from neus2_amd import pyngp
    n_steps = args.psnr_steps
    tb = make_testbed(sc, grp, device, args, fixed_rays=False)
    t0 = time.perf_counter()
    done = 0
    while done < n_steps:
        k = min(2000, n_steps - done)
        tb.train_steps(k)
        done += k
        tb.synchronize()  # also a progress point for long runs
    grp.barrier()
    train_s = grp.max(time.perf_counter() - t0)
    out = {"unit": "dB", "steps": n_steps, "train_wall_s": round(train_s, 2), "n_gpus": grp.world,
           "protocol": "view 0, spp 8, black bg, snap_to_pixel_centers, min_T 1e-4, EMA weights",
           "training": f"reference schedule: adaptive rays/batch, Nc=2^18 per GPU, base.json, dp{grp.world}"}
    if grp.rank == 0:
        tb.background_color = [0.0, 0.0, 0.0, 0.0]
        tb.snap_to_pixel_centers = True
        tb.nerf.rendering_min_transmittance = 1e-4
        tb.set_camera_to_training_view(0)
        gt = sc["images"][0]
        t1 = time.perf_counter()
        img = tb.render(gt.shape[1], gt.shape[0], spp=8)
        out["render_s"] = round(time.perf_counter() - t1, 3)
        psnr, _ = pyngp.eval_psnr(img, gt)
        out["value"] = round(float(psnr), 3)
    grp.barrier()
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


def host_cpu():
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return cpu, os.cpu_count(), aff


def cpu_baseline(sc, args):
    """The CPU oracle's train step (oracle/cpu_step.py, the reference's algorithm restated in C++ with OpenMP; the
    reference has no CPU path) beside the GPU run:
      * Config S at R = Nc = 4096 ('CS-small'), --cpu-steps steps after an untimed first step;
      * config 1 in full: the 1-view 64x64 sphere, 1-level grid, width-16 MLPs, R = Nc = 4096, 100 steps from step 0
        (occupancy updates at the reference cadence included).
    Threads: OpenMP's count in this process (OMP_NUM_THREADS when set: the GPU pool sets it to the lease's CPU share)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from cpu_step import CpuTrainer
    from neus2_amd import scenes
    from neus2_amd.pyngp import geometric_init_weights
    cfg = O.make_cfg()
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    p = O.init_params(cfg, geo=False)
    geo = geometric_init_weights(14, 64)
    p[: geo.size] = geo
    tr = CpuTrainer(cfg, ds, p, batch=4096, rays_per_batch=4096, fixed_rays=True)
    tr.step()  # step 0 includes the 2M-sample occupancy bootstrap; not timed
    t = time.perf_counter()
    for _ in range(args.cpu_steps):
        tr.step()
    dt = time.perf_counter() - t
    cpu, nproc, aff = host_cpu()
    out = {"value": 4096 * args.cpu_steps / dt, "unit": "samples/s", "cores": O.num_threads(), "kind": "port",
           "sample": f"{args.cpu_steps} CPU-oracle train steps (incl. occupancy updates at cadence), Config S, R=Nc=4096",
           "ms_per_step": round(dt / args.cpu_steps * 1e3, 1),
           "host": {"cpu": cpu, "nproc": nproc, "affinity_cpus": aff, "omp_threads": O.num_threads(),
                    "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}}
    if args.cpu_config1_steps > 0:
        c1 = scenes.config1_scene()
        cfg1 = O.make_cfg(n_levels=1, width=16, per_level_scale=2.0)
        ds1 = O.Dataset(c1["images"], c1["focal"], c1["principal"], c1["xforms"])
        p1 = O.init_params(cfg1, geo=False)
        g1 = geometric_init_weights(1, 16)
        p1[: g1.size] = g1
        tr1 = CpuTrainer(cfg1, ds1, p1, batch=4096, rays_per_batch=4096, fixed_rays=True)
        t = time.perf_counter()
        for _ in range(args.cpu_config1_steps):
            tr1.step()
        dt1 = time.perf_counter() - t
        out["config1"] = {"value": 4096 * args.cpu_config1_steps / dt1, "unit": "samples/s", "steps": args.cpu_config1_steps,
                          "ms_per_step": round(dt1 / args.cpu_config1_steps * 1e3, 1),
                          "sample": "config 1 in full: 1 view 64x64, L=1, W=16, R=Nc=4096, steps 0..99 incl. occupancy updates",
                          "last_loss": round(float(tr1.last["loss"]), 6)}
    return out


if __name__ == "__main__":
    main()
