"""Data-parallel decomposition on the CPU (world_size 2, gloo), SURVEY.md §8(e):

* rank r samples global rays r*R .. r*R+R-1 (rng.advance(i_g * 8), image_idx over world*R), so the
  union over ranks is bit-identical to one process sampling world*R rays;
* per-rank gradients are summed (the RCCL all-reduce of the device build) together with the two
  step counters, after which every rank takes the same Adam step and the parameters stay identical.

The ranks run the CPU train-step composer (oracle/cpu_step.py) over the oracle kernels; the device
build runs the same decomposition with ncclAllReduce inside NeusTestbed::train_step."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from neus2_amd import scenes
    sc = scenes.small_scene(n_views=4, width=32, height=24)
    cfg = O.make_cfg(n_levels=2, log2_hashmap_size=12, base_resolution=8, per_level_scale=2.0)
    ds = O.Dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"])
    return O, cfg, ds


def _worker(rank, world, port, R, steps, out_dir):
    os.environ["OMP_NUM_THREADS"] = "2"
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    O, cfg, ds = _setup()
    from cpu_step import CpuTrainer
    p0 = O.init_params(cfg)
    tr = CpuTrainer(cfg, ds, p0, batch=8192, rays_per_batch=R, fixed_rays=True, rank=rank, world=world)
    ref = CpuTrainer(cfg, ds, p0, batch=8192, rays_per_batch=R * world, fixed_rays=True)
    for s in range(steps):
        g = tr.grads()
        # the sampling of this rank equals its slice of the single-process world*R sampling
        ref.grads(skip_occupancy=False)
        sl = slice(rank * R, (rank + 1) * R)
        np.testing.assert_array_equal(tr.last["rays"].view(np.uint32), ref.last["rays"][sl].view(np.uint32))
        # per-ray step counts agree wherever both runs kept the ray (each run applies its own
        # max-samples cap over its own prefix sum, so the kept sets may differ at the tail)
        mine, theirs = tr.last["numsteps"][:, 0], ref.last["numsteps"][sl, 0]
        both = (mine > 0) & (theirs > 0)
        assert both.sum() > R // 4
        np.testing.assert_array_equal(mine[both], theirs[both])
        gt = torch.from_numpy(g)
        dist.all_reduce(gt)
        cnt = torch.tensor([tr.last["numsteps_counter"], tr.last["compacted"]], dtype=torch.int64)
        dist.all_reduce(cnt)
        tr.finish(gt.numpy(), (int(cnt[0]), int(cnt[1])))
        # keep the single-process reference in lock-step on the parameters and rng
        ref.params[:] = tr.params
        ref.finish(np.zeros_like(g), (int(cnt[0]), int(cnt[1])))
        ref.params[:] = tr.params
    np.save(os.path.join(out_dir, f"params_{rank}.npy"), tr.params)
    np.save(os.path.join(out_dir, f"state_{rank}.npy"), np.array([tr.rng_state, tr.n_rays_total, tr.R], np.uint64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_gloo_world2_rays_and_allreduce(tmp_path):
    import torch.multiprocessing as mp
    world, R, steps = 2, 256, 2
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, R, steps, str(tmp_path)), nprocs=world, join=True, start_method="spawn")
    p0, p1 = np.load(tmp_path / "params_0.npy"), np.load(tmp_path / "params_1.npy")
    np.testing.assert_array_equal(p0, p1)
    s0, s1 = np.load(tmp_path / "state_0.npy"), np.load(tmp_path / "state_1.npy")
    np.testing.assert_array_equal(s0, s1)
    assert int(s0[1]) == steps * world * R  # n_rays_total advances by the global ray count
