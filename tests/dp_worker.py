"""One data-parallel rank as its own process (tests/test_gpu_dp_procs.py): the 8-view 64x48 scene, base.json at a
4096-sample batch and `rays` fixed rays per rank, attached to a cross-process host group (neus_host_group_create) on
GPU 0, `steps` training steps, then the rank's parameters, gradients, EMA weights, density grid and counters to an .npz.
Usage: python tests/dp_worker.py RANK WORLD PORT STEPS RAYS OVERLAP OUT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, steps, rays, overlap = (int(v) for v in sys.argv[1:7])
    out = sys.argv[7]
    import numpy as np
    from neus2_amd import pyngp, scenes
    sc = scenes.small_scene(n_views=8, width=64, height=48)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf, device=0)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096, fixed_rays_per_batch=rays)
    group = pyngp.HostGroup(rank, world, "127.0.0.1", port, token=(port * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
    group.join(tb)
    tb.set_exchange_overlap(bool(overlap))
    tb.train_steps(steps)
    st = tb.stats()
    info = tb.data_parallel_info()
    grid, bf = tb.get_density_grid()
    np.savez(out, params=tb.get_params(), grads=tb.get_gradients(), ema=tb.get_ema_params(), grid=grid, bitfield=bf,
             stats=np.array([st["training_step"], st["rays_per_batch"], st["measured_batch_size"], st["n_rays_total"]], np.uint64),
             loss=np.float32(st["loss"]), coll_calls=np.uint64(info["collective_calls"]), coll_bytes=np.uint64(info["allreduce_bytes"]),
             host_group=np.uint32(info["host_group"]))
    del tb
    del group
    print(f"rank {rank}: {steps} steps ok", flush=True)


if __name__ == "__main__":
    main()
