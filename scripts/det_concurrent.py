"""Development check: two testbeds of the same (or different, AB=1) scatter mode trained step by step on their own
streams, concurrently; the first step whose parameters / occupancy grid differ is reported with where they differ."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
torch.cuda.set_device(0)
from neus2_amd import pyngp, scenes
sc = scenes.small_scene(n_views=8, width=64, height=48)


def mk(mode):
    if mode: os.environ['NEUS_SCATTER'] = mode
    else: os.environ.pop('NEUS_SCATTER', None)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
    os.environ.pop('NEUS_SCATTER', None)
    return tb


reps, steps = int(os.environ.get("REPS", "3")), int(os.environ.get("STEPS", "40"))
mode_b = 'binned' if os.environ.get("AB", "0") == "1" else None
for rep in range(reps):
    a, b = mk(None), mk(mode_b)
    lay = a.layout()
    offs = lay.get("level_offsets")
    found = False
    for k in range(steps):
        a.train_steps(1); b.train_steps(1)
        pa, pb = a.get_params(), b.get_params()
        ga, gb = a.get_density_grid(), b.get_density_grid()
        d = np.nonzero(pa.view(np.uint32) != pb.view(np.uint32))[0]
        dg = [int(np.count_nonzero(np.asarray(x).view(np.uint8) != np.asarray(y).view(np.uint8))) for x, y in zip(ga, gb)]
        if len(d) or any(dg):
            g0 = lay["grid_offset"]
            gi = d[d >= g0] - g0
            print(f"rep {rep} step {k}: {len(d)} params differ (MLP {int((d < g0).sum())}, grid {len(gi)}; first grid entries "
                  f"{(gi[:6] // 2).tolist()}); density grid / bitfield bytes differ {dg}", flush=True)
            found = True
            break
    if not found:
        print(f"rep {rep}: equal through {steps} steps", flush=True)
    del a, b
