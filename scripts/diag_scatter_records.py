"""Records per level of the grid-gradient scatter after the wave run merge, on the bench workload after warm-up
(development tool): records / (samples x 8 corners) shows how much the merge removes per level."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from neus2_amd import pyngp, scenes
from neus2_amd._lib import lib, check
torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
tb.train_steps(int(os.environ.get("WARM", "800")))
L = tb.layout()["n_levels"]
rec = np.zeros(L, np.uint64)
mx = C.c_uint32()
check(lib().neus_debug_scatter_stats(tb.handle, rec.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(mx)))
n = 1 << 18
for l in range(L):
    print(f"level {l:2d}: {int(rec[l]):10d} records = {rec[l] / (8 * n):.3f} of 8 per sample")
print(f"total {int(rec.sum())} records ({rec.sum() * 6 / 1e6:.1f} MB at 6 B), largest region {mx.value}")
