"""The occupancy update's density pass split by its halves (development tool): after PREP bench-shape training steps,
neus_debug_time_kernel id 14 times k_nerf_density MODE 2 over both halves (nc/4 uniform samples in cell order + nc/4
occupancy-biased samples, the update after step 256), the uniform half alone and the occupancy-biased half alone."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from neus2_amd import pyngp, scenes  # noqa: E402
from neus2_amd._lib import check, lib  # noqa: E402

torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
tb.train_steps(int(os.environ.get("PREP", "800")))
tb.synchronize()
for variant, name in ((0, "both halves"), (1, "uniform half"), (2, "occupancy-biased half")):
    ms = C.c_float()
    check(lib().neus_debug_time_kernel(tb.handle, 14, variant, 5, C.byref(ms)))
    print(f"occupancy density pass, {name}: {ms.value * 1e3:.1f} us", flush=True)
