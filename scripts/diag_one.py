"""Times kernels (K: comma list of neus_testbed_time_kernel ids) over variants (V) after WARM training
steps (development tool; run under rocprofv3 --pmc for counters: V=99 launches only the timed kernel)."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from neus2_amd import pyngp, scenes
from neus2_amd._lib import lib, check
torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
tb.train_steps(int(os.environ.get("WARM", "800")))
for kern in [int(x) for x in os.environ.get("K", "0").split(",")]:
    for v in [int(x) for x in os.environ.get("V", "0").split(",")]:
        ms = C.c_float()
        check(lib().neus_debug_time_kernel(tb.handle, kern, v, int(os.environ.get("ITERS", "3")), C.byref(ms)))
        print(f"kernel {kern} v{v}: {ms.value * 1e3:9.1f} us", flush=True)
