"""Times kernel variants on the bench workload after warm-up (development tool)."""
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
names = {0: "march_count", 1: "march_write", 2: "loss_scan", 3: "nerf_infer", 4: "loss_alpha", 5: "mlp_train", 6: "wgrad", 7: "grid_scatter"}
for kern, variants in [(0, (0,)), (1, (0,)), (2, (0,)), (3, (0,)), (4, (0,)), (5, (0,)), (6, (0,)), (7, (0,))]:
    for v in variants:
        ms = C.c_float()
        check(lib().neus_debug_time_kernel(tb.handle, kern, v, 10, C.byref(ms)))
        print(f"{names[kern]:12s} v{v}: {ms.value * 1e3:9.1f} us", flush=True)
