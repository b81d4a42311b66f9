"""Level-partitioned gather experiment (development tool): on the bench workload after warm-up, times the
fused one-pass inference over the kept samples against the level-major encode alone (enc only, every level, the
blocks of one level resident together so its 2 MiB table sits in each XCD's L2) over the same samples."""
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
for name, kern, var in [("nerf_infer (fused, one pass)", 3, 0), ("encode only, 2048 wg/level", 11, 2048),
                        ("encode only, 4096 wg/level", 11, 4096), ("encode only, 1024 wg/level", 11, 1024),
                        ("encode only, 512 wg/level", 11, 512), ("train encode (Nc, enc + dy/dx)", 8, 0)]:
    ms = C.c_float()
    check(lib().neus_debug_time_kernel(tb.handle, kern, var, 9, C.byref(ms)))
    print(f"{name:34s}: {ms.value * 1e3:8.1f} us", flush=True)
