"""Launch gaps of single kernels replayed back to back (development tool, run under rocprofv3 --kernel-trace; then
scripts/prof_gaps.py --all): after 40 bench-shape training steps, ITERS replays each of the pre-compaction inference
(k_nerf_infer, one pass), the grid encode and the loss scan, so that the idle time between two launches of the same
kernel shows whether the gaps seen around k_nerf_infer in the step belong to that kernel's launch."""
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
tb.train_steps(40)
tb.synchronize()
iters = int(os.environ.get("ITERS", "10"))
variant = int(os.environ.get("VARIANT", "98"))  # 98: back to back, no event between the launches
for kid in (3, 8, 2):
    ms = C.c_float()
    check(lib().neus_debug_time_kernel(tb.handle, kid, variant, iters, C.byref(ms)))
    print("kernel", kid, "ms per launch", round(ms.value, 4), flush=True)
