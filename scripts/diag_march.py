"""SIMT efficiency of the occupancy march on the bench workload (development tool).
Per ray: march_step calls (outer), skip-loop additions (inner), samples; per wave of 64 rays the
loop runs max(outer) iterations."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from neus2_amd import pyngp, scenes
from neus2_amd._lib import lib, check
torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
done = 0
for target in [int(x) for x in os.environ.get("STEPS", "100,800,2000").split(",")]:
    tb.train_steps(target - done); done = target
    n = 1 << 18
    out = np.zeros(3 * n, np.uint32)
    check(lib().neus_debug_march_stats(tb.handle, n, out.ctypes.data_as(C.POINTER(C.c_uint32))))
    o = out.reshape(n, 3).astype(np.float64)
    outer, inner, ns = o[:, 0], o[:, 1], o[:, 2]
    w = outer.reshape(-1, 64)
    eff = w.mean(1).sum() / w.max(1).sum()
    print(f"step {target}: rays {n} outer mean {outer.mean():.1f} max {outer.max():.0f} p50 {np.median(outer):.0f} p99 {np.percentile(outer, 99):.0f}; "
          f"inner mean {inner.mean():.1f}; samples mean {ns.mean():.1f} max {ns.max():.0f}; wave SIMT eff {eff:.3f}; "
          f"sum wave-max {w.max(1).sum():.3e} vs sum/64 {outer.sum() / 64:.3e}", flush=True)
    m = int(os.environ.get("FIRST", "22000"))
    print(f"   first {m} rays: outer mean {outer[:m].mean():.1f} p99 {np.percentile(outer[:m], 99):.0f} max {outer[:m].max():.0f}; "
          f"inner mean {inner[:m].mean():.1f} max {inner[:m].max():.0f}; samples mean {ns[:m].mean():.1f} max {ns[:m].max():.0f}", flush=True)
    for k in (1, 2, 4, 8):  # efficiency if waves took k*64 rays with perfect refill
        ww = outer.reshape(-1, 64 * k)
        print(f"   refill pool {64 * k}: max-lane-sum bound eff {(ww.sum(1) / 64).sum() / np.maximum(ww.max(1), ww.sum(1) / 64).sum():.3f}")
