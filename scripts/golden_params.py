"""Regression fingerprint (development tool): trains the bench scene for a few steps at a reduced batch and saves
the parameters, the occupancy grid and the per-ray counts, so a kernel restructuring that must not change a bit
can be compared against the build before it: python scripts/golden_params.py OUT.npz [--compare REF.npz]."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from neus2_amd import pyngp, scenes
torch.cuda.set_device(0)
out = sys.argv[1]
sc = scenes.sphere_scene(16, 400, 300, principal=(0.51, 0.52))
res = {}
for name, steps, extra in (("early", 12, None), ("late", 300, None)):
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 16)
    tb.train_steps(steps)
    res[name + "_params"] = tb.get_params()
    res[name + "_ema_h"] = tb.get_half_params(True).view(np.uint16)
    g, bf = tb.get_density_grid()
    res[name + "_grid"] = g
    res[name + "_counts"] = np.concatenate(tb.ray_counts(1 << 16)[:2])
    del tb
import hashlib
# digests of the full arrays + every 257th element (small enough to travel back from the GPU box)
small = {k: v[::257].copy() for k, v in res.items()}
small.update({k + "_sha": np.frombuffer(hashlib.sha256(v.tobytes()).digest(), np.uint8) for k, v in res.items()})
np.savez(out, **small)
if "--compare" in sys.argv:
    ref = np.load(sys.argv[sys.argv.index("--compare") + 1])
    bad = [k for k in res if not np.array_equal(small[k + "_sha"], ref[k + "_sha"])]
    for k in res:
        if k in bad:
            a, b = small[k].astype(np.float64), ref[k].astype(np.float64)
            print(f"{k}: DIFFERENT (sampled) max|d| {np.abs(a - b).max():.3g} frac {np.mean(a != b):.3g}")
        else:
            print(f"{k}: identical")
    sys.exit(1 if bad else 0)
