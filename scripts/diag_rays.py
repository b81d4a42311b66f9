"""Ray-length statistics of the bench workload after warm-up (diagnostic for the per-ray kernels)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from neus2_amd import pyngp, scenes
torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
out = {}
for steps in (300, 800, 2000):
    tb.train_steps(steps - tb.training_step)
    nreq, cn, comp = tb.ray_counts()
    q = lambda a: [int(np.percentile(a, p)) for p in (50, 90, 99, 99.9, 100)]
    kept = nreq[comp > 0] if (comp > 0).any() else nreq[:0]
    out[steps] = dict(rays_with_req=int((nreq > 0).sum()), req_total=int(nreq.sum()), req_pct=q(nreq[nreq > 0]) if (nreq > 0).any() else [],
                      cn_total=int(cn.sum()), cn_pct=q(cn[cn > 0]) if (cn > 0).any() else [], comp_rays=int((comp > 0).sum()),
                      last_kept_ray=int(np.nonzero(comp)[0].max()) if (comp > 0).any() else -1)
    print(steps, json.dumps(out[steps]), flush=True)
