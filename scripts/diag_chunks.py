"""Per-ray sample statistics of the training step at several training states (development tool for the progressive
inference's chunk boundaries): per ray with samples the requested count ns and the composited count cc (samples up to
the transmittance cut-off), and the samples each candidate boundary set would evaluate (min(ns, first boundary >= cc))."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from neus2_amd import pyngp, scenes  # noqa: E402

torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
CANDS = [(32, 64, 96), (24, 48), (32, 64), (40, 80), (48, 96), (56, 112), (64, 128), (80, 160)]
done = 0
for warm in [int(x) for x in os.environ.get("STATES", "400,800,1200,1600,2400").split(",")]:
    tb.train_steps(warm - done)
    done = warm
    st = tb.stats()
    _, cc, ns = tb.ray_counts(1 << 18)  # ns: kept samples per ray slot (0: no samples or dropped past the cap)
    m = ns > 0
    ns, cc = ns[m].astype(np.int64), cc[m].astype(np.int64)
    q = np.percentile(cc, [25, 50, 75, 90, 99])
    print(f"step {warm}: rays with samples {m.sum()} (stats {st['n_rays_with_samples']}), kept {ns.sum()}, composited {cc.sum()} "
          f"(measured_batch_size {st['measured_batch_size']}), mean cc {cc.mean():.1f} mean ns {ns.mean():.1f}, "
          f"cc quartiles/p90/p99 {q.round(0).tolist()}", flush=True)
    for c in CANDS:
        ev = ns.copy()
        open_ = np.ones_like(ns, bool)
        first = np.full_like(ns, -1)
        for e in c:
            hit = open_ & (cc <= e)
            first[hit] = e
            open_ &= ~hit
        ev = np.where(first >= 0, np.minimum(ns, first), ns)
        print(f"   chunks {c}: evaluated {ev.sum()} ({ev.sum() / ns.sum():.3f} of kept), rounds {len(c) + 1}", flush=True)
