"""Bitwise fingerprint of training at the bench's shape (development tool): Config S (49 views of 1600x1200), base.json,
R = Nc = 2^18 fixed, STEPS steps in one train call (default 900: the all-levels state, the progressive rounds, the
compaction cut, the lookahead), then SHA-256 of the parameters, fp16 EMA weights, occupancy grid and the final counters.
Run it under two settings and compare: python scripts/fingerprint_bench_shape.py OUT.json [--compare REF.json]."""
import hashlib
import json
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
tb.train_steps(int(os.environ.get("STEPS", "900")))
st = tb.stats()
g, bf = tb.get_density_grid()
sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
res = {"params": sha(tb.get_params()), "ema_h": sha(tb.get_half_params(True)), "grid": sha(g), "bitfield": sha(bf),
       "counters": {k: st[k] for k in ("training_step", "rays_per_batch", "measured_batch_size", "measured_batch_size_before_compaction",
                                       "n_rays_total", "loss")},
       "work": {k: st[k] for k in ("evaluated_samples_total", "cut_steps", "lookahead_steps", "progressive_steps", "march_cut_steps",
                                   "march_cut_reruns")},
       "env": {k: v for k, v in os.environ.items() if k.startswith("NEUS_")}}
json.dump(res, open(sys.argv[1], "w"), indent=1)
print(json.dumps(res))
if "--compare" in sys.argv:
    ref = json.load(open(sys.argv[sys.argv.index("--compare") + 1]))
    same = all(res[k] == ref[k] for k in ("params", "ema_h", "grid", "bitfield", "counters"))
    print("FINGERPRINT", "EQUAL" if same else "DIFFERENT", {k: res[k] == ref[k] for k in ("params", "ema_h", "grid", "bitfield", "counters")})
    sys.exit(0 if same else 1)
