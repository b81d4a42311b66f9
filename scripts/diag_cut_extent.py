"""Where the compaction cut falls among the marched ray slots (development tool, round 6).

At the bench's shape (Config S, base.json L=14, R = Nc = 2^18 fixed) this trains one testbed to the states in STATES and,
after each (the last step of a call never cuts, so its per-ray counters are complete), reads per ray slot the march's
requested sample count (nreq), the composited count (ccount) and the compaction base (numsteps[2r + 1]). It reports the
kept extent (slots the march keeps under the pre-compaction cap), the cut (the first slot whose compaction base reaches the
batch: no later ray contributes a training sample), and the share of the march's work (requested samples, and the rays
with samples) below the cut - what a march limited to the cut would still have to do.
Output: one JSON line per state."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from neus2_amd import pyngp, scenes  # noqa: E402
from neus2_amd._lib import check, lib  # noqa: E402


def buf(tb, i, n, dt=np.uint32):
    a = np.zeros(n, dt)
    check(lib().neus_debug_get_buffer(tb.handle, i, C.c_uint64(0), C.c_uint64(a.nbytes), a.ctypes.data_as(C.c_void_p)))
    return a


def main():
    states = [int(x) for x in os.environ.get("STATES", "200,800,1600").split(",")]
    torch.cuda.set_device(0)
    R = 1 << 18
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=R, fixed_rays_per_batch=R)
    done = 0
    for s in states:
        tb.train_steps(s - done)
        tb.synchronize()
        done = s
        st = tb.stats()
        nreq = buf(tb, 14, R).astype(np.int64)
        cc = buf(tb, 8, R).astype(np.int64)
        ns = buf(tb, 12, 2 * R).reshape(R, 2).astype(np.int64)
        extent = int(st["kept_ray_extent"])
        cb = ns[:, 1]
        kept = np.arange(R) < extent
        past = np.nonzero(kept & (cb >= R))[0]
        cut = int(past[0]) if len(past) else extent
        req = np.where(kept, nreq, 0)
        out = {"step": st["training_step"], "kept_extent": extent, "cut": cut, "cut_over_extent": round(cut / max(1, extent), 4),
               "requested_below_cut": int(req[:cut].sum()), "requested_kept": int(req.sum()),
               "requested_share_below_cut": round(float(req[:cut].sum()) / max(1, req.sum()), 4),
               "rays_with_samples_below_cut": int((req[:cut] > 0).sum()), "rays_with_samples_kept": int((req > 0).sum()),
               "composited_below_cut": int(cc[:cut].sum()), "batch": R, "progressive_chunk_end": st["progressive_chunk_end"],
               "march_first_pass_rays": st.get("march_first_pass_rays")}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
