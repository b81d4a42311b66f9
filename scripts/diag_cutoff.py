"""How many of the inferred pre-compaction samples the loss ever reads (development tool): per ray, the samples
the march requested (nreq, kept ones only) vs the samples composited before the transmittance cut-off
(ccount). Samples past the cut-off have network outputs nobody reads."""
import os, sys
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
done = 0
for w in (5, 25, 200, 800, 2000):
    tb.train_steps(w - done); done = w
    st = tb.stats()
    nreq, cc, ns = tb.ray_counts(1 << 18)
    kept = ns.astype(np.int64)  # numsteps after the loss: compacted count; use nreq for the march's requests
    tot_req = int(nreq.astype(np.int64).sum())
    tot_cc = int(cc.astype(np.int64).sum())
    has = nreq > 0
    # the first-pass position of the cut-off within each ray
    frac = cc[has].astype(np.float64) / nreq[has]
    q = np.percentile(nreq[has], [50, 90, 99, 100]) if has.any() else [0]
    print(f"step {w}: Npre {st['measured_batch_size_before_compaction']} n_kept~{min(tot_req, 1 << 22)} sum nreq {tot_req} "
          f"sum ccount {tot_cc} ({tot_cc / max(1, tot_req):.3f}) rays with samples {int(has.sum())} "
          f"nreq p50/p90/p99/max {q} ccount/nreq mean {frac.mean():.3f} compacted {st['measured_batch_size']}", flush=True)
    # samples a chunked (progressive) inference would evaluate: rounds of per-ray chunks [e_k, e_k+1) until the chunk
    # that holds the ray's last composited sample; launches = rounds with any active ray
    n, c = nreq[has].astype(np.int64), np.maximum(cc[has].astype(np.int64), 1)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"cutoff_{w}.npz"), nreq=n.astype(np.uint16), cc=c.astype(np.uint16),
                        ns=ns[has].astype(np.uint16))
    for sched in ((16,), (32,), (8, 32), (16, 64), (16, 48, 112), (8, 16, 32, 64)):
        ends = np.array(sched + (1 << 30,), np.int64)
        k = np.searchsorted(ends, c)  # first chunk end >= c
        inf = np.minimum(n, ends[k])
        act = [int((k >= j).sum()) for j in range(len(ends))]
        print(f"   chunks {sched}: inferred {int(inf.sum())} ({inf.sum() / max(1, tot_req):.3f}) active rays per round {act}", flush=True)
