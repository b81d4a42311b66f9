"""Diagnostic: does the bench-shape step read device memory it never wrote? A testbed on fresh allocations is the
reference; a second one is created after a "dirty" testbed (trained a few steps, then destroyed) so that its allocations
are likely to land on memory holding that testbed's data; a third, the same with every fresh allocation zero-filled
(NEUS_DBG_POISON). Per step the compacted batch's dL/doutput, the gradients and the parameters are compared bitwise. If
the recycled run differs and the zero-filled one does not, the allocation responsible is bisected (zero-filling a prefix
of the allocations, in creation order) and listed with its size (NEUS_DBG_ALLOC_LOG on stderr).
Usage: python scripts/diag_recycle.py [--steps 3] [--dirty 20] [--progressive 2]"""
import argparse
import ctypes as C
import gc
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B = 1 << 18


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dirty", type=int, default=20)
    ap.add_argument("--progressive", type=int, default=2)
    ap.add_argument("--max-allocs", type=int, default=1 << 12)
    args = ap.parse_args()
    from neus2_amd import pyngp, scenes
    from neus2_amd._lib import check, lib
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))

    def make():
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=B, fixed_rays_per_batch=B)
        if args.progressive >= 0:
            tb.set_progressive_inference(args.progressive)
        return tb

    def run(poison=None):
        if poison is None:
            os.environ.pop("NEUS_DBG_POISON", None)
        else:
            os.environ["NEUS_DBG_POISON"] = poison
        tb = make()
        rec = []
        for _ in range(args.steps):
            tb.train_steps(1)
            dl = np.zeros((B, 16), np.uint16)
            check(lib().neus_debug_get_batch(tb.handle, None, C.c_void_p(dl.ctypes.data), None))
            rec.append({"dl": dl, "grads": tb.get_gradients().view(np.uint32), "params": tb.get_params().view(np.uint32)})
        os.environ.pop("NEUS_DBG_POISON", None)
        del tb
        gc.collect()
        return rec

    def dirty():
        tb = make()
        tb.train_steps(args.dirty)
        tb.synchronize()
        del tb
        gc.collect()

    def diff(a, b):
        for step, (x, y) in enumerate(zip(a, b)):
            d = {k: int((x[k] != y[k]).sum()) for k in x if not np.array_equal(x[k], y[k])}
            if d:
                return {"first_step": step + 1, "differs": d}
        return None

    ref = run()
    dirty()
    r1 = run()
    res = {"case": "recycled", "diff": diff(ref, r1)}
    print(json.dumps(res), flush=True)
    dirty()
    r2 = run("0")
    print(json.dumps({"case": "recycled_zero_filled", "diff": diff(ref, r2)}), flush=True)
    if res["diff"] is None:
        return
    # smallest hi such that zero-filling allocations [0, hi) restores the fresh run
    lo, hi = 0, args.max_allocs
    while hi - lo > 1:
        mid = (lo + hi) // 2
        dirty()
        ok = diff(ref, run(f"0:0:{mid}")) is None
        print(json.dumps({"bisect": [0, mid], "fixed": ok}), flush=True)
        if ok:
            hi = mid
        else:
            lo = mid
    k = hi - 1
    dirty()
    alone = diff(ref, run(f"0:{k}:{k + 1}")) is None
    print(json.dumps({"culprit_alloc": k, "zero_fill_alone_fixes": alone}), flush=True)
    os.environ["NEUS_DBG_ALLOC_LOG"] = "1"
    tb = make()
    del tb
    os.environ.pop("NEUS_DBG_ALLOC_LOG", None)


if __name__ == "__main__":
    main()
