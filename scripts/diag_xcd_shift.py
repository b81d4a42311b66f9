"""Diagnostic: does the training step depend on the workgroup -> XCD placement? One testbed trained alone as the
reference, then the same training with a no-op kernel of k workgroups before every kernel of the step
(neus_debug_set_xcd_shift: the round-robin placement of every launch moves by k XCDs). Per step: the compacted batch's
dL/doutput, the gradients and the parameters are compared bitwise with the reference.
Usage: python scripts/diag_xcd_shift.py [--steps 3] [--shifts 1,3,5] [--progressive 2] [--prepare 0]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--shifts", default="1,3,5")
    ap.add_argument("--progressive", type=int, default=2)
    ap.add_argument("--prepare", type=int, default=0)
    ap.add_argument("--batch", type=int, default=1 << 18)
    args = ap.parse_args()
    from neus2_amd import pyngp, scenes
    from neus2_amd._lib import check, lib
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    B = args.batch

    def make(shift):
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=B, fixed_rays_per_batch=B)
        if args.progressive >= 0:
            tb.set_progressive_inference(args.progressive)
        if args.prepare:
            tb.train_steps(args.prepare)
        check(lib().neus_debug_set_xcd_shift(tb.handle, C.c_uint32(shift)))
        return tb

    def run(tb):
        rec = []
        for _ in range(args.steps):
            tb.train_steps(1)
            dl = np.zeros((B, 16), np.uint16)
            check(lib().neus_debug_get_batch(tb.handle, None, C.c_void_p(dl.ctypes.data), None))
            rec.append({"dl": dl, "grads": tb.get_gradients().view(np.uint32), "params": tb.get_params().view(np.uint32)})
        return rec

    ref = run(make(0))
    for k in [int(v) for v in args.shifts.split(",")]:
        got = run(make(k))
        out = {"shift": k, "prepare": args.prepare, "progressive": args.progressive}
        for step, (a, b) in enumerate(zip(ref, got)):
            diff = {key: int((a[key] != b[key]).sum()) for key in a if not np.array_equal(a[key], b[key])}
            if diff:
                out["first_step"] = step + 1
                out["differs"] = diff
                if "dl" in diff:
                    out["dl_cols"] = [int(c) for c in np.nonzero((a["dl"] != b["dl"]).any(0))[0]]
                break
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
