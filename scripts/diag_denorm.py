"""Diagnostic: is fp32 denormal arithmetic on the MI355X the same in every lane and every launch, alone and while other
work shares the GPU? The concurrent-testbed divergence (scripts/diag_concurrency*.py) changed only dL/doutput column 7
(the variance term, which multiplies exp(-sdf * inv_s) - a denormal for sdf * inv_s in (87, 103) - by inv_s * 10) and
only in lanes 48-63 of a wave. neus_debug_denorm_probe evaluates denormal-producing expressions (det_expf, products,
ldexpf) per lane and compares every launch's bits with the CPU's, and reads each wave's MODE register.
Usage: python scripts/diag_denorm.py [--launches 50] [--train-steps 300] [--testbeds 2]"""
import argparse
import ctypes as C
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B = 1 << 18
NAMES = ["launches", "mismatches", "row0", "row1", "row2", "row3", "flushed", "modes", "mode0", "mode_other"]


def probe(n, launches):
    from neus2_amd._lib import check, lib
    st = np.zeros(10, np.uint64)
    check(lib().neus_debug_denorm_probe(C.c_int(0), C.c_uint32(n), C.c_uint32(launches), C.c_void_p(st.ctypes.data)))
    return {k: (hex(int(v)) if k.startswith("mode") and k != "modes" else int(v)) for k, v in zip(NAMES, st)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--train-steps", type=int, default=300)
    ap.add_argument("--testbeds", type=int, default=2)
    args = ap.parse_args()
    print(json.dumps({"case": "alone", **probe(args.n, args.launches)}), flush=True)
    from neus2_amd import pyngp, scenes
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    tbs = []
    for _ in range(args.testbeds):
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=B, fixed_rays_per_batch=B)
        tb.set_progressive_inference(2)
        tbs.append(tb)
    done = threading.Event()

    def train(tb):
        tb.train_steps(args.train_steps)
        tb.synchronize()

    ts = [threading.Thread(target=train, args=(tb,)) for tb in tbs]
    for t in ts:
        t.start()
    k = 0
    while any(t.is_alive() for t in ts) and k < 40:
        print(json.dumps({"case": f"during_training_{args.testbeds}", "round": k, **probe(args.n, max(1, args.launches // 10))}), flush=True)
        k += 1
    for t in ts:
        t.join()
    done.set()
    print(json.dumps({"case": "after", **probe(args.n, args.launches)}), flush=True)


if __name__ == "__main__":
    main()
