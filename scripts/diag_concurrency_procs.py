"""Diagnostic: the concurrent-testbed divergence (scripts/diag_concurrency_batch.py) with the two concurrent testbeds in
separate PROCESSES (separate address spaces) instead of two threads of one process, and with the two in-process
testbeds running different progressive modes. Prints, per trial, whether each concurrent testbed's first-step dL/doutput
equals the one of a testbed trained alone.
Usage: python scripts/diag_concurrency_procs.py --trials 4            (processes)
       python scripts/diag_concurrency_procs.py --threads --mode-b 0   (threads; testbed b one-pass)"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
B = 1 << 18


def make(sc, mode):
    from neus2_amd import pyngp
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=B, fixed_rays_per_batch=B)
    tb.set_progressive_inference(mode)
    return tb


def dl_of(tb):
    from neus2_amd._lib import check, lib
    dl = np.zeros((B, 16), np.uint16)
    check(lib().neus_debug_get_batch(tb.handle, None, C.c_void_p(dl.ctypes.data), None))
    return dl


def scene():
    from neus2_amd import scenes
    return scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))


def worker(out, mode, go_file):
    import time
    sc = scene()
    tb = make(sc, mode)
    tb.synchronize()
    open(go_file + ".ready." + str(os.getpid()), "w").close()
    while not os.path.exists(go_file):
        time.sleep(0.001)
    tb.train_steps(1)
    np.save(out, dl_of(tb))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--threads", action="store_true")
    ap.add_argument("--mode-a", type=int, default=2)
    ap.add_argument("--mode-b", type=int, default=2)
    ap.add_argument("--worker", nargs=3)
    args = ap.parse_args()
    if args.worker:
        worker(args.worker[0], int(args.worker[1]), args.worker[2])
        return
    sc = scene()
    ref = make(sc, args.mode_a)
    ref.train_steps(1)
    want = dl_of(ref)
    del ref
    tmp = os.path.join(ROOT, "gpurun_out", "conc_tmp")
    os.makedirs(tmp, exist_ok=True)
    for trial in range(args.trials):
        if args.threads:
            tbs = [make(sc, args.mode_a), make(sc, args.mode_b)]
            ts = [threading.Thread(target=lambda tb=tb: tb.train_steps(1)) for tb in tbs]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            got = [dl_of(tbs[0])]
            del tbs
        else:
            go = os.path.join(tmp, f"go{trial}")
            outs = [os.path.join(tmp, f"t{trial}_{r}.npy") for r in range(2)]
            ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", outs[r], str(args.mode_a if r == 0 else args.mode_b), go])
                  for r in range(2)]
            import time
            t0 = time.time()
            while len([f for f in os.listdir(tmp) if f.startswith(f"go{trial}.ready.")]) < 2 and time.time() - t0 < 120:
                time.sleep(0.01)
            open(go, "w").close()
            for p in ps:
                p.wait(timeout=180)
            got = [np.load(outs[0])] + ([np.load(outs[1])] if args.mode_b == args.mode_a else [])
            for f in outs + [go] + [os.path.join(tmp, f) for f in os.listdir(tmp) if f.startswith(f"go{trial}.ready.")]:
                if os.path.exists(f):
                    os.remove(f)
        res = {"trial": trial, "threads": args.threads, "mode_a": args.mode_a, "mode_b": args.mode_b,
               "equal": [bool(np.array_equal(g, want)) for g in got], "rows_differing": [int((g != want).any(1).sum()) for g in got]}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
