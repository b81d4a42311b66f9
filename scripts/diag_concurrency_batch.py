"""Diagnostic: where two concurrently trained testbeds leave a testbed trained alone (scripts/diag_concurrency.py found
the variance gradient of step 1 differing with progressive inference forced on). Per step of every testbed: the
compacted batch (coords, dL/doutput), per-ray losses and counts, gradients; the first differing step is dissected.
Usage: python scripts/diag_concurrency_batch.py [--steps 3] [--pairs 3] [--progressive 2]"""
import argparse
import ctypes as C
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--progressive", type=int, default=2)
    ap.add_argument("--buffers", type=int, default=1)
    args = ap.parse_args()
    from neus2_amd import pyngp, scenes
    from neus2_amd._lib import check, lib
    sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
    B, R = args.batch, args.batch

    def make():
        tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
        tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
        tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=B, fixed_rays_per_batch=R)
        if args.progressive >= 0:
            tb.set_progressive_inference(args.progressive)
        return tb

    def snap(tb):
        co = np.zeros((B, 7), np.float32)
        dl = np.zeros((B, 16), np.uint16)
        lo = np.zeros(1 << 18, np.float32)
        check(lib().neus_debug_get_batch(tb.handle, C.c_void_p(co.ctypes.data), C.c_void_p(dl.ctypes.data), C.c_void_p(lo.ctypes.data)))
        nreq, cc, ns = tb.ray_counts(R)
        out = {"coords": co, "dl": dl, "loss": lo, "nreq": nreq, "cc": cc, "ns": ns, "grads": tb.get_gradients(), "params": tb.get_params()}
        if os.environ.get("NEUS_DBG_LOSS_VALS") == "1":
            dv = np.zeros((B, 8), np.float32)
            check(lib().neus_debug_get_buffer(tb.handle, C.c_int(16), C.c_uint64(0), C.c_uint64(B * 32), C.c_void_p(dv.ctypes.data)))
            out["dbg_vals"] = dv
        rdl = np.zeros((B, 16), np.uint16)
        check(lib().neus_debug_replay_loss_grad(tb.handle, C.c_void_p(rdl.ctypes.data)))
        out["replay_dl"] = rdl
        if os.environ.get("NEUS_DBG_LOSS_REPLAY") == "1":
            idl = np.zeros((B, 16), np.uint16)
            check(lib().neus_debug_get_buffer(tb.handle, C.c_int(15), C.c_uint64(0), C.c_uint64(B * 32), C.c_void_p(idl.ctypes.data)))
            out["instep_replay_dl"] = idl
            names = ["sa", "ekt", "ck4", "cke", "racc", "rgr", "rT", "rek", "ccount", "net_out", "pcoords", "base", "numsteps", "cmap", "nreq"]
            for k, nm in enumerate(names):
                fin = np.zeros(1, np.uint8)
                # sizes: read the final buffer and its in-step snapshot (same size)
                sizes = {"sa": 16, "ekt": 4, "ck4": 16, "cke": 4, "racc": 16, "rgr": 16, "rT": 4, "rek": 4, "ccount": 4, "net_out": 32,
                         "pcoords": 28, "base": 4, "numsteps": 8, "cmap": 4, "nreq": 4}
                M = 16 * B
                n_el = {"sa": M, "ekt": M, "ck4": M // 8 + 1, "cke": M // 8 + 1, "racc": 1 << 18, "rgr": 1 << 18, "rT": 1 << 18, "rek": 1 << 18,
                        "ccount": 1 << 18, "net_out": M, "pcoords": M, "base": 1 << 18, "numsteps": 1 << 18, "cmap": B, "nreq": 1 << 18}[nm]
                nb = n_el * sizes[nm]
                fin = np.zeros(nb, np.uint8)
                snp = np.zeros(nb, np.uint8)
                check(lib().neus_debug_get_buffer(tb.handle, C.c_int(k), C.c_uint64(0), C.c_uint64(nb), C.c_void_p(fin.ctypes.data)))
                check(lib().neus_debug_get_buffer(tb.handle, C.c_int(20 + k), C.c_uint64(0), C.c_uint64(nb), C.c_void_p(snp.ctypes.data)))
                d = np.nonzero(fin != snp)[0]
                out["snapdiff_" + nm] = (int(d.size), int(d[0]) if d.size else -1)
        if args.buffers:
            M = 16 * B
            for name, bid, nbytes, dt in (("sa", 0, M * 16, np.float32), ("ekt", 1, M * 4, np.float32), ("ck4", 2, (M // 8 + 1) * 16, np.float32),
                                          ("cke", 3, (M // 8 + 1) * 4, np.float32), ("racc", 4, (1 << 18) * 16, np.float32),
                                          ("rgr", 5, (1 << 18) * 16, np.float32), ("rT", 6, (1 << 18) * 4, np.float32), ("ccount", 8, (1 << 18) * 4, np.uint32),
                                          ("net_out", 9, M * 32, np.uint16), ("pcoords", 10, M * 28, np.float32), ("base", 11, (1 << 18) * 4, np.uint32),
                                          ("numsteps", 12, (1 << 18) * 8, np.uint32), ("cmap", 13, B * 4, np.uint32)):
                a = np.zeros(nbytes // np.dtype(dt).itemsize, dt)
                check(lib().neus_debug_get_buffer(tb.handle, C.c_int(bid), C.c_uint64(0), C.c_uint64(nbytes), C.c_void_p(a.ctypes.data)))
                out["buf_" + name] = a
        return out

    def run(tb, rec):
        for _ in range(args.steps):
            tb.train_steps(1)
            rec.append(snap(tb))

    ref = make()
    rr = []
    run(ref, rr)
    del ref
    lay = None
    for trial in range(args.pairs):
        pair = [make(), make()]
        lay = pair[0].layout()
        recs = [[], []]
        ts = [threading.Thread(target=run, args=(pair[i], recs[i])) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        del pair
        for i in range(2):
            out = {"trial": trial, "testbed": i}
            for k, (a, b) in enumerate(zip(rr, recs[i])):
                diff = [key for key in a if not key.startswith("snapdiff_") and key != "dbg_vals" and not np.array_equal(a[key].view(np.uint8), b[key].view(np.uint8))]
                if not diff:
                    continue
                out["step"] = k + 1
                out["differs"] = diff
                if "dl" in diff:
                    rows = np.nonzero((a["dl"] != b["dl"]).any(1))[0]
                    cols = np.nonzero((a["dl"] != b["dl"]).any(0))[0]
                    out["dl_rows"] = [int(x) for x in rows[:20]]
                    out["dl_n_rows"] = int(rows.size)
                    out["dl_cols"] = [int(x) for x in cols]
                    r0 = rows[0]
                    lanes = np.bincount(rows % 64, minlength=64)
                    out["dl_row_lanes"] = {int(k): int(v) for k, v in enumerate(lanes) if v}
                    if "dbg_vals" in a:
                        names = ["inv_s", "dloss_dalpha", "dadem", "dem_dinvs", "dadpe", "dpe_dinvs", "dloss_dinvs", "dloss_dvar"]
                        va, vb = a["dbg_vals"][rows], b["dbg_vals"][rows]
                        out["vals_differ_in_dl_rows"] = {nm: int((va[:, k].view(np.uint32) != vb[:, k].view(np.uint32)).sum()) for k, nm in enumerate(names)}
                        allr = np.nonzero((a["dbg_vals"].view(np.uint32) != b["dbg_vals"].view(np.uint32)).any(1))[0]
                        out["vals_rows_differ_total"] = int(allr.size)
                        out["vals_rows_lanes"] = {int(k): int(v) for k, v in enumerate(np.bincount(allr % 64, minlength=64)) if v}
                        r0_ = rows[0]
                        out["vals_first"] = {"ref": a["dbg_vals"][r0_].tolist(), "got": b["dbg_vals"][r0_].tolist()}
                    out["dl_first"] = {"ref": a["dl"][r0].view(np.float16).astype(float).tolist(), "got": b["dl"][r0].view(np.float16).astype(float).tolist(),
                                       "coords": a["coords"][r0].tolist()}
                for key in ("loss", "cc", "nreq", "ns"):
                    if key in diff:
                        rays = np.nonzero(a[key] != b[key])[0]
                        out[f"{key}_rays"] = [int(x) for x in rays[:20]]
                        out[f"{key}_n"] = int(rays.size)
                if "dl" in diff and args.buffers:
                    row = int(np.nonzero((a["dl"] != b["dl"]).any(1))[0][0])
                    r = int(a["buf_cmap"][row])
                    rb, ns_r, cb = int(a["buf_base"][r]), int(a["buf_numsteps"][2 * r]), int(a["buf_numsteps"][2 * r + 1])
                    out["ray"] = {"r": r, "rb": rb, "ns(compacted)": ns_r, "cb": cb, "row": row, "cc": int(a["cc"][r]), "nreq": int(a["nreq"][r])}
                    n_s = int(a["nreq"][r])
                    per_ray = {k: (a["buf_" + k][4 * r:4 * r + 4] if k in ("racc", "rgr") else a["buf_" + k][r:r + 1]) for k in ("racc", "rgr", "rT", "ccount")}
                    per_ray_b = {k: (b["buf_" + k][4 * r:4 * r + 4] if k in ("racc", "rgr") else b["buf_" + k][r:r + 1]) for k in ("racc", "rgr", "rT", "ccount")}
                    out["ray_state_differs"] = [k for k in per_ray if not np.array_equal(per_ray[k].view(np.uint8), per_ray_b[k].view(np.uint8))]
                    sl = slice(rb, rb + n_s)
                    for k, w in (("sa", 4), ("ekt", 1), ("net_out", 16), ("pcoords", 7)):
                        x, y = a["buf_" + k].reshape(-1, w)[sl], b["buf_" + k].reshape(-1, w)[sl]
                        d = np.nonzero((x.view(np.uint8).reshape(len(x), -1) != y.view(np.uint8).reshape(len(y), -1)).any(1))[0]
                        out[f"sample_{k}_differs"] = [int(v) for v in d[:12]]
                    ck = slice(rb // 8, (rb + n_s) // 8 + 1)
                    x, y = a["buf_ck4"].reshape(-1, 4)[ck], b["buf_ck4"].reshape(-1, 4)[ck]
                    d = np.nonzero((x != y).any(1))[0]
                    out["ck4_slots_differ"] = [int(v) + rb // 8 for v in d[:12]]
                    if d.size:
                        q = int(d[0]) + rb // 8
                        out["ck4_first"] = {"slot": q, "ref": a["buf_ck4"].reshape(-1, 4)[q].tolist(), "got": b["buf_ck4"].reshape(-1, 4)[q].tolist(),
                                            "slot_sample": 8 * q}
                if "grads" in diff:
                    g = np.nonzero(a["grads"].view(np.uint32) != b["grads"].view(np.uint32))[0]
                    out["grad_idx_first"] = [int(x) for x in g[:10]]
                    out["grad_n"] = int(g.size)
                    out["var_off"] = lay["variance_offset"]
                    out["grad_var"] = [float(a["grads"][lay["variance_offset"]]), float(b["grads"][lay["variance_offset"]])]
                break
            for key, rec in (("ref", rr), ("got", recs[i])):
                last = rec[0]
                out[f"{key}_replay_equals_step"] = bool(np.array_equal(last["replay_dl"], last["dl"]))
            out["got_replay_equals_ref_step"] = bool(np.array_equal(recs[i][0]["replay_dl"], rr[0]["dl"]))
            if "instep_replay_dl" in recs[i][0]:
                out["got_instep_replay_equals_got_step"] = bool(np.array_equal(recs[i][0]["instep_replay_dl"], recs[i][0]["dl"]))
                out["got_instep_replay_equals_ref"] = bool(np.array_equal(recs[i][0]["instep_replay_dl"], rr[0]["dl"]))
                out["snapdiff_got"] = {k[9:]: v for k, v in recs[i][0].items() if k.startswith("snapdiff_") and v[0]}
                out["snapdiff_ref"] = {k[9:]: v for k, v in rr[0].items() if k.startswith("snapdiff_") and v[0]}
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
