"""Turn the per-kernel PMC table of scripts/gpu_traffic.sh (pmc_table.py output) into profiles/traffic.json
entries: memory-side bytes per launch, corrected as MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE
tallies 128-B requests at 64 B, so reads are recomputed from the request-size breakdown; WRITE_SIZE is KB).
Usage: traffic_json.py TABLE LEVELS [--commit SHA] [--only-named] [--name KERNEL=KEY] [--out profiles/traffic.json]"""
import argparse
import json
import os
import re

NAMES = {"k_nerf_infer": "inference", "k_march": "march", "k_grid_encode": "train_encode", "k_loss_alpha": "loss_alpha",
         "k_mlp_train_rgb": "mlp_train_rgb", "k_mlp_train_density": "mlp_train_density", "k_march_write": "march_write",
         "k_scatter_bin_r": "scatter_bin", "k_scatter_accum_r": "scatter_accum", "k_adam_ema": "adam_ema",
         "k_mlp_grad_reduce": "mlp_grad_reduce"}


def parse(path, names=NAMES):
    cur, out = None, {}
    for line in open(path):
        m = re.match(r"\s+(\S.*?) dispatches=\d+ grid=\d+", line)
        if m:
            name = m.group(1)
            # k_march is the march itself: the templated k_march<...> or the balanced k_march_bal (the default), not
            # k_march_numsteps / k_march_write / k_march_scan
            # (names come mangled or demangled: "neus::k_march_bal", "void neus::k_scatter_bin_r<512>")
            cur = next((v for k, v in names.items() if (re.search(r"(^|::)k_march(<|_bal\b)", name) if k == "k_march" else k in name)), None)
            continue
        m = re.match(r"\s+(\w+)\s+([-+0-9.eE]+)$", line)
        if m and cur:
            out.setdefault(cur, {})[m.group(1)] = float(m.group(2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("table")
    ap.add_argument("levels", type=int)
    ap.add_argument("--commit", default="")
    # kernel=key overrides of the traffic.json key (e.g. k_nerf_infer=inference_step for the training step's own rounds)
    ap.add_argument("--name", action="append", default=[])
    # only the --name overrides (the table's other kernels and template variants are left out of the file)
    ap.add_argument("--only-named", action="store_true")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json"))
    a = ap.parse_args()
    try:
        db = json.load(open(a.out))
    except (OSError, ValueError):
        db = {}
    names = {}
    for kv in a.name:  # overrides first: the first key contained in a kernel's name wins
        k, v = kv.split("=", 1)
        names[k] = v
    if not a.only_named:
        for k, v in NAMES.items():
            names.setdefault(k, v)
    for k, c in parse(a.table, names).items():
        if "TCC_EA0_RDREQ_sum" not in c or "WRITE_SIZE" not in c:
            continue
        r128, r32 = c.get("TCC_EA0_RDREQ_128B_sum", 0.0), c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        reads = 128 * r128 + 32 * r32 + 64 * (c["TCC_EA0_RDREQ_sum"] - r128 - r32)
        writes = c["WRITE_SIZE"] * 1024
        db[f"{k}@L{a.levels}"] = {"bytes_per_launch": reads + writes, "read_bytes": reads, "write_bytes": writes,
                                  "fetch_size_kb": c.get("FETCH_SIZE"), "tcc_hit": c.get("TCC_HIT_sum"), "tcc_miss": c.get("TCC_MISS_sum"),
                                  "commit": a.commit, "source": os.path.basename(a.table)}
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
