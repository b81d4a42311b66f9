"""Summarise rocprofv3 counter_collection.csv files: per kernel (and grid size), mean counter value per
dispatch. --last N keeps only each kernel's last N dispatches (the diag_one.py launches after warm-up)."""
import argparse, csv, collections, glob
ap = argparse.ArgumentParser()
ap.add_argument("paths", nargs="+")
ap.add_argument("--last", type=int, default=0)
a = ap.parse_args()
for path in a.paths:
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        rows = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            rows[r["Kernel_Name"].split("(")[0][:60]].append(r)
        print(f)
        for k, rs in rows.items():
            ids = sorted({int(r["Dispatch_Id"]) for r in rs})
            if a.last: ids = ids[-a.last:]
            keep = set(ids)
            agg = collections.defaultdict(float)
            for r in rs:
                if int(r["Dispatch_Id"]) in keep: agg[r["Counter_Name"]] += float(r["Counter_Value"])
            print(f"  {k} dispatches={len(ids)} grid={rs[-1]['Grid_Size']}")
            for c, x in sorted(agg.items()): print(f"      {c:32s} {x / len(ids):16.4g}")
