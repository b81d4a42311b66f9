"""Summarise rocprofv3 counter_collection.csv files: per kernel (and grid size), mean counter value per dispatch."""
import csv, collections, glob, sys
for path in sys.argv[1:]:
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0][:60], r["Grid_Size"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
        print(f)
        for k, v in agg.items():
            n = len(disp[k])
            print(f"  {k[0]} grid={k[1]} dispatches={n}")
            for c, x in sorted(v.items()): print(f"      {c:28s} {x / n:16.4g}")
