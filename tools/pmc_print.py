"""Print median per-dispatch PMC counters of the transform kernel from gpurun_out/<dir>/p*/."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    per = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "k_xform" in r["Kernel_Name"] or "k_mx" in r["Kernel_Name"]:
                agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in agg.items():
            per[c].append(v)
    print(d)
    for c, v in sorted(per.items()):
        print(f"  {c:28s} {sorted(v)[len(v) // 2]:.4g}")
