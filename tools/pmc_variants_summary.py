"""Per-launch counter means of one kernel (default k_xform) from tools/pmc_variants.sh-style output
(<root>/<variant>/g<i>/...), with derived rates.
Usage: python tools/pmc_variants_summary.py gpurun_out/pmcv [kernel]"""
import csv, glob, os, re, sys
from collections import defaultdict

root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_xform"
KRE = re.compile(r"(?<![A-Za-z0-9_])%s(?![A-Za-z0-9_])" % kern)
for vdir in sorted(glob.glob(os.path.join(root, "*"))):
    vals = defaultdict(list)
    durs = []
    for f in glob.glob(os.path.join(vdir, "g*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if KRE.search(row["Kernel_Name"]):
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for k, d in per.items():
            vals[k] += list(d.values())
    for f in glob.glob(os.path.join(vdir, "g*", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if KRE.search(row["Kernel_Name"]):
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    m = {k: sum(v) / len(v) for k, v in vals.items() if v}
    us = sum(durs) / len(durs) if durs else float("nan")
    print(f"== {os.path.basename(vdir)}: {kern} {us:.1f} us (mean of {len(durs)} traced launches)")
    for k in sorted(m):
        print(f"   {k:24s} {m[k]:16.0f}")
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                print(f"   {k}/WAVE_CYCLES = {m[k] / wc:.3f}")
    if "GRBM_GUI_ACTIVE" in m and durs:
        print(f"   GRBM_GUI_ACTIVE / us = {m['GRBM_GUI_ACTIVE'] / us:.0f} (per-us, summed over XCDs?)")
