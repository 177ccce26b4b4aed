"""Summarise tools/gpu_r4_subpmc.sh output (true 4:2:2 / 4:2:0 bench under rocprofv3: kernel stats
and PMC passes) into one committed profile JSON: per mode the bench line, the kernel's rocprof
stats row and the per-launch PMC means (FETCH_SIZE doubled as tools/pmc_summary.py does for the
traffic ratio).
Usage: python tools/sub_pmc_summary.py gpurun_out/r5sub profiles/r05_sub_pmc.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
KERN = {1: "k_mxs422", 2: "k_mxs420"}
BPP = {1: 7, 2: 6}
out = {}
for sr, kern in KERN.items():
    rec = {}
    with open(os.path.join(src, f"bench{sr}.json")) as f:
        rec["bench"] = json.loads(f.read().strip().splitlines()[-1])
    for path in glob.glob(os.path.join(src, f"stats{sr}", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if f"::{kern}(" in row["Name"]:
                rec["rocprof_stats"] = row
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(src, f"sr{sr}_p*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(path)):
            if f"::{kern}(" in row["Kernel_Name"] or row["Kernel_Name"].endswith(kern):
                per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for k, d in per.items():
            vals[k] += list(d.values())
    m = {k: sum(v) / len(v) for k, v in vals.items() if v}
    rec["pmc_mean_per_launch"] = m
    alg = 8 * 3840 * 2160 * BPP[sr]
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        traffic = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
        rec["traffic_bytes_per_launch"] = traffic
        rec["traffic_over_algorithmic"] = traffic / alg
    steps = 8 * 3840 * 2160 / 64 / 8        # 8-Y-block steps per launch
    rec["per_step"] = {k: round(m[k] / steps, 1) for k in m if k.startswith("SQ_INSTS")}
    if "SQ_WAVE_CYCLES" in m:
        rec["per_step"]["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 3)
    out[kern] = rec
    print(kern, rec["bench"]["roofline"]["frac"], rec.get("traffic_over_algorithmic"), rec["per_step"])
json.dump(out, open(dst, "w"), indent=1)
