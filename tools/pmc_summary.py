"""Summarise rocprofv3 output (tools/gpu_check.sh kernel-trace stats + tools/gpu_prof.sh PMC
passes) for k_xform into a committed profile JSON.

  python tools/pmc_summary.py gpurun_out profiles/r02_k_mx_pmc.json [k_mx|k_xform]

HBM traffic per launch follows MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and
WRITE_SIZE come from separate passes, are reported in KiB, and on gfx950 FETCH_SIZE counts half
of the bytes of wide coalesced streaming reads (so it is doubled).  The kernel source hash is
stored so bench.py only quotes the traffic figure for the kernel it was measured on."""
import csv
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "csrc")
KSRCS = {"k_mx": ("jpgx_mx.hip", "jpgx_internal.h", "xform_math.h", "jx_consts.h"),
         "k_mxs": ("jpgx_mx.hip", "jpgx_internal.h", "xform_math.h", "jx_consts.h"),
         "k_xform": ("jpgx_kernels.hip", "jpgx_internal.h", "xform_math.h", "jx_consts.h")}
BYTES_PER_LAUNCH = 8 * 3840 * 2160 * 9          # bench.py workload, 9 B/px algorithmic


def kernel_source_sha(kernel="k_mx"):
    """sha256 over the device sources the kernel is built from."""
    h = hashlib.sha256()
    for name in KSRCS[kernel]:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def is_kernel(name, kernel):
    """name (mangled `..15k_mxsE..` or demangled `..::k_mxs(..`) is exactly `kernel`, not a
    longer name that starts with it (k_mx vs k_mxs / k_mx422)"""
    return re.search(r"(?<![A-Za-z_])%s(?=[(E<]|$)" % re.escape(kernel), name) is not None


def counters(path, kernel="k_xform"):
    """{counter: [per-dispatch values]} for dispatches of `kernel` (summed over dimensions)."""
    per = defaultdict(lambda: defaultdict(float))
    with open(path) as f:
        for row in csv.DictReader(f):
            if not is_kernel(row["Kernel_Name"], kernel):
                continue
            per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: [v[d] for d in sorted(v, key=int)] for k, v in per.items()}


def trace_ms(path, kernel="k_xform"):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if is_kernel(row["Kernel_Name"], kernel):
                out.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    return out


def mean(x):
    return sum(x) / len(x) if x else None


def main(src, dst, kernel="k_xform"):
    pmc = {}
    for p in sorted(os.listdir(os.path.join(src, "pmc"))):
        f = os.path.join(src, "pmc", p, "run_counter_collection.csv")
        if os.path.exists(f):
            for k, v in counters(f, kernel).items():
                pmc[k] = mean(v)
    res = {"kernel": kernel, "kernel_source_sha256": kernel_source_sha(kernel),
           "workload": "8 x 3840x2160 RGB, q=90 (bench.py)",
           "algorithmic_bytes_per_launch": BYTES_PER_LAUNCH, "pmc_mean_per_launch": pmc}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        rd = pmc["FETCH_SIZE"] * 1024 * 2          # KiB, x2 gfx950 wide-read correction
        wr = pmc["WRITE_SIZE"] * 1024
        res["hbm_read_bytes"] = rd
        res["hbm_write_bytes"] = wr
        res["traffic_bytes_per_launch"] = rd + wr
        res["traffic_over_algorithmic"] = (rd + wr) / BYTES_PER_LAUNCH
    for stats in ("prof/run_kernel_stats.csv",):
        f = os.path.join(src, stats)
        if os.path.exists(f):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if is_kernel(row["Name"], kernel):
                        res["rocprof_stats"] = {k: row[k] for k in row}
    tr = os.path.join(src, "prof", "run_kernel_trace.csv")
    if os.path.exists(tr):
        ms = trace_ms(tr, kernel)
        res["trace_mean_ms"] = mean(ms)
        res["trace_launches"] = len(ms)
    for name in ("bench.json", "prof_bench.json"):    # bench lines of the same box session
        f = os.path.join(src, name)
        if os.path.exists(f) and os.path.getsize(f):
            with open(f) as fh:
                res["session_" + name.replace(".json", "")] = json.loads(fh.read().splitlines()[-1])
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in res if k != "pmc_mean_per_launch"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
