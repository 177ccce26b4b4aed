"""Per-step PMC counters of tools/kpmc.sh runs: python tools/kpmc_summary.py gpurun_out/DIR [KERNEL]
(KERNEL default k_mxs; steps per launch = 8 x 4K frames / 8 blocks = 129,600)."""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import counters, mean  # noqa: E402

STEPS = 8 * 480 * 270 // 8


def main(d, kernel="k_mxs"):
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        tag = os.path.relpath(f, d).split(os.sep)[0]
        for k, v in sorted(counters(f, kernel).items()):
            print(f"{tag:50s} {k:28s} per launch {mean(v):14.1f}  per step {mean(v) / STEPS:9.2f}  n={len(v)}")


if __name__ == "__main__":
    main(*sys.argv[1:])
