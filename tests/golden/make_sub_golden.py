"""Add true 4:2:2 / 4:2:0 (the JPGX_FLAG_SUBSAMPLE extension) 4K goldens to
tests/golden/big_golden.json: 3840x2160, q=75, splitmix seeds 1000..1003, output hashed as the
product lays it out (Y [nb][64] | Cb [nbc][64] | Cr [nbc][64], int16 little-endian).  Y is the
oracle's 4:4:4 luma (the reference's own Y, x0 = -8 quirk included), chroma is
oracle.chroma_sub (cpu_ref.h's definition: level-shifted Cb/Cr averaged over the pixel pair /
2x2 quad, then the exact DCT and quantisation).  The reference has no behaviour here (its
subsample_422/420 only print, src/downsample.c:24-32), so these pin the extension to the oracle
definition only.

Run (this container): python tests/golden/make_sub_golden.py"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.join(HERE, "big_golden.json")


def main():
    W, H, Q = 3840, 2160, 75
    g = json.load(open(OUT))
    ent = {"W": W, "H": H, "quality": Q, "seeds": [1000 + f for f in range(4)],
           "generator": "tests/golden/make_sub_golden.py"}
    for sr in (1, 2):
        hs = []
        for seed in ent["seeds"]:
            rgb = O.gen_splitmix(seed, W, H)
            y = O.blocks(rgb, Q, sr, nthreads=os.cpu_count())[0]
            c = O.chroma_sub(rgb, Q, sr).reshape(-1, 64)
            out = np.concatenate([y, c]).astype("<i2")
            hs.append(hashlib.sha256(out.tobytes()).hexdigest())
            print(sr, seed, hs[-1], flush=True)
        ent[f"sr{sr}_coef_sha256"] = hs
    g["sub_4k_q75"] = ent
    with open(OUT, "w") as f:
        json.dump(g, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
