"""Regenerate tests/golden/big_golden.json: BASELINE.json configs[3] and configs[4] at full size
(this container only; the GPU box never runs this).

configs[4] -- 16384x16384, sample_ratio 1 ("4:2:2", whose reference output is 4:4:4), q=50,
  splitmix seed 5 (SURVEY.md 8c generator G):
  * the REAL reference (oracle/_ref/ref_dump: preprocess_jpeg -> chroma_subsample -> dct ->
    quantise -> zig_zag compiled from /root/reference/src by `make -C oracle ref`) is run once
    on the whole frame written as a BMP (about 20 min, 12 GB).  Its output hash, per-channel
    hashes, per-stripe hashes (the 8 block-row stripes of an 8-GPU node) and the [3][8] bytes
    glibc really left in front of r_new/g_new/b_new (the x0 = -8 underflow of block-row 0,
    src/preprocess.c:127-129,159-160, after the file-buffer malloc/free of src/bitmap.c:113,151)
    are recorded.
  * REF_STOP_AFTER_PREPROCESS runs of the same harness record the real mmap-case underflow bytes
    of 4096^2 and 8192^2 frames in seconds.
configs[3] -- 64 x 3840x2160, 4:4:4, q=90, frame f = splitmix seed 1000 + f (bench.rank_plan's
  global batch): per-frame output hashes from the oracle restatement (oracle/cpu_ref.c, exact
  order, table cosines), which tests/test_oracle.py pins to the real reference at 4K.  One frame
  (seed 1000) is also run through the real reference and must agree.

Run:  python tests/golden/make_big_golden.py [--skip-16k]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402

OUT = os.path.join(HERE, "big_golden.json")


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stripe(nrows: int, parts: int, k: int):
    """jpgx.stripe: block-rows [r0, r1) of part k (the same split as the product's)."""
    base, extra = divmod(nrows, parts)
    r0 = k * base + min(k, extra)
    return r0, r0 + base + (1 if k < extra else 0)


def underflow_after_preprocess(rgb: np.ndarray, td: str) -> list:
    bmp = os.path.join(td, "u.bmp")
    O.write_bmp(bmp, rgb)
    n = rgb.shape[0] * rgb.shape[1]
    env = dict(os.environ, REF_WATCH_PIXELS=str(n), REF_STOP_AFTER_PREPROCESS="1")
    r = subprocess.run([os.path.join(O.REF_DIR, "ref_dump"), bmp, os.path.join(td, "x"), "50", "0"],
                       check=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                       text=True)
    seen = [l.split("=")[1] for l in r.stderr.split() if l.startswith("pre[")]
    os.remove(bmp)
    return [list(bytes.fromhex(s)) for s in seen[-3:]]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-16k", action="store_true")
    args = ap.parse_args()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "all", "ref"], check=True)
    g = json.load(open(OUT)) if os.path.exists(OUT) else {}
    g["generator"] = "tests/golden/make_big_golden.py"

    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        # mmap-case underflow bytes straight from glibc (preprocess only)
        g["mmap_underflow"] = {}
        for side in (4096, 8192):
            rgb = O.gen_splitmix(7, side, side)
            g["mmap_underflow"][str(side)] = underflow_after_preprocess(rgb, td)
            print(side, g["mmap_underflow"][str(side)], flush=True)
            del rgb

        # configs[3]: 64 x 4K q90, seeds 1000 + f
        W, H, Q = 3840, 2160, 90
        frames = []
        for f in range(64):
            rgb = O.gen_splitmix(1000 + f, W, H)
            out = O.blocks(rgb, Q, nthreads=os.cpu_count())
            frames.append({"seed": 1000 + f, "input_sha256": sha(rgb),
                           "coef_sha256": sha(out.astype("<i2"))})
            if f == 0:
                bmp = os.path.join(td, "f0.bmp")
                O.write_bmp(bmp, rgb)
                ref = O.ref_dump(bmp, Q)
                os.remove(bmp)
                assert np.array_equal(ref, out), "oracle != reference on frame 1000"
        g["batch64_4k_q90"] = {"W": W, "H": H, "quality": Q, "sample_ratio": 0,
                               "frames": frames, "reference_checked_frame": 1000}
        print("batch64 done", flush=True)

        if not args.skip_16k:
            W = H = 16384
            Q, SR, SEED = 50, 1, 5
            rgb = O.gen_splitmix(SEED, W, H)
            insha = sha(rgb)
            bmp = os.path.join(td, "big.bmp")
            O.write_bmp(bmp, rgb)
            del rgb
            t = time.time()
            outp = os.path.join(td, "big.bin")
            a, uf = O.ref_dump(bmp, Q, SR, tmp_out=outp, want_underflow=True)
            dt = time.time() - t
            os.remove(bmp)
            a16 = a.astype("<i2")
            assert np.array_equal(a16.astype(np.int32), a)
            del a
            bpr = W // 8
            st = []
            for k in range(8):
                r0, r1 = stripe(H // 8, 8, k)
                st.append({"rows": [r0, r1],
                           "coef_sha256": sha(a16[:, r0 * bpr:r1 * bpr])})
            g["frame16k_q50_sr1"] = {
                "W": W, "H": H, "quality": Q, "sample_ratio": SR, "seed": SEED,
                "input_sha256": insha, "underflow": uf.tolist(),
                "coef_sha256": sha(a16),
                "channel_sha256": [sha(a16[c]) for c in range(3)],
                "stripes8": st,
                "block_row0_sha256": sha(a16[:, :bpr]),
                "reference_seconds": round(dt, 1)}
            print("16k done", dt, flush=True)

    with open(OUT, "w") as f:
        json.dump(g, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
