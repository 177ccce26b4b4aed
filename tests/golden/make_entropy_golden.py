"""Regenerate tests/golden/entropy_stats.json from the REAL reference (this container only).

oracle/_ref/ref_dump (oracle/ref_harness.c, the reference's stage sources compiled in place by
`make -C oracle ref`) runs preprocess -> ... -> zig_zag -> dpcm and then the terminating first
half of huffman_encode (src/huffman.c:23-44: initialize_huffman and the per-block
calculate_freq_block_DC / _AC calls; construct_huffman_table never terminates and is not
called).  Recorded per case: the four freq[257] tables (lum_DC, lum_AC, chrom_DC, chrom_AC)
and the sha256 of the post-dpcm DC values (int32, Y then Cb then Cr).  Nothing here is computed
by the oracle restatement; tests/test_entropy.py checks it against these vectors.

Run:  python tests/golden/make_entropy_golden.py      (about 20 s)
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as O  # noqa: E402  (file I/O helpers only)


def run(bmp: str, q: int):
    with tempfile.TemporaryDirectory() as td:
        out, st = os.path.join(td, "o.bin"), os.path.join(td, "s.bin")
        subprocess.run([os.path.join(O.REF_DIR, "ref_dump"), bmp, out, str(q), "0", "1", st],
                       check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        d = np.fromfile(out, np.int32).reshape(3, -1, 64)[:, :, 0].reshape(-1)
        h = np.fromfile(st, np.int32).reshape(4, 257)
    return hashlib.sha256(d.astype("<i4").tobytes()).hexdigest(), h.tolist()


def main() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    cases = []
    for name in ("cam", "tiger"):
        for q in (50, 90):
            dsha, h = run(os.path.join(HERE, "images", f"{name}.bmp"), q)
            cases.append({"image": name, "q": q, "dc_sha256": dsha, "hist": h})
    with tempfile.TemporaryDirectory() as td:
        for kind, W, H, seed, q in (("G", 512, 512, 1, 50), ("G", 512, 512, 1, 90),
                                    ("T", 512, 512, 0, 50), ("G", 64, 48, 15, 25),
                                    ("G", 1920, 1080, 2, 90)):
            rgb = O.gen_splitmix(seed, W, H) if kind == "G" else O.gen_tie(W, H)
            bmp = os.path.join(td, "f.bmp")
            O.write_bmp(bmp, rgb)
            dsha, h = run(bmp, q)
            cases.append({"kind": kind, "W": W, "H": H, "seed": seed, "q": q,
                          "dc_sha256": dsha, "hist": h})
            print(kind, W, H, q, "done", flush=True)
    with open(os.path.join(HERE, "entropy_stats.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_entropy_golden.py (real reference binaries)",
                   "cases": cases}, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
