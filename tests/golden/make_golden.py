"""Regenerate tests/golden/golden.json from the REAL reference (this container only).

The reference is compiled in place from /root/reference/src by `make -C oracle ref`
(oracle/_ref/ref_dump, a driver around preprocess_jpeg -> chroma_subsample -> dct ->
quantise -> zig_zag [-> dpcm], src/jpg_encode.c:32-47) and its own test binary
(oracle/_ref/jpg_kat = the reference's main() -> test_dct(), src/jpg_driver.c:21-150).
Every expected output below comes from running those binaries; nothing is computed by the
oracle restatement, which the tests then check against these vectors.

Fixture data committed alongside: images/cam.bmp and images/tiger.bmp are the reference's
bundled sample images (src/images/), kept as input data.

Run:  python tests/golden/make_golden.py        (about 2 minutes; 4K frames dominate)
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
import oracle as O  # noqa: E402  (test infrastructure: only used for file I/O helpers here)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def coef_sha(a: np.ndarray) -> str:
    return sha(a.astype("<i2"))


def main() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    g: dict = {"generator": "tests/golden/make_golden.py (real reference binaries)"}

    # 1. the reference's own known-answer test (jpg_driver.c:54-150)
    kat = subprocess.run([os.path.join(O.REF_DIR, "jpg_kat")], check=True, capture_output=True,
                         text=True).stdout.split("Testing zig-zag ordering:")[1].split()
    g["kat_zigzag"] = [int(v) for v in kat]

    # 2. bundled images through the reference BMP loader (trailing bytes quirk included)
    g["images"] = {}
    for name in ("cam", "tiger"):
        path = os.path.join(HERE, "images", f"{name}.bmp")
        size = os.path.getsize(path)
        ent = {"file_size": size, "coef_sha256": {}, "dpcm_sha256": {}}
        ent["underflow"] = O.ref_dump(path, 50, want_underflow=True)[1].tolist()
        for q in (50, 75, 90):
            ent["coef_sha256"][str(q)] = coef_sha(O.ref_dump(path, q))
            ent["dpcm_sha256"][str(q)] = sha(O.ref_dump(path, q, dpcm_=True).astype("<i4"))
        g["images"][name] = ent
    # full arrays for cam (small): lets a failing test show WHERE it differs
    np.save(os.path.join(HERE, "cam_q75_ref.npy"),
            O.ref_dump(os.path.join(HERE, "images", "cam.bmp"), 75).astype(np.int16))

    # 3. synthetic frames (SURVEY.md 8c generator G, tie frame T) written as 54-byte-header
    #    bottom-up BMPs with no trailing bytes, then run through the reference
    cases = [("G", 512, 512, 1, [50, 75, 90]), ("T", 512, 512, 0, [50]),
             ("G", 8, 8, 11, [50, 90]), ("G", 16, 8, 12, [75]), ("G", 8, 24, 13, [90]),
             ("G", 24, 16, 14, [1, 97]), ("G", 64, 48, 15, [10, 25, 49, 51]),
             ("G", 40, 16, 16, [90]), ("T", 128, 64, 0, [50, 90]),
             ("G", 1920, 1080, 2, [90]), ("G", 3840, 2160, 3, [90, 75])]
    g["synthetic"] = []
    with tempfile.TemporaryDirectory() as td:
        for kind, W, H, seed, qs in cases:
            rgb = O.gen_splitmix(seed, W, H) if kind == "G" else O.gen_tie(W, H)
            bmp = os.path.join(td, "f.bmp")
            O.write_bmp(bmp, rgb)
            ent = {"kind": kind, "W": W, "H": H, "seed": seed, "input_sha256": sha(rgb),
                   "coef_sha256": {}, "sample_ratio": 0,
                   # the [3][8] bytes glibc really left in front of r_new/g_new/b_new
                   "underflow": O.ref_dump(bmp, qs[0], want_underflow=True)[1].tolist()}
            for q in qs:
                ent["coef_sha256"][str(q)] = coef_sha(O.ref_dump(bmp, q))
                if W * H <= 64 * 48:
                    ent.setdefault("coef", {})[str(q)] = O.ref_dump(bmp, q).astype(int).tolist()
            # "4:2:2" parity: the reference's 4:2:2 is a no-op (downsample.c:24-27)
            if W % 16 == 0 and W * H <= 512 * 512:
                ent["coef_sha256_sr1"] = coef_sha(O.ref_dump(bmp, qs[0], sample_ratio=1))
            g["synthetic"].append(ent)
            print(kind, W, H, "done", flush=True)

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)


if __name__ == "__main__":
    main()
