"""Diagnostics (GPU box): the golden 4K frame (tests/golden/golden.json, G 3840x2160 seed 3) at
q75 and q90 through the library in JPGX_LIB, REPS launches each, against the oracle: every
mismatching (channel, block, zig-zag index, got, want) and whether it repeats launch to launch.
Usage: JPGX_LIB=... python tools/diag_golden.py [REPS]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import jpgx  # noqa: E402
import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
g = json.load(open(os.path.join(REPO, "tests", "golden", "golden.json")))
ent = [e for e in g["synthetic"] if e["W"] == 3840][0]
rgb = O.gen_splitmix(ent["seed"], ent["W"], ent["H"])
d = torch.from_numpy(np.ascontiguousarray(rgb)).cuda()
print("lib", os.environ.get("JPGX_LIB", "product"), flush=True)
for q in (75, 90):
    ref = O.blocks(rgb, q, underflow=ent["underflow"])
    seen = {}
    for r in range(reps):
        out = jpgx.encode_blocks(d, q, 0, underflow=ent["underflow"]).cpu().numpy()
        bad = np.argwhere(out != ref)
        blocks = sorted({(int(c), int(b)) for c, b, _ in bad})
        print(f"q{q} rep {r}: {len(bad)} coefficient(s) in {len(blocks)} block(s) "
              f"{[(c, b, b % 8) for c, b in blocks[:12]]}", flush=True)
        for c, b, k in bad[:40]:
            key = (int(c), int(b), int(k))
            seen[key] = seen.get(key, 0) + 1
            if seen[key] == 1 and len(seen) <= 40:
                print(f"   ch {c} block {b} (row {b // 480}, col {b % 480}, step slot {b % 8}) zz {k}: "
                      f"got {out[c, b, k]} want {ref[c, b, k]}")
