"""Mismatch census of the product 4:4:4 kernel on the golden 1080p frame and smaller frames:
which blocks / channels differ from the oracle and by how much (diagnostics; GPU box)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd"), os.path.join(REPO, "oracle")]
import jpgx  # noqa: E402
import oracle as O  # noqa: E402

for (W, H, q, seed) in ((1920, 1080, 90, 2), (256, 64, 90, 5), (240, 64, 90, 5), (1920, 64, 90, 9)):
    rgb = O.gen_splitmix(seed, W, H)
    out = jpgx.encode_blocks(torch.from_numpy(rgb).cuda(), q).cpu().numpy()
    ref = O.blocks(rgb, q)
    bad = out != ref
    nb = out.shape[1]
    bpr = W // 8
    blocks = sorted(set(int(b) for b in np.argwhere(bad.any(axis=2))[:, 1]))
    print(f"{W}x{H} q{q}: {bad.sum()} coefficient mismatches in {len(blocks)} blocks (nb {nb})")
    print("  blocks:", [(b, b // bpr, b % bpr, (b // 8) % 3, b % 8) for b in blocks[:12]])
    for c in range(3):
        print("  ch", c, "bad blocks", int(bad[c].any(axis=1).sum()))
    if blocks:
        b = blocks[0]
        for c in range(3):
            if bad[c, b].any():
                print("  ch", c, "block", b, "got", out[c, b, :12].tolist(), "ref", ref[c, b, :12].tolist())
