"""Locate k_mx mismatches on small frames: per channel / block / coefficient vs the oracle."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd"), os.path.join(REPO, "oracle")]
import jpgx  # noqa: E402
import oracle as O  # noqa: E402

ZZ = [0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43, 9, 11,
      18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60, 21, 34,
      37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63]
inv = {z: (i // 8, i % 8) for i, z in enumerate(ZZ)}
for (W, H, q) in ((80, 8, 50), (512, 16, 50)):
    rgb = O.gen_splitmix(7, W, H)
    out = jpgx.encode_blocks(torch.from_numpy(rgb).cuda(), q).cpu().numpy()
    ref = O.blocks(rgb, q)
    bad = out != ref
    print(f"{W}x{H} q{q}: {bad.sum()} / {bad.size} mismatches")
    for c in range(3):
        nbk = bad[c].sum(axis=1)
        print(" ch", c, "per block:", nbk[:16].tolist())
    # per (v,u) for channel 0 and 2 over blocks
    for c in range(3):
        m = np.zeros((8, 8), int)
        for z in range(64):
            v, u = inv[z]
            m[v, u] = bad[c, :, z].sum()
        print(" ch", c, "per (v,u):\n", m)
    print(" block 0 ch0 got", out[0, 0, :12].tolist(), "\n want", ref[0, 0, :12].tolist())
    print(" block 1 ch2 got", out[2, 1, :12].tolist(), "\n want", ref[2, 1, :12].tolist())

# multi-step waves: a 4K frame (16200 steps over ~3072 waves)
W, H, q = 3840, 2160, 50
rgb = O.gen_splitmix(11, W, H)
out = jpgx.encode_blocks(torch.from_numpy(rgb).cuda(), q).cpu().numpy()
bpr = W // 8
rows = [0, 1, 100, 269]
for r in rows:
    sub = rgb[max(0, 8 * r - 8):8 * r + 8]
    ref = O.blocks(sub, q, underflow=list(jpgx.glibc_underflow(W * H)),
                   rows=(0, 1) if r == 0 else (1, 2))
    got = out[:, r * bpr:(r + 1) * bpr]
    bad = (got != ref).any(axis=(0, 2))
    idx = np.nonzero(bad)[0]
    print(f"4K row {r}: {len(idx)} bad blocks; first cols {idx[:24].tolist()}")
    if len(idx):
        b = idx[0]
        for c in range(3):
            print("  ch", c, "got", got[c, b, :10].tolist(), "want", ref[c, b, :10].tolist())
