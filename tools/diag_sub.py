"""Diagnostics (GPU box): REPS launches of 2 x 4K q75 frames (seeds 1000, 1001) through the library
in JPGX_LIB, for sr in SRS (0 = 4:4:4, 1 = true 4:2:2, 2 = true 4:2:0), each launch compared block by
block with the oracle: the wrong blocks per launch as (frame, plane, block, block % 8).
Usage: JPGX_LIB=... python tools/diag_sub.py REPS [SR ...]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import jpgx  # noqa: E402
import oracle as O  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
srs = [int(x) for x in sys.argv[2:]] or [1, 2]
W, H, q, seeds = 3840, 2160, 75, [1000, 1001]
frames = [O.gen_splitmix(s, W, H) for s in seeds]
d_in = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).cuda()
nb = (H // 8) * (W // 8)
print("lib", os.environ.get("JPGX_LIB", "product"), flush=True)
for sr in srs:
    S = jpgx.FLAG_SUBSAMPLE if sr else 0
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, S) if sr else nb
    per = nb + 2 * nbc
    if sr:
        want = np.stack([np.concatenate([O.blocks(f, q, sr)[0], O.chroma_sub(f, q, sr).reshape(-1, 64)])
                         for f in frames])
    else:
        want = np.stack([O.blocks(f, q).reshape(-1, 64) for f in frames])
    fr = jpgx.frames(W, H, nframes=len(frames), out_frame_stride=per * 64)
    p = jpgx.default_params(W, H, q, sr, flags=S)
    for r in range(reps):
        out = torch.zeros((len(frames), per, 64), dtype=torch.int16, device="cuda")
        jpgx.blocks_gpu(fr, p, d_in, out, 0)
        got = out.cpu().numpy()
        bad = np.argwhere((got != want).any(axis=2))
        desc = []
        for f, b in bad[:int(os.environ.get("DIAG_SHOW", "10"))]:
            plane = 0 if b < nb else (1 if b < nb + nbc else 2)
            bb = b if plane == 0 else (b - nb if plane == 1 else b - nb - nbc)
            desc.append((int(f), plane, int(bb) // (W // 8), int(bb) % (W // 8)) if plane == 0 else (int(f), plane, int(bb)))
        print(f"sr{sr} rep {r}: {len(bad)} wrong block(s) {desc}", flush=True)
