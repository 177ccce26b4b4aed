"""Diagnostics (GPU box): error RATE of the library in JPGX_LIB -- N launches of 2 x 4K q75 frames
(seeds 1000, 1001) per sample ratio, each compared on the GPU with the oracle's output: launches
with a wrong block, wrong blocks in all, and their step slots (block % 8) and planes.
Usage: JPGX_LIB=... python tools/diag_rate.py N [SR ...]"""
import collections
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import jpgx  # noqa: E402
import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
srs = [int(x) for x in sys.argv[2:]] or [0, 1, 2]
W, H, q, seeds = 3840, 2160, 75, [1000, 1001]
frames = [O.gen_splitmix(s, W, H) for s in seeds]
d_in = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).cuda()
nb = (H // 8) * (W // 8)
print("lib", os.path.basename(os.environ.get("JPGX_LIB", "product")), flush=True)
for sr in srs:
    S = jpgx.FLAG_SUBSAMPLE if sr else 0
    nbc = jpgx.chroma_blocks(W, 0, H // 8, sr, S) if sr else nb
    per = nb + 2 * nbc
    if sr:
        want = np.stack([np.concatenate([O.blocks(f, q, sr)[0], O.chroma_sub(f, q, sr).reshape(-1, 64)])
                         for f in frames])
    else:
        want = np.stack([O.blocks(f, q).reshape(-1, 64) for f in frames])
    d_want = torch.from_numpy(want).cuda()
    fr = jpgx.frames(W, H, nframes=len(frames), out_frame_stride=per * 64)
    p = jpgx.default_params(W, H, q, sr, flags=S)
    out = torch.zeros((len(frames), per, 64), dtype=torch.int16, device="cuda")
    nbad_launch, nblocks, slots, planes = 0, 0, collections.Counter(), collections.Counter()
    for r in range(n):
        out.zero_()
        jpgx.blocks_gpu(fr, p, d_in, out, 0)
        bad = torch.nonzero((out != d_want).any(dim=2)).cpu().numpy()
        if len(bad):
            nbad_launch += 1
            nblocks += len(bad)
            for f, b in bad:
                plane = 0 if b < nb else (1 if b < nb + nbc else 2)
                bb = b if plane == 0 else (b - nb if plane == 1 else b - nb - nbc)
                slots[int(bb) % 8] += 1
                planes[plane] += 1
    print(f"sr{sr}: {nbad_launch}/{n} launches wrong, {nblocks} wrong blocks, slots {dict(sorted(slots.items()))}, "
          f"planes {dict(sorted(planes.items()))}", flush=True)
