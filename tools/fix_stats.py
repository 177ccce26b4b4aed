"""Exact-pass statistics for the bench workload (GPU box): how many block-channels k_xform
queued for k_fix, per channel, read back from the workspace (jpgx_internal.h jx_fixlist
layout: counts [3][nwaves] u32 at byte 256).  Diagnostic only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import jpgx  # noqa: E402

W, H, F = 3840, 2160, 8
q = int(sys.argv[1]) if len(sys.argv) > 1 else 90
dev = torch.device("cuda:0")
d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
for f in range(F):
    jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
nb = (W // 8) * (H // 8)
out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F)
ws = torch.zeros(jpgx.workspace_size(fr), dtype=torch.uint8, device=dev)
p = jpgx.default_params(W, H, q)
jpgx.blocks_gpu(fr, p, d_in, out, ws)
torch.cuda.synchronize()
props = torch.cuda.get_device_properties(0)
raw = ws[256:].cpu().numpy().view(np.uint32)
ntiles = (F * nb + 63) // 64
for nwaves in sorted({props.multi_processor_count * k * 4 for k in (1, 2, 3, 4)}):
    if 3 * nwaves > raw.size:
        continue
    c = raw[:3 * nwaves].reshape(3, nwaves)
    print(f"nwaves={nwaves}: items per channel {c.sum(axis=1).tolist()} total {int(c.sum())} "
          f"per tile {c.sum() / ntiles:.3f}; max per wave {c.max(axis=1).tolist()}")
