"""Fault probe (GPU box; a JX_MXS_DUMP build in JPGX_LIB): k_mxs writes, per step and lane, the R
pairs of the Y|Cb set-1 tile (acc[1]), its scales w0 and the R pairs of the Cr tile into a debug
buffer.  R launches of 2 x 4K q75 (seeds 1000, 1001); per launch the wrong output blocks (against
the oracle) and which dumped values differ from the majority over the launches (lane group, field).
Usage: JPGX_LIB=.../libjpgx_dump.so python tools/diag_dump.py [R]"""
import collections
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import jpgx  # noqa: E402
import oracle as O  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
W, H, q, seeds = 3840, 2160, 75, [1000, 1001]
frames = [O.gen_splitmix(s, W, H) for s in seeds]
d_in = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).cuda()
nb = (H // 8) * (W // 8)
want = np.stack([O.blocks(f, q).reshape(-1, 64) for f in frames])
d_want = torch.from_numpy(want).cuda()
fr = jpgx.frames(W, H, nframes=2, out_frame_stride=3 * nb * 64)
p = jpgx.default_params(W, H, q, 0)
out = torch.zeros((2, 3 * nb, 64), dtype=torch.int16, device="cuda")
nsteps = 2 * nb // 8
dbg = torch.zeros(nsteps * 64 * 24, dtype=torch.float32, device="cuda")
jpgx.lib.jx_dbg_set.argtypes = [ctypes.c_void_p]
assert jpgx.lib.jx_dbg_set(ctypes.c_void_p(dbg.data_ptr())) == 0
dumps, bads = [], []
for r in range(R):
    out.zero_()
    dbg.fill_(float("nan"))
    jpgx.blocks_gpu(fr, p, d_in, out, 0)
    torch.cuda.synchronize()
    bad = torch.nonzero((out != d_want).any(dim=2)).cpu().numpy()
    bl = sorted({(int(f), int(b) // nb, int(b) % nb) for f, b in bad})   # (frame, plane, block)
    bads.append(bl)
    dumps.append(dbg.view(nsteps, 64, 24).cpu().numpy().view(np.uint32).copy())
    print(f"launch {r}: {len(bl)} wrong blocks {bl[:8]}", flush=True)
D = np.stack(dumps)                                        # [R, step, lane, 24]
# majority per element (R >= 3): the value most launches agree on
maj = np.median(D.astype(np.float64), axis=0)              # exact for uint32 when a majority agrees
dev = D != maj[None].astype(np.uint32)
names = {0: "R(acc1)", 8: "w0", 16: "R(Cr)"}
for r in range(R):
    s_idx, l_idx, f_idx = np.nonzero(dev[r])
    kinds = collections.Counter()
    for s, l, f in zip(s_idx, l_idx, f_idx):
        kinds[(names[(f // 8) * 8], int(l) // 16)] += 1
    steps = sorted(set(int(s) for s in s_idx))
    print(f"launch {r}: {len(s_idx)} deviating values in {len(steps)} steps; by (field, lane group): "
          f"{dict(sorted(kinds.items()))}", flush=True)
    for s in steps[:6]:
        ls, fs = np.nonzero(dev[r, s])
        f0 = s * 8 // nb
        blk = s * 8 % nb
        print(f"   step {s} (frame {f0}, blocks {blk}..{blk + 7}, wave step {(s % 3)}): lanes {sorted(set(ls.tolist()))[:20]} "
              f"fields {sorted(set(fs.tolist()))}", flush=True)
        l, f = int(ls[0]), int(fs[0])
        got = D[r, s, l].view(np.float32)
        m = maj[s, l].astype(np.uint32).view(np.float32)
        print(f"      lane {l}: got {np.round(got[(f//8)*8:(f//8)*8+8], 4).tolist()}\n"
              f"           maj {np.round(m[(f//8)*8:(f//8)*8+8], 4).tolist()}", flush=True)
    # wrong output blocks without a deviating dumped value
    dsteps = set(steps)
    miss = [(f, pl, b) for f, pl, b in bads[r] if (f * nb + b) // 8 not in dsteps]
    print(f"   wrong blocks whose step has no deviating dumped value: {len(miss)} {miss[:6]}", flush=True)
