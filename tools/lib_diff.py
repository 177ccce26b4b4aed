"""Output of the library in JPGX_LIB on one batch (4:4:4 / true 4:2:2 / 4:2:0, 4K frames),
saved for a block-by-block comparison between two builds (diagnostics; GPU box).
Usage: JPGX_LIB=... python tools/lib_diff.py save NAME SR  |  python tools/lib_diff.py cmp A B SR"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
W, H, F, Q = 3840, 2160, 4, 75

if sys.argv[1] == "save":
    import torch
    sys.path[:0] = [os.path.join(REPO, "jpeg-encoder-and-decoder_amd")]
    import jpgx
    name, sr = sys.argv[2], int(sys.argv[3])
    S = jpgx.FLAG_SUBSAMPLE if sr else 0
    d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device="cuda")
    for i in range(F):
        jpgx.gen_splitmix_gpu(d_in[i * W * H * 3:(i + 1) * W * H * 3], 1000 + i)
    nb = (H // 8) * (W // 8)
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, sr, S) if sr else 3 * nb
    out = torch.empty((F, per, 64), dtype=torch.int16, device="cuda")
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, Q, sr, flags=S), d_in, out, 0)
    np.save(os.path.join(OUT, f"diff_{name}_{sr}.npy"), out.cpu().numpy())
else:
    a, b, sr = sys.argv[2], sys.argv[3], int(sys.argv[4])
    A = np.load(os.path.join(OUT, f"diff_{a}_{sr}.npy"))
    B = np.load(os.path.join(OUT, f"diff_{b}_{sr}.npy"))
    nb = (H // 8) * (W // 8)
    bad = (A != B).any(axis=2)
    print("bad blocks per frame:", bad.sum(axis=1).tolist(), "of", A.shape[1])
    for f in range(F):
        idx = np.flatnonzero(bad[f])
        if not len(idx):
            continue
        y = idx[idx < nb]
        c = idx[idx >= nb] - nb
        print(f"frame {f}: Y bad {len(y)}, chroma bad {len(c)}")
        if sr == 2:
            mpr = W // 16
            ym = [(int(i) // (W // 8) // 2 * mpr + (int(i) % (W // 8)) // 2) for i in y[:20]]
            print("  Y blocks", y[:20].tolist(), "-> MCU", ym, "mcu%12", [m % 12 for m in ym])
            nmcu = (H // 16) * mpr
            cm = (c % nmcu)
            print("  chroma MCU", cm[:20].tolist(), "mcu%12", (cm[:20] % 12).tolist(), "cr?", (c[:20] >= nmcu).tolist())
        else:
            print("  blocks", idx[:20].tolist())
        i0 = idx[0]
        print("  first", A[f, i0, :10].tolist(), B[f, i0, :10].tolist())
