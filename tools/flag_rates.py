"""Guard-band flag rates of k_mxs by (channel, u, v), estimated on the host.

For a splitmix frame (the bench's input) every block's exact quotient t = F / Q is computed in
float64 (the reference's definition: colour + level shift, preprocess.c:160-162,186-188; the 8x8
DCT, dct.c:36-59; the transposed divisor, quantise.c:58) and a coefficient counts as flagged when
|t - rint(t)| >= lim, lim = k_mxs's band limit for its plan column and v (jx_plan_tables_mx, the
table the kernel's rare path tests; the kernel tests the fp32 quotient, which lies within the
band's error bound of t, so this is the kernel's rate up to that bound).  Reports, per quality:
flagged coefficients per step (8 blocks x 3 channels), per block-channel, the hottest (c, u, v)
cells, and the share of flagged steps holding exactly one flagged coefficient (the whole-wave case
of mx_exact_inline).

Usage: python tools/flag_rates.py [W H] [q ...]     (default 3840 2160, q 50 75 90)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402  (test infrastructure: the input generator and the scale tables)

LIB = ctypes.CDLL(os.path.join(ROOT, "jpeg-encoder-and-decoder_amd", "lib", "libjpgx.so"))
LIB.jx_plan_tables_mx.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3


def tables(q):
    w = np.zeros((24, 8), np.float32)
    lim = np.zeros((24, 8), np.float32)
    qq = np.zeros((2, 64), np.int16)
    rc = LIB.jx_plan_tables_mx(q, w.ctypes.data, lim.ctypes.data, qq.ctypes.data)
    assert rc == 0, rc
    return lim, qq.reshape(2, 8, 8).astype(np.float64)     # q[t][u][v]


def channels(rgb):
    r, g, b = (rgb[..., k].astype(np.float64) for k in range(3))
    y = 0.299 * r + 0.587 * g + 0.114 * b - 128.0
    cb = 128.0 - (0.168736 * r - 0.331264 * g + 0.5 * b) - 128.0   # the reference's sign quirk
    cr = 128.0 + (0.5 * r - 0.418688 * g - 0.081312 * b) - 128.0
    return [y, cb, cr]


def main():
    args = [int(a) for a in sys.argv[1:]]
    W, H = (args[0], args[1]) if len(args) >= 2 else (3840, 2160)
    qs = args[2:] if len(args) > 2 else [50, 75, 90]
    rgb = oracle.gen_splitmix(1, W, H)
    n = np.arange(8)
    C = np.cos((2 * n[None, :] + 1) * n[:, None] * np.pi / 16)      # C[u][x]
    alpha = np.where(n == 0, 1 / np.sqrt(2), 1.0)
    nb = (W // 8) * (H // 8)
    for q in qs:
        lim, Q = tables(q)
        print(f"q{q}: {W}x{H}, {nb} blocks per channel, {nb // 8} steps")
        step_flags = np.zeros(nb // 8, np.int64)
        tot = []
        cells = []
        grids = []
        for c, X in enumerate(channels(rgb)):
            Xb = X.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8)   # [blk][y][x]
            # D[v][u] = 1/4 a(u) a(v) sum_x sum_y X[y][x] cos_u[x] cos_v[y]
            D = 0.25 * np.einsum("byx,ux,vy->bvu", Xb, C, C) * alpha[None, :, None] * alpha[None, None, :]
            t = D / Q[0 if c == 0 else 1].T[None]                    # divisor table[u][v] at (v, u)
            dist = np.abs(t - np.rint(t))
            L = np.stack([lim[(8 * c + u) if c < 2 else 16 + u] for u in range(8)], 1)   # L[v][u]
            f = dist >= L[None]
            rate = f.mean(0)                                         # [v][u]
            grids.append(rate)
            tot.append(f.sum() / nb)
            step_flags += f.reshape(nb // 8, 8, 64).sum((1, 2))
            for v in range(8):
                for u in range(8):
                    cells.append((rate[v, u], ("Y", "Cb", "Cr")[c], u, v))
        fl = step_flags[step_flags > 0]
        print(f"  flagged per step {step_flags.mean():.4f}; per block-channel Y {tot[0]:.5f} Cb {tot[1]:.5f} "
              f"Cr {tot[2]:.5f}; flagged steps {len(fl) / len(step_flags):.4f}, of which one coefficient "
              f"{(fl == 1).mean():.3f}")
        cells.sort(reverse=True)
        print("  hottest cells (rate per block, channel, u, v):",
              ", ".join(f"{r:.2e} {ch}({u},{v})" for r, ch, u, v in cells[:10]))
        print("  rate per block x 1e4, rows v = 0..7, columns u = 0..7 (Y | Cb | Cr):")
        for v in range(8):
            print("   " + " | ".join(" ".join(f"{1e4 * g[v, u]:5.2f}" for u in range(8)) for g in grids))


if __name__ == "__main__":
    main()
