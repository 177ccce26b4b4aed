"""Diagnostics (GPU box): how often each kernel's inline exact pass runs on the bench workload
(8 x 4K splitmix frames; q90 for 4:4:4, q75 for 4:2:2 / 4:2:0), from the counting build
(libjpgx_cnt.so: build/vsrc/cnt.hip, made by the round-5 session notes in profiles/r05_*): per
launch the exact-pass entries, those the whole-wave single-coefficient path finished, the 8-lane
batches, and the flagged coefficients.
Usage: JPGX_LIB=.../libjpgx_cnt.so python tools/diag_exact_count.py [launches]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402
import jpgx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W, H, F = 3840, 2160, 8
dev = torch.device("cuda:0")
cnt = jpgx.lib.jx_dbg_counters
cnt.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
d = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
for f in range(F):
    jpgx.gen_splitmix_gpu(d[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
nb = (W // 8) * (H // 8)
for sr, kind, q, steps_per in ((0, 0, 90, 8), (1, 1, 75, 8), (2, 2, 75, 16)):
    fl = jpgx.FLAG_SUBSAMPLE if sr else 0
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, sr, fl)
    out = torch.empty((F, per, 64), dtype=torch.int16, device=dev)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
    p = jpgx.default_params(W, H, q, sr, flags=fl)
    torch.cuda.synchronize()
    cnt(buf, 1)
    for _ in range(n):
        jpgx.blocks_gpu(fr, p, d, out, ws)
    torch.cuda.synchronize()
    cnt(buf, 1)
    e, one, b8, bits = (buf[4 * kind + i] / n for i in range(4))
    cols, rare, rare_fl, lanes = buf[10] / n, buf[8] / n, buf[9] / n, buf[11] / n
    units = F * nb / steps_per
    what = "step" if steps_per == 8 else "step pair"
    print(f"sr{sr} q{q}: per launch {e:.0f} exact passes ({e / units:.4f} per {what}), whole-wave "
          f"{one:.0f} ({one / max(e, 1):.3f}), 8-lane batches {b8:.0f}, flagged coefficients {bits:.0f} "
          f"({bits / units:.4f} per {what})", flush=True)
    if cols:
        print(f"   column passes {cols:.0f}: prefilter fired in {rare:.0f} ({rare / cols:.4f}; lanes {lanes / cols:.3f} "
              f"per pass), of which flagged {rare_fl:.0f} ({rare_fl / max(rare, 1):.3f})", flush=True)
