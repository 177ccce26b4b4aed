"""Diagnostics (GPU box): latency of each kernel's inline exact pass on the bench workload, from the
timing build (libjpgx_cnt3.so: s_memtime around the pass; counters [2k] passes, [2k+1] clocks, k = 0
4:4:4, 1 4:2:2, 2 4:2:0), and the prefilter counters of cnt2 ([8..11]).
Usage: JPGX_LIB=.../libjpgx_cnt3.so python tools/diag_exact_time.py [launches]"""
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
for sr, kind, q in ((0, 0, 90), (1, 1, 75), (2, 2, 75)):
    fl = jpgx.FLAG_SUBSAMPLE if sr else 0
    per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, sr, fl)
    out = torch.empty((F, per, 64), dtype=torch.int16, device=dev)
    fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
    ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
    p = jpgx.default_params(W, H, q, sr, flags=fl)
    jpgx.blocks_gpu(fr, p, d, out, ws)
    torch.cuda.synchronize()
    cnt(buf, 1)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        jpgx.blocks_gpu(fr, p, d, out, ws)
    e1.record()
    torch.cuda.synchronize()
    cnt(buf, 1)
    passes, clk = buf[2 * kind] / n, buf[2 * kind + 1] / n
    print(f"sr{sr} q{q}: {e0.elapsed_time(e1) * 1e3 / n:.1f} us per launch; {passes:.0f} exact passes per launch, "
          f"mean {clk / max(passes, 1):.0f} s_memtime ticks each; prefilter fired in {buf[8] / n:.0f} of "
          f"{buf[10] / n:.0f} column passes", flush=True)
