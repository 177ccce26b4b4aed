"""k_xform+exact time vs frames per launch (fixed startup/tail cost = intercept of the line).
Usage (GPU box): python tools/frames_sweep.py [lib]"""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jpeg-encoder-and-decoder_amd"))
import torch, jpgx
W, H, q = 3840, 2160, 90
dev = torch.device("cuda:0")
res = {}
for F in (1, 2, 4, 8, 16, 24):
    d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
    for f in range(F):
        jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
    nb = (W // 8) * (H // 8)
    out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device=dev)
    fr = jpgx.frames(W, H, nframes=F)
    ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
    p = jpgx.default_params(W, H, q)
    for _ in range(3):
        jpgx.blocks_gpu(fr, p, d_in, out, ws)
    torch.cuda.synchronize()
    ts = []
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            jpgx.blocks_gpu(fr, p, d_in, out, ws)
        e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    ms = min(ts)
    res[F] = ms
    print(f"frames {F:3d}: {ms:.4f} ms  {ms / F * 1000:.1f} us/frame  {F * W * H * 9 / ms / 1e6:.0f} GB/s", flush=True)
    del d_in, out, ws
