"""k_mx launch time vs input content (power / DVFS check): splitmix noise (the bench), a
constant frame, and a smooth gradient, each as 2 alternating 8 x 4K input sets (fresh input),
settled.  Usage (GPU box): python tools/data_ab.py [lib ...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402

import jpgx  # noqa: E402

W, H, F, q = 3840, 2160, 8, 90
dev = torch.device("cuda:0")
n = F * W * H * 3
sets = {}
a = torch.empty(n, dtype=torch.uint8, device=dev)
for f in range(F):
    jpgx.gen_splitmix_gpu(a[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
sets["splitmix"] = [a, a.clone()]
sets["const128"] = [torch.full((n,), 128, dtype=torch.uint8, device=dev) for _ in range(2)]
yy = torch.arange(H, device=dev).view(H, 1, 1)
xx = torch.arange(W, device=dev).view(1, W, 1)
cc = torch.arange(3, device=dev).view(1, 1, 3)
g = ((xx * 255) // W + (yy * 3) // 17 + cc * 40) % 256
g = g.to(torch.uint8).reshape(-1).repeat(F)
sets["gradient"] = [g, g.clone()]
out = torch.empty((F, 3, (W // 8) * (H // 8), 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F)
p = jpgx.default_params(W, H, q)
for name, ins in sets.items():
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(10):
            jpgx.blocks_gpu(fr, p, ins[k % 2], out, 0)
            k += 1
        torch.cuda.synchronize()
    ts = []
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            jpgx.blocks_gpu(fr, p, ins[k % 2], out, 0)
            k += 1
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ts.sort()
    print(f"{name:10s} us per launch: min {ts[0]:.1f} med {ts[2]:.1f}  frac(min) {n * 3 / (ts[0] * 1e-6) / 8e12:.3f}",
          flush=True)
