"""Eager launches vs a captured HIP graph of the same jpgx_blocks_gpu calls (GPU box):
how much of a step is launch/inter-kernel overhead.  Diagnostic only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402

import jpgx  # noqa: E402

W, H, F, q, N = 3840, 2160, 8, 90, 10
dev = torch.device("cuda:0")
d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
for f in range(F):
    jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
nb = (W // 8) * (H // 8)
out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F)
ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
p = jpgx.default_params(W, H, q)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3):
        jpgx.blocks_gpu(fr, p, d_in, out, ws, stream=s)
torch.cuda.synchronize()
ref = out.clone()


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / N)
    return sorted(ts)


def eager():
    for _ in range(N):
        jpgx.blocks_gpu(fr, p, d_in, out, ws, stream=s)


g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for _ in range(N):
        jpgx.blocks_gpu(fr, p, d_in, out, ws, stream=s)
torch.cuda.synchronize()
out.zero_()
g.replay()
torch.cuda.synchronize()
assert torch.equal(out, ref), "graph replay output differs"
with torch.cuda.stream(s):
    te = timed(eager)
    tg = timed(g.replay)
print(f"eager median {te[len(te) // 2]:.4f} ms/step  graph median {tg[len(tg) // 2]:.4f} ms/step")
