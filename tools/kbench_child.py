"""One kbench measurement in its own process (tools/kbench.py runs it per library; tools/kpmc.sh
runs it under rocprofv3 --pmc): the library named by JPGX_LIB on 8 x 4K frames with fresh input
(two input sets alternating), KB_SUB = sample ratio with JPGX_FLAG_SUBSAMPLE (0: 4:4:4 q90),
KB_REPS rounds of 20 launches after a 300 ms settle.  Prints {"hash", "us"}."""
import os, sys, json, time, hashlib
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jpeg-encoder-and-decoder_amd"))
import torch, jpgx
W, H, F = 3840, 2160, 8
sr = int(os.environ.get("KB_SUB", "0"))
fl = jpgx.FLAG_SUBSAMPLE if sr else 0
q = 75 if sr else 90
dev = torch.device("cuda:0")
ins = []
for s in range(2):
    d = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
    for f in range(F):
        jpgx.gen_splitmix_gpu(d[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f + 100 * s)
    ins.append(d)
nb = (W // 8) * (H // 8)
per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, sr, fl)
out = torch.empty((F, per, 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
p = jpgx.default_params(W, H, q, sr, flags=fl)
jpgx.blocks_gpu(fr, p, ins[0], out, ws); torch.cuda.synchronize()
h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
i = 0
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    for _ in range(10):
        jpgx.blocks_gpu(fr, p, ins[i & 1], out, ws); i += 1
    torch.cuda.synchronize()
ts = []
for r in range(int(os.environ.get("KB_REPS", "5"))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        jpgx.blocks_gpu(fr, p, ins[i & 1], out, ws); i += 1
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / 20)
print(json.dumps({"hash": h, "us": sorted(ts)}))
