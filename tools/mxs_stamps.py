"""Per-wave timeline of k_mxs on the bench workload (8 x 4K q90, two input sets alternating):
a -DJX_MXS_STAMP build (tools/build_variants.sh NAME "-DJX_MXS_C=C -DJX_MXS_STAMP") records, per
wave, s_memrealtime (100 MHz) at start, after the workgroup image + B reads, after step 0, at the
end (and after its stores drained), s_memtime at start / end (shader clock) and its XCC/SE/CU.
Usage (GPU box): python tools/mxs_stamps.py NAME [C]"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1]
C = int(sys.argv[2]) if len(sys.argv) > 2 else 3
os.environ["JPGX_LIB"] = os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "variants", f"libjpgx_{name}.so")
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import jpgx  # noqa: E402

W, H, F = 3840, 2160, 8
dev = torch.device("cuda:0")
ins = []
for s in range(2):
    d = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
    for f in range(F):
        jpgx.gen_splitmix_gpu(d[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f + 100 * s)
    ins.append(d)
nb = (W // 8) * (H // 8)
out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F)
ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
p = jpgx.default_params(W, H, 90)
t0 = time.perf_counter()
i = 0
while time.perf_counter() - t0 < 0.3:
    for _ in range(10):
        jpgx.blocks_gpu(fr, p, ins[i & 1], out, ws)
        i += 1
    torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
jpgx.blocks_gpu(fr, p, ins[i & 1], out, ws)
e1.record()
torch.cuda.synchronize()
nwaves = (F * nb // 8 + C - 1) // C
buf = np.zeros(1 << 20, np.uint64)
f = jpgx.lib.jx_mxs_stamps
f.restype = ctypes.c_int
assert f(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(1 << 20)) == 0
ts = buf[:8 * nwaves].reshape(nwaves, 8).astype(np.int64)
ts = ts[ts[:, 0] > 0]
base = ts[:, 0].min()
us = lambda x: x / 100.0                         # s_memrealtime ticks (100 MHz) -> us
start, img, step0, end, drained = (us(ts[:, k] - base) for k in (0, 1, 2, 3, 6))
life = end - start
clk = (ts[:, 4] - ts[:, 5]) / np.maximum(ts[:, 3] - ts[:, 0], 1) * 100.0
print(f"{name}: C={C} waves={len(ts)} launch {e0.elapsed_time(e1) * 1e3:.1f} us, span {end.max():.1f} us")
q = lambda a: " ".join(f"{np.percentile(a, x):7.2f}" for x in (10, 50, 90))
print("                      p10     p50     p90 (us)")
print("start->image+B     ", q(img - start))
print("image->step0 done  ", q(step0 - img))
print("step0->end         ", q(end - step0))
print("lifetime           ", q(life))
print("end->stores drained", q(drained - end))
print("start time         ", q(start))
print(f"shader clock MHz    {np.percentile(clk, 50):.0f} (p10 {np.percentile(clk, 10):.0f}, p90 {np.percentile(clk, 90):.0f})")
# concurrency: waves alive over time (1 us bins)
t = np.arange(0, end.max(), 1.0)
alive = [(np.sum((start <= x) & (end > x))) for x in t]
print("waves alive (every 10 us):", " ".join(str(int(alive[k])) for k in range(0, len(alive), 10)))
# workgroup granularity: a workgroup's resources are held from its first wave's start to its last
# wave's end; efficiency = sum of wave lifetimes / (4 x that span)
wg = (np.nonzero(buf[:8 * nwaves].reshape(nwaves, 8)[:, 0])[0]) // 4
ws_ = {}
for k, w in enumerate(wg):
    ws_.setdefault(w, []).append(k)
eff = []
for w, ks in ws_.items():
    if len(ks) == 4:
        span = end[ks].max() - start[ks].min()
        eff.append(life[ks].sum() / (4 * span))
print(f"workgroup occupancy efficiency: mean {np.mean(eff):.3f} (p10 {np.percentile(eff, 10):.3f})")
# per-CU handover: on each (xcc, se, cu), the gap between a workgroup's last end and the next
# workgroup start after it
hw = ts[:, 7]
cu = ((hw >> 32) & 7) * 4096 + ((hw >> 13) & 7) * 256 + ((hw >> 8) & 15)
order = np.lexsort((start, cu))
gaps = []
for c in np.unique(cu):
    idx = order[cu[order] == c]
    s_, e_ = start[idx], end[idx]
    for k in range(1, len(idx)):
        if s_[k] > s_[k - 1] + 0.05:
            prev_end = e_[:k][e_[:k] <= s_[k]]
            if len(prev_end):
                gaps.append(s_[k] - prev_end.max())
print(f"start after the latest end on its CU (us): p10 {np.percentile(gaps, 10):.2f} p50 {np.percentile(gaps, 50):.2f} p90 {np.percentile(gaps, 90):.2f}")
