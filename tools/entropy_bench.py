"""Time the entropy-stage statistics (jpgx_entropy_stats_gpu: the reference's dpcm + Huffman
frequency pass) on the hot path's own output: 8 x 4K frames at q90, one call per
frame (EB_MODE=frame) or one batch call over the 8 frames (EB_MODE=batch, default), HIP events on
the launch stream around K rounds (settled first).
Algorithmic bytes per block: 128 (its coefficients, read once) + 4 (its dpcm'd DC, written) --
SURVEY.md 8(d)'s output size; the histograms and chunk sums are < 0.1 %.
Usage (GPU box): python tools/entropy_bench.py [LIB ...]   (default: the product library)"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time, ctypes
sys.path.insert(0, os.path.join(%(repo)r, "jpeg-encoder-and-decoder_amd"))
import torch, jpgx
W, H, F, q = 3840, 2160, 8, 90
dev = torch.device("cuda:0")
d = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
for f in range(F):
    jpgx.gen_splitmix_gpu(d[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
nb = (W // 8) * (H // 8)
out = torch.empty((F, 3 * nb, 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F, out_frame_stride=3 * nb * 64)
ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q, 0), d, out, ws)
del d
dc = torch.empty((F, 3 * nb), dtype=torch.int32, device=dev)
hist = torch.empty((F, 4, 257), dtype=torch.int32, device=dev)
wsz = max(int(jpgx.lib.jpgx_entropy_workspace_size(nb, nb)), 8)
ews = torch.empty((F, wsz), dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream().cuda_stream
batch = os.environ.get("EB_MODE", "batch") == "batch"
bwsz = int(jpgx.lib.jpgx_entropy_workspace_size_batch(nb, nb, F)) if batch else 8
bws = torch.empty(bwsz, dtype=torch.uint8, device=dev)
def run():
    if batch:                                   # one call over the 8 frames
        rc = jpgx.lib.jpgx_entropy_stats_gpu_batch(out.data_ptr(), 3 * nb * 64, F, nb, nb, None, dc.data_ptr(),
                                                    hist.data_ptr(), bws.data_ptr(), bwsz, stream)
        assert rc == 0, rc
        return
    for f in range(F):                          # one call per frame
        rc = jpgx.lib.jpgx_entropy_stats_gpu(out[f].data_ptr(), nb, nb, None, dc[f].data_ptr(),
                                              hist[f].data_ptr(), ews[f].data_ptr(), wsz, stream)
        assert rc == 0, rc
run(); torch.cuda.synchronize()
# the histograms against the library's own first call (the tests pin it to the oracle)
ref = hist.clone(); refdc = dc.clone()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    run()
torch.cuda.synchronize()
same = bool(torch.equal(hist, ref) and torch.equal(dc, refdc))
ts = []
for r in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / 10 / F)
alg = 3 * nb * (128 + 4)
print(json.dumps({"us_per_frame": sorted(ts), "bytes_per_frame": alg,
                  "gbs_min": alg / min(ts) / 1e3, "frac_min": alg / min(ts) / 1e3 / 8000.0,
                  "repeat_equal": same,
                  "hash": int(hist.to(torch.int64).mul(torch.arange(1, hist.numel() + 1, device=dev).view_as(hist)).sum())
                          ^ int(dc.to(torch.int64).mul(torch.arange(1, dc.numel() + 1, device=dev).view_as(dc)).sum())}))
'''


def main():
    libs = sys.argv[1:] or ["product"]
    mode = os.environ.get("EB_MODE", "batch")
    first = None
    for n in libs:
        env = dict(os.environ)
        if n != "product":
            env["JPGX_LIB"] = os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "variants",
                                           f"libjpgx_{n}.so")
        r = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO}], env=env,
                           capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(n, "failed", r.stderr[-2000:])
            sys.exit(r.returncode)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        first = d["hash"] if first is None else first
        print(f"{n + ' ' + mode:18s} min {d['us_per_frame'][0]:8.1f} us/frame  med {d['us_per_frame'][2]:8.1f}  "
              f"{d['gbs_min']:7.1f} GB/s  frac(min) {d['frac_min']:.4f}  repeat-equal={d['repeat_equal']}  "
              f"same-as-first={d['hash'] == first}",
              flush=True)


if __name__ == "__main__":
    main()
