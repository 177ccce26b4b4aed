"""What makes the first launches of a session slow?  Per-launch HIP-event times of the 4:4:4
kernel over the first 300 launches, (a) into a freshly allocated output, (b) into an output that
was zero-filled first, (c) the same buffers again after 1 s idle, (d) after 0.2 s of a plain
copy kernel keeping HBM busy.  Usage (GPU box): python tools/ramp_probe.py OUT.json"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402

import jpgx  # noqa: E402

W, H, F, q = 3840, 2160, 8, 90


def run(fr, p, d_in, out, n=300):
    ts = []
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in evs:
        e0.record()
        jpgx.blocks_gpu(fr, p, d_in, out, 0)
        e1.record()
    torch.cuda.synchronize()
    for e0, e1 in evs:
        ts.append(e0.elapsed_time(e1))
    return ts


def summ(ts):
    return [round(sum(ts[i:i + 25]) / 25, 4) for i in range(0, len(ts), 25)]


def main():
    dev = torch.device("cuda:0")
    d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
    for f in range(F):
        jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
    nb = (W // 8) * (H // 8)
    fr = jpgx.frames(W, H, nframes=F)
    p = jpgx.default_params(W, H, q)
    res = {}
    out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    res["a_fresh_output"] = run(fr, p, d_in, out)
    out2 = torch.zeros((F, 3, nb, 64), dtype=torch.int16, device=dev)
    torch.cuda.synchronize()
    time.sleep(1.0)
    res["b_zeroed_output_after_1s_idle"] = run(fr, p, d_in, out2)
    time.sleep(1.0)
    res["c_same_after_1s_idle"] = run(fr, p, d_in, out2)
    big = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    t0 = time.time()
    while time.time() - t0 < 0.2:
        big[: 1 << 29].copy_(big[1 << 29:])
    res["d_after_200ms_copy"] = run(fr, p, d_in, out2)
    for k, v in res.items():
        print(k, summ(v))
    with open(sys.argv[1], "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
