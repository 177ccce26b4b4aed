"""4:4:4 kernel time vs frames per launch, 3840x2160 q90 (bench.py's frames, seeds 1000+f).
The fixed startup/tail cost is the intercept of the line; a flat us/frame from 8 frames (199 MB
of input, under the 256 MiB Infinity Cache) to 16 and 24 frames (398 / 597 MB, over it) says the
bench's 8-frame launch is not flattered by cache residency.

Usage (GPU box): python tools/frames_sweep.py OUT.json [xform mx]
After 200 ms of untimed launches (the GPU's ramp out of idle), HIP events around
10 back-to-back launches, 5 repetitions: min and median of the per-launch mean are reported."""
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402

import jpgx  # noqa: E402

W, H, q = 3840, 2160, 90


def sweep(kernel, dev):
    if kernel == "xform":
        os.environ["JPGX_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jpeg-encoder-and-decoder_amd", "lib", "libjpgx_alt.so")
    rows = []
    for F in (1, 2, 4, 8, 16, 24):
        d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
        for f in range(F):
            jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
        nb = (W // 8) * (H // 8)
        out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device=dev)
        fr = jpgx.frames(W, H, nframes=F)
        p = jpgx.default_params(W, H, q)
        import time
        t0 = time.perf_counter()                   # settle: the GPU's ramp out of idle (~20 ms)
        while time.perf_counter() - t0 < 0.2:
            for _ in range(5):
                jpgx.blocks_gpu(fr, p, d_in, out, 0)
            torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                jpgx.blocks_gpu(fr, p, d_in, out, 0)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        r = {"frames": F, "input_MB": F * W * H * 3 / 1e6, "ms_min": min(ts),
             "ms_median": statistics.median(ts), "us_per_frame_min": min(ts) / F * 1e3,
             "us_per_frame_median": statistics.median(ts) / F * 1e3,
             "GBps_median": F * W * H * 9 / statistics.median(ts) / 1e6}
        rows.append(r)
        print(kernel, json.dumps(r), flush=True)
        del d_in, out
        torch.cuda.empty_cache()
    return rows


def main():
    dst = sys.argv[1]
    kernels = sys.argv[2:] or ["xform", "mx"]
    dev = torch.device("cuda:0")
    res = {"workload": f"F x {W}x{H} RGB, q={q}, one launch per F frames",
           "timing": "HIP events around 10 launches, 5 reps", "device": torch.cuda.get_device_name(0),
           "sweeps": {k: sweep(k, dev) for k in kernels}}
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
