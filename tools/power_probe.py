"""Sustained-load probe: run the 4:4:4 kernel back to back for a few seconds while sampling the
GPU's power and clocks with amd-smi / rocm-smi (read-only), to see whether the sustained rate is
set by a power/clock limit.  Usage (GPU box): python tools/power_probe.py OUT.json [kernel]"""
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402

import jpgx  # noqa: E402


def sample(stop, out):
    while not stop.is_set():
        t = time.time()
        try:
            r = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"],
                               capture_output=True, text=True, timeout=5)
            out.append({"t": t, "smi": json.loads(r.stdout) if r.stdout.strip().startswith("{") else r.stdout[-400:]})
        except Exception as e:  # noqa: BLE001
            out.append({"t": t, "err": str(e)})
        time.sleep(0.3)


def main():
    dst = sys.argv[1]
    if len(sys.argv) > 2:
        if sys.argv[2] == "xform":
            os.environ["JPGX_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jpeg-encoder-and-decoder_amd", "lib", "libjpgx_alt.so")
    W, H, F, q = 3840, 2160, 8, 90
    dev = torch.device("cuda:0")
    d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
    for f in range(F):
        jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
    out = torch.empty((F, 3, (W // 8) * (H // 8), 64), dtype=torch.int16, device=dev)
    fr = jpgx.frames(W, H, nframes=F)
    p = jpgx.default_params(W, H, q)
    jpgx.blocks_gpu(fr, p, d_in, out, 0)
    torch.cuda.synchronize()
    samples, stop = [], threading.Event()
    idle = []
    sample_once = threading.Thread(target=sample, args=(stop, idle))
    sample_once.start()
    time.sleep(1.0)
    stop.set()
    sample_once.join()
    stop = threading.Event()
    th = threading.Thread(target=sample, args=(stop, samples))
    th.start()
    t0 = time.time()
    ms = []
    while time.time() - t0 < 6.0:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            jpgx.blocks_gpu(fr, p, d_in, out, 0)
        e1.record()
        torch.cuda.synchronize()
        ms.append((time.time() - t0, e0.elapsed_time(e1) / 50))
    stop.set()
    th.join()
    res = {"kernel": ("xform" if os.environ.get("JPGX_LIB", "").endswith("_alt.so") else "mx"), "launch_ms": ms, "idle": idle,
           "load": samples}
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({"first": ms[:3], "last": ms[-3:], "n": len(ms)}))
    for s in samples[:2] + samples[-2:]:
        print(json.dumps(s)[:600])


if __name__ == "__main__":
    main()
