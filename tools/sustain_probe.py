"""Kernel time vs time under sustained load: bench.py's workload (8 x 4K q90, two input sets
alternating = fresh input every launch) launched back to back for SECONDS; every 20 launches are
timed by HIP events on the launch stream, stamped with the wall time since the first launch, while a
thread samples rocm-smi (power, clocks, temperature; read-only).  Prints the mean us per launch
over windows of the load's age.  Usage (GPU box): python tools/sustain_probe.py OUT.json [SECONDS]"""
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


def smi(stop, out, t0):
    while not stop.is_set():
        t = time.perf_counter() - t0
        try:
            r = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--showtemp", "--json"],
                               capture_output=True, text=True, timeout=5)
            out.append({"t": t, "smi": json.loads(r.stdout) if r.stdout.strip().startswith("{") else r.stdout[-300:]})
        except Exception as e:  # noqa: BLE001
            out.append({"t": t, "err": str(e)})
        time.sleep(0.25)


def main():
    dst = sys.argv[1]
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
    W, H, F, q = 3840, 2160, 8, 90
    dev = torch.device("cuda:0")
    ins = []
    for s in range(2):
        d = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
        for f in range(F):
            jpgx.gen_splitmix_gpu(d[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
        ins.append(d)
    out = torch.empty((F, 3, (W // 8) * (H // 8), 64), dtype=torch.int16, device=dev)
    fr = jpgx.frames(W, H, nframes=F)
    p = jpgx.default_params(W, H, q)
    jpgx.blocks_gpu(fr, p, ins[0], out, 0)
    torch.cuda.synchronize()
    time.sleep(1.0)                               # idle, as between a driver's runs
    samples, stop = [], threading.Event()
    t0 = time.perf_counter()
    th = threading.Thread(target=smi, args=(stop, samples, t0))
    th.start()
    wins, i = [], 0
    while time.perf_counter() - t0 < secs:
        evs = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                jpgx.blocks_gpu(fr, p, ins[i & 1], out, 0)
                i += 1
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        wins += [(t, a.elapsed_time(b) * 1e3 / 20) for a, b in evs]
    stop.set()
    th.join()
    edges = [0, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0, 10.0]
    summ = []
    for a, b in zip(edges, edges[1:]):
        v = [us for t, us in wins if a <= t < b]
        if v:
            summ.append({"from_s": a, "to_s": b, "us_mean": round(sum(v) / len(v), 2), "us_min": round(min(v), 2), "n": len(v)})
            print(f"{a:5.2f}-{b:5.2f} s: {sum(v) / len(v):7.2f} us/launch (min {min(v):7.2f}, {len(v)} x 20)")
    with open(dst, "w") as f:
        json.dump({"windows": wins, "summary": summ, "smi": samples}, f)


if __name__ == "__main__":
    main()
