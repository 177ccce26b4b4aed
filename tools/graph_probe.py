"""Inter-kernel gaps of the bench loop: bench.py's workload (8 x 4K q90, two input sets
alternating) as K eager launches vs the same K launches captured once in a HIP graph
(torch.cuda.CUDAGraph over the library's launches on the capturing stream): span / K by HIP events,
settled, interleaved rounds.  Output equality of the two is checked.
Usage (GPU box): python tools/graph_probe.py [K] [ROUNDS]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import torch  # noqa: E402

import jpgx  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
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
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for i in range(4):
            jpgx.blocks_gpu(fr, p, ins[i & 1], out, 0, stream=st)
    torch.cuda.synchronize()
    ref = out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for i in range(K):
            jpgx.blocks_gpu(fr, p, ins[i & 1], out, 0, stream=st)
    torch.cuda.synchronize()

    def eager():
        for i in range(K):
            jpgx.blocks_gpu(fr, p, ins[i & 1], out, 0, stream=st)

    def span(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record(st)
            fn()
            e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / K

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        with torch.cuda.stream(st):
            eager()
        torch.cuda.synchronize()
    res = {"eager": [], "graph": []}
    for _ in range(R):
        res["eager"].append(span(eager))
        res["graph"].append(span(g.replay))
    out_ok = torch.equal(out, ref)
    for k, v in res.items():
        v.sort()
        print(f"{k:6s} us per launch (span / {K}): min {v[0]:7.2f}  med {v[len(v) // 2]:7.2f}  all {[round(x, 1) for x in v]}")
    print("graph output equal to eager:", out_ok)


if __name__ == "__main__":
    main()
