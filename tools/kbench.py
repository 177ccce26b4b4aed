"""Time variant libraries (lib/variants/libjpgx_NAME.so; "product" = lib/libjpgx.so) on the bench
workload with fresh input (8 x 4K q90, two input sets alternating, settled 300 ms): HIP-event
us per launch (min / median of 5 x 20), fraction of 8 TB/s at 9 B/px, and whether the output
of frame set 0 equals the product library's.  One process per library, interleaved rounds.
Usage (GPU box): python tools/kbench.py [ROUNDS] name ..."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time, hashlib
sys.path.insert(0, os.path.join(%(repo)r, "jpeg-encoder-and-decoder_amd"))
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
for r in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        jpgx.blocks_gpu(fr, p, ins[i & 1], out, ws); i += 1
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3 / 20)
print(json.dumps({"hash": h, "us": sorted(ts)}))
'''


def lib_path(n):
    if n == "product":
        return os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "libjpgx.so")
    return os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "variants", f"libjpgx_{n}.so")


def main():
    args = sys.argv[1:]
    rounds = int(args.pop(0)) if args and args[0].isdigit() else 2
    names = args
    sr = int(os.environ.get("KB_SUB", "0"))
    bpp = 9 if sr == 0 else (7 if sr == 1 else 6)
    res = {}
    for _ in range(rounds):
        for n in ["product"] + [x for x in names if x != "product"]:
            env = dict(os.environ, JPGX_LIB=lib_path(n))
            r = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO}], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode:
                print(n, "ERROR", r.stderr[-400:], flush=True)
                continue
            res.setdefault(n, []).append(json.loads(r.stdout.strip().splitlines()[-1]))
            d = res[n][-1]
            print(f"{n:12s} min {d['us'][0]:7.1f} us  med {d['us'][2]:7.1f}  frac(min) "
                  f"{8 * 3840 * 2160 * bpp / (d['us'][0] * 1e-6) / 8e12:.4f}  "
                  f"same-as-product={d['hash'] == res['product'][0]['hash']}", flush=True)


if __name__ == "__main__":
    main()
