"""Time k_xform variants (lib/variants/libjpgx_*.so) in one process each, interleaved rounds.
Each variant is checked bit-exact against the default library's output before timing.
Usage (GPU box): python tools/variant_bench.py [names...]"""
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "variants")

CHILD = r'''
import os, sys, json
sys.path.insert(0, os.path.join(%(repo)r, "jpeg-encoder-and-decoder_amd"))
import torch, jpgx, hashlib
W, H, q = 3840, 2160, 90
F = int(os.environ.get("VB_FRAMES", "8"))       # 16+: input beyond the 256 MiB Infinity Cache
sr = int(os.environ.get("VB_SUB", "0"))          # 1 / 2: true 4:2:2 / 4:2:0 at q75
fl = jpgx.FLAG_SUBSAMPLE if sr else 0
q = 75 if sr else q
dev = torch.device("cuda:0")
d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device=dev)
for f in range(F):
    jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
nb = (W // 8) * (H // 8)
per = nb + 2 * jpgx.chroma_blocks(W, 0, H // 8, sr, fl)
out = torch.empty((F, per, 64), dtype=torch.int16, device=dev)
fr = jpgx.frames(W, H, nframes=F, out_frame_stride=per * 64)
ws = torch.empty(max(jpgx.workspace_size(fr), 1), dtype=torch.uint8, device=dev)
p = jpgx.default_params(W, H, q, sr, flags=fl)
import time
t0 = time.perf_counter()                          # settle: the GPU's ramp out of idle
while time.perf_counter() - t0 < 0.2:
    for _ in range(5):
        jpgx.blocks_gpu(fr, p, d_in, out, ws)
    torch.cuda.synchronize()
h = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()
ts = []
for r in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        jpgx.blocks_gpu(fr, p, d_in, out, ws)
    e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10)
print(json.dumps({"hash": h, "ms": sorted(ts)}))
'''


def run(lib):
    env = dict(os.environ, JPGX_LIB=lib)
    if lib.endswith("#xform"):             # the test-only cross-check library (k_xform)
        env.update(JPGX_LIB=os.path.join(os.path.dirname(lib.split("#")[0]), "libjpgx_alt.so"))
    elif "#" in lib:
        env.update(JPGX_LIB=lib.split("#")[0])
    r = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO}], env=env, capture_output=True,
                       text=True, timeout=300)
    if r.returncode:
        return {"error": r.stderr[-500:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    names = sys.argv[1:] or sorted(os.path.basename(p)[8:-3] for p in glob.glob(f"{VAR}/libjpgx_*.so"))
    libs = {"default": os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "libjpgx.so")}
    libs.update({n: f"{VAR}/libjpgx_{n}.so" + ("#mx" if n.startswith("mx") else "") for n in names if n not in ("default", "xform", "mx")})
    for k in ("xform", "mx"):
        if k in names:
            libs[k] = libs["default"] + "#" + k
    res = {}
    for rnd in range(int(os.environ.get("VB_ROUNDS", "2"))):   # interleaved rounds
        for n, lib in libs.items():
            r = run(lib)
            res.setdefault(n, []).append(r)
    ref = res["default"][0].get("hash")
    sr = int(os.environ.get("VB_SUB", "0"))
    bytes_moved = int(os.environ.get("VB_FRAMES", "8")) * 3840 * 2160 * (9 if sr == 0 else (7 if sr == 1 else 6))
    for n, rs in res.items():
        ms = sorted(m for r in rs for m in r.get("ms", []))
        ok = all(r.get("hash") == ref for r in rs)
        if not ms:
            print(f"{n:24s} ERROR {rs[0].get('error')}")
            continue
        print(f"{n:24s} median {ms[len(ms)//2]:.4f} ms  min {ms[0]:.4f}  "
              f"{bytes_moved / ms[0] / 1e6:.0f} GB/s  exact={'yes' if ok else 'NO'}", flush=True)


if __name__ == "__main__":
    main()
