"""Nondeterminism hunt for a k_mxs build (GPU box): the library in JPGX_LIB runs the first 8 frames
of configs[3]'s golden batch REPS times; each run's frames are hashed against the golden, and a
wrong frame's differing blocks are located against the product library's output (same frames,
lib/libjpgx.so in a child process): channel, block % 8 (A-operand row group), step of the wave
(block / 8 % C), coefficient positions.  Usage: JPGX_LIB=... python tools/mxs_race.py REPS C"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
reps, C = int(sys.argv[1]), int(sys.argv[2])
gold = json.load(open(os.path.join(REPO, "tests", "golden", "big_golden.json")))["batch64_4k_q90"]
W, H, q = gold["W"], gold["H"], gold["quality"]
seeds = [f["seed"] for f in gold["frames"][:8]]
want = [f["coef_sha256"] for f in gold["frames"][:8]]
ref_path = os.path.join(REPO, "gpurun_out", "race_ref.npy")
if not os.path.exists(ref_path):
    env = dict(os.environ, JPGX_LIB=os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "libjpgx.so"))
    subprocess.run([sys.executable, __file__, "0", str(C)], env=env, check=True)
import jpgx  # noqa: E402

nb = (W // 8) * (H // 8)
d_in = torch.empty(8 * W * H * 3, dtype=torch.uint8, device="cuda")
for i, s in enumerate(seeds):
    jpgx.gen_splitmix_gpu(d_in[i * W * H * 3:(i + 1) * W * H * 3], s)
out = torch.empty((8, 3, nb, 64), dtype=torch.int16, device="cuda")
fr = jpgx.frames(W, H, nframes=8)
p = jpgx.default_params(W, H, q)
if reps == 0:
    jpgx.blocks_gpu(fr, p, d_in, out, 0)
    got = out.cpu().numpy()
    assert [hashlib.sha256(g.astype("<i2").tobytes()).hexdigest() for g in got] == want
    np.save(ref_path, got)
    sys.exit(0)
ref = np.load(ref_path)
nbad = 0
for r in range(reps):
    out.fill_(0)
    jpgx.blocks_gpu(fr, p, d_in, out, 0)
    got = out.cpu().numpy()
    for f in range(8):
        if hashlib.sha256(got[f].astype("<i2").tobytes()).hexdigest() == want[f]:
            continue
        nbad += 1
        bad = np.argwhere((got[f] != ref[f]).any(axis=2))
        print(f"run {r} frame {f}: {len(bad)} wrong blocks")
        for c, b in bad[:8]:
            g = f * nb + b                                  # launch-global block
            pos = np.flatnonzero(got[f, c, b] != ref[f, c, b])
            print(f"   ch {c} block {b} (b%8 {g % 8}, step-of-wave {g // 8 % C}) zz {pos[:12].tolist()} "
                  f"got {got[f, c, b, pos[:4]].tolist()} want {ref[f, c, b, pos[:4]].tolist()}")
print(f"{reps} runs x 8 frames: {nbad} wrong frames")
