"""Exact-pass statistics of k_mx (a -DJX_MX_DBG_COUNT build) on the bench workload.
Needs the measurement hooks: git apply tools/probes/k_mx_debug_knobs.patch, then build the
variant with -DJX_MX_DBG_COUNT (tools/build_variants.sh).
"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["JPGX_LIB"] = os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "variants",
                                      "libjpgx_mxCount.so")
sys.path.insert(0, os.path.join(REPO, "jpeg-encoder-and-decoder_amd"))
import jpgx  # noqa: E402

W, H, F = 3840, 2160, 8
rd = jpgx.lib.jx_mx_dbg_read
rd.argtypes = [ctypes.c_void_p]
for q in (50, 90):
    d_in = torch.empty(F * W * H * 3, dtype=torch.uint8, device="cuda")
    for f in range(F):
        jpgx.gen_splitmix_gpu(d_in[f * W * H * 3:(f + 1) * W * H * 3], 1000 + f)
    nb = (W // 8) * (H // 8)
    out = torch.empty((F, 3, nb, 64), dtype=torch.int16, device="cuda")
    fr = jpgx.frames(W, H, nframes=F)
    ws = torch.empty(jpgx.workspace_size(fr), dtype=torch.uint8, device="cuda")
    buf = (ctypes.c_ulonglong * 4)()
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q), d_in, out, ws)
    rd(buf)
    jpgx.blocks_gpu(fr, jpgx.default_params(W, H, q), d_in, out, ws)
    rd(buf)
    steps = F * nb // 8
    print(f"q{q}: steps {steps} flushes {buf[0]} ({buf[0] / steps:.4f}/step) deferred tasks {buf[1]} "
          f"({buf[1] / steps:.3f}/step) inline passes {buf[2]}")
