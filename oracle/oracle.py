"""ctypes view of oracle/cpu_ref.c -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / the timed CPU baseline.  The product (jpeg-encoder-and-decoder_amd/)
never imports it.  Reference map: see oracle/cpu_ref.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libcpuref.so")
REF_DIR = os.path.join(HERE, "_ref")

MODE_TABLE = 0
MODE_REFCOST = 1

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.cpuref_blocks_rows.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_int16)]
        L.cpuref_blocks_rows.restype = ctypes.c_int
        L.cpuref_glibc_underflow.argtypes = [ctypes.c_longlong, ctypes.c_longlong, u8p]
        L.cpuref_gen_splitmix.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, u8p]
        L.cpuref_gen_tie.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.cpuref_bmp_decode.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int), u8p]
        L.cpuref_bmp_decode.restype = ctypes.c_int
        L.cpuref_dct_block.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.cpuref_quantise_block.argtypes = [ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_int)]
        L.cpuref_zigzag_block.argtypes = [ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_int)]
        L.cpuref_scale_table.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_int)]
        L.cpuref_dpcm_i32.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.c_long]
        L.cpuref_chroma_sub_rows.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int16)]
        L.cpuref_chroma_sub_rows.restype = ctypes.c_int
        L.cpuref_chroma_sample.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_long, ctypes.c_long]
        L.cpuref_chroma_sample.restype = ctypes.c_double
        L.cpuref_entropy_stats.argtypes = [ctypes.POINTER(ctypes.c_int16), ctypes.c_long,
                                           ctypes.c_long, ctypes.POINTER(ctypes.c_int32),
                                           ctypes.POINTER(ctypes.c_int32)]
        L.cpuref_entropy_stats.restype = None
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def glibc_underflow(n_pixels: int, file_size: int | None = None) -> np.ndarray:
    if file_size is None:
        file_size = 54 + 3 * n_pixels
    out = np.zeros(8, np.uint8)
    lib().cpuref_glibc_underflow(n_pixels, file_size, _u8(out))
    return out


def gen_splitmix(seed: int, W: int, H: int) -> np.ndarray:
    out = np.empty((H, W, 3), np.uint8)
    lib().cpuref_gen_splitmix(seed, W, H, _u8(out))
    return out


def gen_tie(W: int, H: int) -> np.ndarray:
    out = np.empty((H, W, 3), np.uint8)
    lib().cpuref_gen_tie(W, H, _u8(out))
    return out


def blocks(rgb: np.ndarray, quality: int, sample_ratio: int = 0, underflow=None,
           mode: int = MODE_TABLE, nthreads: int = 0, rows: tuple[int, int] | None = None,
           pitch: int | None = None) -> np.ndarray:
    """int16 [3][nb][64] zig-zag coefficients of block-rows `rows` (default: all)."""
    H, W = rgb.shape[0], rgb.shape[1]
    rgb = np.ascontiguousarray(rgb)
    if pitch is None:
        pitch = W * 3
    if underflow is None:
        underflow = glibc_underflow(W * H)
    underflow = np.asarray(underflow, np.uint8)
    if underflow.shape == (8,):          # same chunk word in front of all three planes
        underflow = np.tile(underflow, (3, 1))
    underflow = np.ascontiguousarray(underflow.reshape(3, 8))
    r0, r1 = rows if rows is not None else (0, H // 8)
    nb = max(r1 - r0, 0) * (W // 8)
    out = np.empty((3, nb, 64), np.int16)
    rc = lib().cpuref_blocks_rows(_u8(rgb), W, H, pitch, quality, sample_ratio, _u8(underflow),
                                  mode, nthreads, r0, r1,
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
    if rc != 0:
        raise ValueError(f"cpuref_blocks_rows failed: {rc}")
    return out


def chroma_sub(rgb: np.ndarray, quality: int, sample_ratio: int, mode: int = MODE_TABLE,
               nthreads: int = 0, crows: tuple[int, int] | None = None) -> np.ndarray:
    """int16 [2][nbc][64]: true 4:2:2 (sample_ratio 1) / 4:2:0 (2) Cb, Cr blocks (EXTENSION,
    semantics defined by cpu_ref.h, parity with the reference unpinned)."""
    H, W = rgb.shape[0], rgb.shape[1]
    rgb = np.ascontiguousarray(rgb)
    Hc = H // 2 if sample_ratio == 2 else H
    r0, r1 = crows if crows is not None else (0, Hc // 8)
    nbc = max(r1 - r0, 0) * (W // 16)
    out = np.empty((2, nbc, 64), np.int16)
    rc = lib().cpuref_chroma_sub_rows(_u8(rgb), W, H, W * 3, quality, sample_ratio, mode, nthreads,
                                      r0, r1, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
    if rc != 0:
        raise ValueError(f"cpuref_chroma_sub_rows failed: {rc}")
    return out


def entropy_stats(coef: np.ndarray, nb_y: int | None = None, nb_c: int | None = None):
    """(dc int32 [nb_y + 2 nb_c], hist int32 [4][257]) of huffman.c's frequency pass over
    the dpcm'd blocks (cpu_ref.h).  coef: [3][nb][64] or a flat [nb_y + 2 nb_c][64]."""
    c = np.ascontiguousarray(coef, np.int16).reshape(-1, 64)
    if nb_y is None:
        nb_y = nb_c = c.shape[0] // 3
    dc = np.empty(nb_y + 2 * nb_c, np.int32)
    hist = np.empty((4, 257), np.int32)
    lib().cpuref_entropy_stats(c.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), nb_y, nb_c,
                               dc.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                               hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return dc, hist


def bmp_decode(data: bytes) -> np.ndarray:
    buf = np.frombuffer(data, np.uint8).copy()
    W, H = ctypes.c_int(), ctypes.c_int()
    if lib().cpuref_bmp_decode(_u8(buf), len(buf), ctypes.byref(W), ctypes.byref(H), None):
        raise ValueError("bad bmp")
    out = np.empty((H.value, W.value, 3), np.uint8)
    lib().cpuref_bmp_decode(_u8(buf), len(buf), ctypes.byref(W), ctypes.byref(H), _u8(out))
    return out


def dct_block(v: np.ndarray, mode: int = MODE_TABLE) -> np.ndarray:
    a = np.ascontiguousarray(v, np.float64).copy().reshape(64)
    lib().cpuref_dct_block(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), mode)
    return a


def scale_table(base: np.ndarray, quality: int) -> np.ndarray:
    b = np.ascontiguousarray(base, np.int32)
    out = np.empty((8, 8), np.int32)
    lib().cpuref_scale_table(b.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), quality,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    return out


def quantise_block(v: np.ndarray, table: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(v, np.float64).copy().reshape(64)
    t = np.ascontiguousarray(table, np.int32)
    lib().cpuref_quantise_block(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                t.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    return a


def zigzag_block(v: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(v, np.float64).reshape(64)
    out = np.empty(64, np.int32)
    lib().cpuref_zigzag_block(a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    return out


def dpcm(coef: np.ndarray) -> np.ndarray:
    """dpcm.c:6-21 on int [3][nb][64]; returns an int32 copy."""
    a = np.ascontiguousarray(coef, np.int32).copy()
    for c in range(a.shape[0]):
        lib().cpuref_dpcm_i32(a[c].ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), a.shape[1])
    return a


# ---- helpers around the real reference binaries (this container only) --------------------
def write_bmp(path: str, rgb: np.ndarray) -> None:
    """24-bit bottom-up BMP, 54-byte header, no row padding needed (W*3 % 4 == 0 asserted),
    no trailing bytes: the reference loader (bitmap.c:129-137) then reads it back exactly."""
    H, W = rgb.shape[:2]
    assert (W * 3) % 4 == 0
    data = np.ascontiguousarray(rgb[::-1]).tobytes()
    fs = 54 + len(data)
    hdr = bytearray(54)
    hdr[0:2] = b"BM"
    hdr[2:6] = fs.to_bytes(4, "little")
    hdr[10:14] = (54).to_bytes(4, "little")
    hdr[14:18] = (40).to_bytes(4, "little")
    hdr[18:22] = W.to_bytes(4, "little")
    hdr[22:26] = H.to_bytes(4, "little")
    hdr[26:28] = (1).to_bytes(2, "little")
    hdr[28:30] = (24).to_bytes(2, "little")
    hdr[34:38] = len(data).to_bytes(4, "little")
    with open(path, "wb") as f:
        f.write(bytes(hdr) + data)


def ref_available() -> bool:
    return os.path.exists(os.path.join(REF_DIR, "ref_dump"))


def ref_dump(bmp_path: str, quality: int, sample_ratio: int = 0, dpcm_: bool = False,
             tmp_out: str | None = None, want_underflow: bool = False):
    """Run the real reference (compiled by `make -C oracle ref`) on a BMP file.
    With want_underflow also return the [3][8] bytes glibc left in front of r_new, g_new,
    b_new (recorded by the harness's malloc wrapper, oracle/ref_harness.c)."""
    import tempfile
    exe = os.path.join(REF_DIR, "ref_dump")
    with open(bmp_path, "rb") as f:
        hdr = f.read(26)
    n = int.from_bytes(hdr[18:22], "little") * int.from_bytes(hdr[22:26], "little")
    env = dict(os.environ, REF_WATCH_PIXELS=str(n))
    with tempfile.TemporaryDirectory() as td:
        out = tmp_out or os.path.join(td, "out.bin")
        args = [exe, bmp_path, out, str(quality), str(sample_ratio)] + (["1"] if dpcm_ else [])
        r = subprocess.run(args, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           env=env, text=True)
        a = np.fromfile(out, np.int32).reshape(3, -1, 64)
    if not want_underflow:
        return a
    seen = [bytes.fromhex(l.split("=")[1]) for l in r.stderr.split() if l.startswith("pre[")]
    uf = np.frombuffer(b"".join(seen[-3:]), np.uint8).reshape(3, 8).copy()
    return a, uf
