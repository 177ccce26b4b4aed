"""ctypes view of include/jpgx_compat.h: the reference-compatible Block API, the JpgData
adapter, the DC recurrence, the BMP reader and the encode stage sequence (all in libjpgx.so).

Reference mapping (matthewT53/JPEG-Encoder-and-Decoder):
    Block, new_block ... destroy_block  <- src/block.c:15-67
    dct_block                           <- src/dct.c:36-59
    quantise_block / quantise_lum/chr   <- src/quantise.c:52-72 (transposed table use)
    scale_table_inplace                 <- src/quantise.c:74-86
    zig_zag_block                       <- src/zig_zag.c:48-58
    JpegData, fill_jpgdata, dpcm        <- src/headers/jpg_encode.h:21-70, src/zig_zag.c:24-32,
                                           src/dpcm.c:6-21
    bmp_read                            <- src/bitmap.c:41-152
    encode_bmp                          <- encode_bmp_to_jpeg, src/jpg_encode.c:19-47
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import JpgxError, lib

c_int_p = ctypes.POINTER(ctypes.c_int)


class BlockStruct(ctypes.Structure):
    _fields_ = [("values", ctypes.c_double * 64)]


BlockPtr = ctypes.POINTER(BlockStruct)


class HuffmanData(ctypes.Structure):
    _fields_ = [("freq", ctypes.c_int * 257), ("code_len", ctypes.c_int * 257),
                ("others", ctypes.c_int * 257), ("bits", ctypes.c_int * 32),
                ("huffval", ctypes.c_int * 256)]


class JpegData(ctypes.Structure):
    _fields_ = [("output_filename", ctypes.c_char_p), ("input_filename", ctypes.c_char_p),
                ("width", ctypes.c_int), ("height", ctypes.c_int),
                ("sample_ratio", ctypes.c_int), ("quality", ctypes.c_int),
                ("num_blocks_Y", ctypes.c_int), ("num_blocks_Cb", ctypes.c_int),
                ("num_blocks_Cr", ctypes.c_int),
                ("Y", ctypes.POINTER(BlockPtr)), ("Cb", ctypes.POINTER(BlockPtr)),
                ("Cr", ctypes.POINTER(BlockPtr)),
                ("zig_zag_Y", ctypes.POINTER(c_int_p)), ("zig_zag_Cb", ctypes.POINTER(c_int_p)),
                ("zig_zag_Cr", ctypes.POINTER(c_int_p)),
                ("lum_DC", HuffmanData), ("lum_AC", HuffmanData),
                ("chrom_DC", HuffmanData), ("chrom_AC", HuffmanData)]


def _setup(L):
    d, i, vp = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
    L.jpgx_new_block.restype = BlockPtr
    L.jpgx_new_block.argtypes = []
    L.jpgx_get_value_block.restype = d
    L.jpgx_get_value_block.argtypes = [BlockPtr, i, i]
    L.jpgx_set_value_block.restype = None
    L.jpgx_set_value_block.argtypes = [BlockPtr, i, i, d]
    L.jpgx_copy_block.restype = BlockPtr
    L.jpgx_copy_block.argtypes = [BlockPtr]
    for f in ("jpgx_show_block", "jpgx_destroy_block", "jpgx_dct_block", "jpgx_quantise_lum",
              "jpgx_quantise_chr"):
        getattr(L, f).restype = None
        getattr(L, f).argtypes = [BlockPtr]
    L.jpgx_quantise_block.restype = None
    L.jpgx_quantise_block.argtypes = [BlockPtr, vp]
    L.jpgx_scale_table_inplace.restype = None
    L.jpgx_scale_table_inplace.argtypes = [vp, i]
    L.jpgx_zig_zag_block.restype = None
    L.jpgx_zig_zag_block.argtypes = [BlockPtr, vp]
    J = ctypes.POINTER(JpegData)
    L.jpgx_fill_jpgdata.argtypes = [J, vp]
    L.jpgx_free_jpgdata.restype = None
    L.jpgx_free_jpgdata.argtypes = [J]
    L.jpgx_dpcm.restype = None
    L.jpgx_dpcm.argtypes = [J]
    L.jpgx_dpcm_dc.argtypes = [vp, ctypes.c_size_t, vp, vp]
    L.jpgx_bmp_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp), c_int_p, c_int_p,
                                ctypes.POINTER(ctypes.c_size_t)]
    L.jpgx_free.restype = None
    L.jpgx_free.argtypes = [vp]
    L.jpgx_encode_bmp.argtypes = [ctypes.c_char_p, i, i, i, i, J]
    L.jpgx_jfif_bound.restype = ctypes.c_size_t
    L.jpgx_jfif_bound.argtypes = [i, i]
    L.jpgx_write_jfif.argtypes = [vp, i, i, i, vp, ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.c_size_t)]
    L.jpgx_encode_bmp_to_jpeg.argtypes = [ctypes.c_char_p, ctypes.c_char_p, i, i]
    L.jpgx_write_jfif_ex.argtypes = [vp, i, i, i, i, i, i, vp, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_size_t)]
    L.jpgx_encode_rgb_to_jpeg.argtypes = [vp, i, i, ctypes.c_size_t, ctypes.c_char_p, i, i,
                                          ctypes.c_uint, i]


_setup(lib)


def _check(rc, what):
    if rc != 0:
        raise JpgxError(rc, what)


class Block:
    """One reference Block (64 doubles, values[y*8+x]) owned by libjpgx."""

    def __init__(self, values=None):
        self.ptr = lib.jpgx_new_block()
        if values is not None:
            v = np.asarray(values, np.float64).reshape(64)
            for k in range(64):
                self.ptr.contents.values[k] = float(v[k])

    def __del__(self):
        if getattr(self, "ptr", None):
            lib.jpgx_destroy_block(self.ptr)
            self.ptr = None

    @classmethod
    def _wrap(cls, ptr):
        b = cls.__new__(cls)
        b.ptr = ptr
        return b

    def get(self, x, y):
        return lib.jpgx_get_value_block(self.ptr, x, y)

    def set(self, x, y, v):
        lib.jpgx_set_value_block(self.ptr, x, y, v)

    def copy(self):
        return Block._wrap(lib.jpgx_copy_block(self.ptr))

    def show(self):
        lib.jpgx_show_block(self.ptr)

    def values(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.ptr.contents.values).copy()

    def dct(self):
        lib.jpgx_dct_block(self.ptr)

    def quantise(self, table):
        t = np.ascontiguousarray(table, np.int32)
        lib.jpgx_quantise_block(self.ptr, t.ctypes.data)

    def quantise_lum(self):
        lib.jpgx_quantise_lum(self.ptr)

    def quantise_chr(self):
        lib.jpgx_quantise_chr(self.ptr)

    def zig_zag(self) -> np.ndarray:
        zz = np.zeros(64, np.int32)
        lib.jpgx_zig_zag_block(self.ptr, zz.ctypes.data)
        return zz


def legacy_table(which: int) -> np.ndarray:
    """A live numpy view of jpgx_q_table_lum (0) / jpgx_q_table_chr (1)."""
    name = "jpgx_q_table_lum" if which == 0 else "jpgx_q_table_chr"
    arr = (ctypes.c_int * 64).in_dll(lib, name)
    return np.ctypeslib.as_array(arr).reshape(8, 8)


def scale_table_inplace(table: np.ndarray, quality: int) -> None:
    assert table.dtype == np.int32 and table.flags.c_contiguous and table.shape == (8, 8)
    lib.jpgx_scale_table_inplace(table.ctypes.data, quality)


def dpcm_dc(coef: np.ndarray, carry=(0, 0, 0)) -> np.ndarray:
    coef = np.ascontiguousarray(coef, np.int16)
    nb = coef.shape[1]
    dc = np.empty((3, nb), np.int32)
    c = np.asarray(carry, np.int32)
    _check(lib.jpgx_dpcm_dc(coef.ctypes.data, nb, c.ctypes.data, dc.ctypes.data), "jpgx_dpcm_dc")
    return dc


def jpgdata_from_coef(width: int, height: int, coef: np.ndarray) -> JpegData:
    j = JpegData()
    j.width, j.height = width, height
    coef = np.ascontiguousarray(coef, np.int16)
    _check(lib.jpgx_fill_jpgdata(ctypes.byref(j), coef.ctypes.data), "jpgx_fill_jpgdata")
    return j


def jpgdata_zigzag(j: JpegData) -> np.ndarray:
    """zig_zag_{Y,Cb,Cr} -> int32 [3][nb][64]"""
    nb = j.num_blocks_Y
    out = np.empty((3, nb, 64), np.int32)
    for c, rows in enumerate((j.zig_zag_Y, j.zig_zag_Cb, j.zig_zag_Cr)):
        for i in range(nb):
            out[c, i] = np.ctypeslib.as_array(rows[i], shape=(64,))
    return out


def dpcm(j: JpegData) -> None:
    lib.jpgx_dpcm(ctypes.byref(j))


def free_jpgdata(j: JpegData) -> None:
    lib.jpgx_free_jpgdata(ctypes.byref(j))


def bmp_read(path: str):
    """-> (rgb [H][W][3] uint8, file_size)"""
    p = ctypes.c_void_p()
    w, h, fs = ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
    _check(lib.jpgx_bmp_read(path.encode(), ctypes.byref(p), ctypes.byref(w), ctypes.byref(h),
                             ctypes.byref(fs)), "jpgx_bmp_read")
    n = w.value * h.value * 3
    out = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(n,)).copy()
    lib.jpgx_free(p)
    return out.reshape(h.value, w.value, 3), fs.value


def encode_bmp(path: str, quality: int, sample_ratio: int = 0, device: int = 0,
               do_dpcm: bool = False) -> JpegData:
    j = JpegData()
    j._path = path.encode()             # j.input_filename points at it (jpg_encode.c:29)
    _check(lib.jpgx_encode_bmp(j._path, quality, sample_ratio, device, int(do_dpcm),
                               ctypes.byref(j)), "jpgx_encode_bmp")
    return j


def write_jfif(coef: np.ndarray, width: int, height: int, quality: int) -> bytes:
    """int16 [3][nb][64] -> baseline JFIF bytes (jpgx_write_jfif)."""
    coef = np.ascontiguousarray(coef, np.int16)
    cap = lib.jpgx_jfif_bound(width, height)
    buf = (ctypes.c_uint8 * cap)()
    n = ctypes.c_size_t()
    _check(lib.jpgx_write_jfif(coef.ctypes.data, width, height, quality,
                               ctypes.cast(buf, ctypes.c_void_p), cap, ctypes.byref(n)),
           "jpgx_write_jfif")
    return bytes(buf[:n.value])


def write_jfif_ex(coef: np.ndarray, width: int, height: int, quality: int, sample_ratio: int = 0,
                  restart_rows: int = -1, nthreads: int = 0, cap: int | None = None) -> bytes:
    """jpgx_write_jfif_ex: restart intervals of `restart_rows` MCU rows (-1 auto, 0 none) coded on
    `nthreads` host threads (0: one per CPU).  `cap`: output buffer size (default: grown on
    demand from the size the library reports)."""
    coef = np.ascontiguousarray(coef, np.int16)
    n = ctypes.c_size_t()
    cap = cap or max(1 << 20, coef.size // 2)
    for _ in range(2):
        buf = np.empty(cap, np.uint8)
        rc = lib.jpgx_write_jfif_ex(coef.ctypes.data, width, height, quality, sample_ratio,
                                    restart_rows, nthreads, buf.ctypes.data, cap, ctypes.byref(n))
        if rc == 0:
            return buf[:n.value].tobytes()
        if rc != -4 or n.value <= cap:                      # JPGX_EARG with the size needed
            break
        cap = n.value
    _check(rc, "jpgx_write_jfif_ex")
    raise JpgxError(rc, "jpgx_write_jfif_ex")


def write_jfif_sub(coef: np.ndarray, width: int, height: int, quality: int,
                   sample_ratio: int) -> bytes:
    """Y|Cb|Cr blocks of the JPGX_FLAG_SUBSAMPLE layout -> 4:2:2 / 4:2:0 JFIF bytes."""
    coef = np.ascontiguousarray(coef, np.int16)
    cap = lib.jpgx_jfif_bound(width, height)
    buf = (ctypes.c_uint8 * cap)()
    n = ctypes.c_size_t()
    _check(lib.jpgx_write_jfif_sub(ctypes.c_void_p(coef.ctypes.data), width, height, quality,
                                   sample_ratio, ctypes.cast(buf, ctypes.c_void_p),
                                   ctypes.c_size_t(cap), ctypes.byref(n)),
           "jpgx_write_jfif_sub")
    return bytes(buf[:n.value])


def encode_bmp_to_jpeg_ex(src: str, dst: str, quality: int, sample_ratio: int, flags: int,
                          device: int = 0) -> None:
    _check(lib.jpgx_encode_bmp_to_jpeg_ex(src.encode(), dst.encode(), quality, sample_ratio,
                                          ctypes.c_uint(flags), device),
           "jpgx_encode_bmp_to_jpeg_ex")


def encode_bmp_to_jpeg(src: str, dst: str, quality: int, sample_ratio: int = 0) -> None:
    _check(lib.jpgx_encode_bmp_to_jpeg(src.encode(), dst.encode(), quality, sample_ratio),
           "jpgx_encode_bmp_to_jpeg")


def encode_rgb_to_jpeg(rgb: np.ndarray, dst: str, quality: int, sample_ratio: int = 0,
                       flags: int = 0, device: int = 0) -> None:
    """In-memory (H, W, 3) uint8 image -> JFIF file (jpgx_encode_rgb_to_jpeg)."""
    if rgb.dtype != np.uint8 or rgb.ndim != 3 or rgb.strides[1:] != (3, 1):
        raise ValueError("rgb must be (H, W, 3) uint8 with packed pixels")
    H, W = rgb.shape[:2]
    _check(lib.jpgx_encode_rgb_to_jpeg(rgb.ctypes.data, W, H, rgb.strides[0], dst.encode(),
                                       quality, sample_ratio, ctypes.c_uint(flags), device),
           "jpgx_encode_rgb_to_jpeg")
