"""jpgx -- Python view of libjpgx.so, the MI355X-native JPEG block-transform hot path.

Everything here calls through the C ABI declared in include/jpgx.h; there is no Python or
CPU implementation of the transform in this package.  If the shared library is missing the
import fails loudly (ImportError) instead of falling back.

Reference mapping (matthewT53/JPEG-Encoder-and-Decoder):
    blocks_gpu / blocks   <- preprocess_jpeg + chroma_subsample + dct + quantise + zig_zag
                             (src/jpg_encode.c:32-44), output = JpgData.zig_zag_{Y,Cb,Cr}
    default_params        <- encode_bmp_to_jpeg(quality, sample_ratio) (src/jpg_encode.c:19)
    scale_table           <- scale_table (src/quantise.c:74-86)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("JPGX_LIB") or os.path.join(PKG_ROOT, "lib", "libjpgx.so")

NO_CHROMA_SUBSAMPLING = 0
HORIZONTAL_SUBSAMPLING = 1
HORIZONTAL_VERTICAL_SUBSAMPLING = 2
FLAG_FORCE_EXACT = 1
FLAG_SUBSAMPLE = 2      # true 4:2:2 / 4:2:0 chroma (extension; see include/jpgx.h)

OK, EGEOMETRY, EQUALITY, ESAMPLE, EARG, EHIP, EWORKSPACE, ENODEV, ENOMEM = 0, -1, -2, -3, -4, -5, -6, -7, -8
_ERRNAMES = {-1: "EGEOMETRY", -2: "EQUALITY", -3: "ESAMPLE", -4: "EARG", -5: "EHIP",
             -6: "EWORKSPACE", -7: "ENODEV", -8: "ENOMEM"}

# every function include/jpgx.h and include/jpgx_compat.h declare (tests check the library
# exports them all)
EXPORTS = [
    "jpgx_validate", "jpgx_default_params", "jpgx_glibc_underflow", "jpgx_scale_table",
    "jpgx_guard_band", "jpgx_workspace_size", "jpgx_blocks_gpu", "jpgx_blocks_gpu_ev",
    "jpgx_blocks_gpu_timed",
    "jpgx_gen_splitmix_gpu",
    "jpgx_gen_tie_gpu", "jpgx_blocks", "jpgx_blocks_multi", "jpgx_stripe",
    "jpgx_device_count", "jpgx_version", "jpgx_chroma_blocks", "jpgx_entropy_workspace_size",
    "jpgx_entropy_stats_gpu", "jpgx_entropy_workspace_size_batch", "jpgx_entropy_stats_gpu_batch",
    "jpgx_host_create", "jpgx_host_destroy", "jpgx_host_blocks",
    "jpgx_host_register", "jpgx_host_unregister", "jpgx_host_release",
]
COMPAT_EXPORTS = [
    "jpgx_new_block", "jpgx_get_value_block", "jpgx_set_value_block", "jpgx_copy_block",
    "jpgx_show_block", "jpgx_destroy_block", "jpgx_dct_block", "jpgx_quantise_block",
    "jpgx_quantise_lum", "jpgx_quantise_chr", "jpgx_scale_table_inplace", "jpgx_zig_zag_block",
    "jpgx_fill_jpgdata", "jpgx_free_jpgdata", "jpgx_dpcm", "jpgx_dpcm_dc", "jpgx_bmp_read",
    "jpgx_free", "jpgx_encode_bmp", "jpgx_jfif_bound", "jpgx_write_jfif",
    "jpgx_encode_bmp_to_jpeg", "jpgx_write_jfif_sub", "jpgx_encode_bmp_to_jpeg_ex",
    "jpgx_encode_rgb_to_jpeg", "jpgx_write_jfif_ex",
]


class JpgxError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what} failed: {_ERRNAMES.get(rc, rc)}")
        self.rc = rc


class Params(ctypes.Structure):
    _fields_ = [("quality", ctypes.c_int), ("sample_ratio", ctypes.c_int),
                ("flags", ctypes.c_uint), ("underflow", (ctypes.c_uint8 * 8) * 3)]


class Frames(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int),
                ("row_begin", ctypes.c_int), ("row_end", ctypes.c_int),
                ("nframes", ctypes.c_int), ("in_pitch", ctypes.c_size_t),
                ("in_frame_stride", ctypes.c_size_t), ("out_frame_stride", ctypes.c_size_t)]


ALT_LIB_PATH = os.path.join(PKG_ROOT, "lib", "libjpgx_alt.so")


def _load(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(f"{os.path.basename(path)} not built ({path}); run __graft_entry__.build()")
    # libjpgx.so and torch both need libamdhip64.so.7 (same soname): load torch first so the
    # process has ONE HIP runtime and device pointers/streams are shared.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    vp, sz, i, u8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p
    P, Fp = ctypes.POINTER(Params), ctypes.POINTER(Frames)
    L.jpgx_validate.argtypes = [i, i, P]
    L.jpgx_default_params.argtypes = [P, i, i, i, i]
    L.jpgx_default_params.restype = None
    L.jpgx_glibc_underflow.argtypes = [ctypes.c_longlong, ctypes.c_longlong, u8p]
    L.jpgx_glibc_underflow.restype = None
    L.jpgx_scale_table.argtypes = [i, i, vp]
    L.jpgx_guard_band.argtypes = [i, vp, vp]
    L.jpgx_workspace_size.argtypes = [Fp]
    L.jpgx_workspace_size.restype = sz
    L.jpgx_blocks_gpu.argtypes = [Fp, P, vp, vp, vp, sz, vp]
    L.jpgx_blocks_gpu_ev.argtypes = [Fp, P, vp, vp, vp, sz, vp, vp]
    L.jpgx_blocks_gpu_timed.argtypes = [Fp, P, vp, vp, vp, sz, vp, vp, vp]
    L.jpgx_gen_splitmix_gpu.argtypes = [vp, sz, ctypes.c_uint64, vp]
    L.jpgx_gen_tie_gpu.argtypes = [vp, i, i, vp]
    L.jpgx_blocks.argtypes = [vp, i, i, sz, P, vp, i]
    L.jpgx_blocks_multi.argtypes = [vp, i, i, sz, P, vp, i]
    L.jpgx_stripe.argtypes = [i, i, i, ctypes.POINTER(i), ctypes.POINTER(i)]
    L.jpgx_stripe.restype = None
    L.jpgx_device_count.argtypes = []
    L.jpgx_chroma_blocks.argtypes = [i, i, i, i, ctypes.c_uint]
    L.jpgx_chroma_blocks.restype = sz
    L.jpgx_entropy_workspace_size.argtypes = [sz, sz]
    L.jpgx_entropy_workspace_size.restype = sz
    L.jpgx_entropy_stats_gpu.argtypes = [vp, sz, sz, vp, vp, vp, vp, sz, vp]
    L.jpgx_entropy_workspace_size_batch.argtypes = [sz, sz, sz]
    L.jpgx_entropy_workspace_size_batch.restype = sz
    L.jpgx_entropy_stats_gpu_batch.argtypes = [vp, sz, sz, sz, sz, vp, vp, vp, vp, sz, vp]
    L.jpgx_version.restype = ctypes.c_char_p
    L.jpgx_host_create.argtypes = [ctypes.POINTER(vp), i, vp, i]
    L.jpgx_host_destroy.argtypes = [vp]
    L.jpgx_host_destroy.restype = None
    L.jpgx_host_blocks.argtypes = [vp, vp, i, i, sz, P, vp]
    L.jpgx_host_register.argtypes = [vp, sz]
    L.jpgx_host_unregister.argtypes = [vp]
    L.jpgx_host_release.argtypes = []
    L.jpgx_host_release.restype = None
    return L


lib = _load()
_alt = None


def alt_library() -> ctypes.CDLL:
    """The TEST-ONLY cross-check build (lib/libjpgx_alt.so: k_xform for 4:4:4, k_xform +
    k_chroma for true 4:2:x), loaded on first use.  Tests swap it in for `lib` to run every
    parity check on the second implementation; the product never loads it."""
    global _alt
    if _alt is None:
        _alt = _load(ALT_LIB_PATH)
    return _alt


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise JpgxError(rc, what)


def version() -> str:
    return lib.jpgx_version().decode()


def device_count() -> int:
    return lib.jpgx_device_count()


def glibc_underflow(n_pixels: int, bmp_file_size: int | None = None) -> bytes:
    if bmp_file_size is None:
        bmp_file_size = 54 + 3 * n_pixels
    out = (ctypes.c_uint8 * 8)()
    lib.jpgx_glibc_underflow(n_pixels, bmp_file_size, ctypes.cast(out, ctypes.c_void_p))
    return bytes(out)


def default_params(width: int, height: int, quality: int, sample_ratio: int = 0,
                   underflow=None, flags: int = 0) -> Params:
    """underflow: None (glibc default), 8 bytes (same for all planes) or [3][8] per plane."""
    p = Params()
    lib.jpgx_default_params(ctypes.byref(p), width, height, quality, sample_ratio)
    if underflow is not None:
        u = np.asarray(list(underflow) if isinstance(underflow, (bytes, bytearray))
                       else underflow, np.uint8)
        u = np.tile(u, (3, 1)) if u.shape == (8,) else u.reshape(3, 8)
        for k in range(3):
            for x in range(8):
                p.underflow[k][x] = int(u[k, x])
    p.flags = flags
    return p


def validate(width: int, height: int, params: Params) -> int:
    return lib.jpgx_validate(width, height, ctypes.byref(params))


def scale_table(which: int, quality: int) -> np.ndarray:
    out = np.zeros((8, 8), np.int32)
    _check(lib.jpgx_scale_table(which, quality, out.ctypes.data), "jpgx_scale_table")
    return out


def guard_band(quality: int) -> tuple[np.ndarray, np.ndarray]:
    w = np.zeros((3, 64), np.float32)
    lim = np.zeros((3, 64), np.float32)
    _check(lib.jpgx_guard_band(quality, w.ctypes.data, lim.ctypes.data), "jpgx_guard_band")
    return w, lim


def stripe(block_rows: int, nshards: int, k: int) -> tuple[int, int]:
    a, b = ctypes.c_int(), ctypes.c_int()
    lib.jpgx_stripe(block_rows, nshards, k, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def frames(width: int, height: int, nframes: int = 1, rows: tuple[int, int] | None = None,
           in_pitch: int | None = None, in_frame_stride: int | None = None,
           out_frame_stride: int | None = None) -> Frames:
    r0, r1 = rows if rows is not None else (0, height // 8)
    fr = Frames()
    fr.width, fr.height, fr.row_begin, fr.row_end, fr.nframes = width, height, r0, r1, nframes
    fr.in_pitch = in_pitch if in_pitch is not None else width * 3
    fr.in_frame_stride = in_frame_stride if in_frame_stride is not None else fr.in_pitch * height
    nb = (r1 - r0) * (width // 8)
    fr.out_frame_stride = out_frame_stride if out_frame_stride is not None else 3 * nb * 64
    return fr


def workspace_size(fr: Frames) -> int:
    return lib.jpgx_workspace_size(ctypes.byref(fr))


# ---- torch (device-memory) helpers -------------------------------------------------------
def _stream_ptr(stream) -> int:
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def blocks_gpu(fr: Frames, params: Params, d_rgb, d_out, d_ws, stream=None,
               event_between=None, kernel_events=None) -> None:
    """Launch the hot path on device tensors (uint8 input, int16 output, uint8 workspace).
    d_rgb must point at pixel (0, 8*row_begin) of frame 0 (pass a tensor view or an int).
    event_between: a torch.cuda.Event recorded right after the transform kernel (it must have
    been recorded once already so that its handle exists).
    kernel_events: (start, stop) torch.cuda.Events (timing-enabled, recorded once already) that
    jpgx_blocks_gpu_timed sets to the transform kernel's own begin / end."""
    def ptr(t):
        return t if isinstance(t, int) else t.data_ptr()
    ws_bytes = d_ws.numel() if hasattr(d_ws, "numel") else workspace_size(fr)
    if kernel_events is not None:                 # (start, stop): the kernel's own interval
        e0, e1 = (e.cuda_event for e in kernel_events)
        _check(lib.jpgx_blocks_gpu_timed(ctypes.byref(fr), ctypes.byref(params), ptr(d_rgb), ptr(d_out),
                                         ptr(d_ws), ws_bytes, _stream_ptr(stream), e0, e1),
               "jpgx_blocks_gpu_timed")
        return
    ev = event_between.cuda_event if event_between is not None else None
    _check(lib.jpgx_blocks_gpu_ev(ctypes.byref(fr), ctypes.byref(params), ptr(d_rgb),
                                  ptr(d_out), ptr(d_ws), ws_bytes, _stream_ptr(stream), ev),
           "jpgx_blocks_gpu")


def gen_splitmix_gpu(d_dst, seed: int, nbytes: int | None = None, stream=None) -> None:
    n = d_dst.numel() if nbytes is None else nbytes
    _check(lib.jpgx_gen_splitmix_gpu(d_dst.data_ptr(), n, seed, _stream_ptr(stream)),
           "jpgx_gen_splitmix_gpu")


def gen_tie_gpu(d_dst, width: int, height: int, stream=None) -> None:
    _check(lib.jpgx_gen_tie_gpu(d_dst.data_ptr(), width, height, _stream_ptr(stream)),
           "jpgx_gen_tie_gpu")


def chroma_blocks(width: int, row_begin: int, row_end: int, sample_ratio: int = 0,
                  flags: int = 0) -> int:
    """Chroma blocks per channel of a stripe (== luma blocks unless FLAG_SUBSAMPLE)."""
    return int(lib.jpgx_chroma_blocks(width, row_begin, row_end, sample_ratio, flags))


def entropy_stats_gpu(d_coef, nb_y: int, nb_c: int, carry=None, stream=None):
    """(dc int32 [nb_y + 2 nb_c], hist uint32 [4][257]) device tensors: the reference's dpcm and
    huffman_encode frequency pass over d_coef (torch int16 tensor, Y|Cb|Cr blocks)."""
    import torch
    dev = d_coef.device
    dc = torch.empty(nb_y + 2 * nb_c, dtype=torch.int32, device=dev)
    hist = torch.empty((4, 257), dtype=torch.int32, device=dev)
    ws = torch.empty(max(int(lib.jpgx_entropy_workspace_size(nb_y, nb_c)), 8), dtype=torch.uint8,
                     device=dev)
    cy = None
    if carry is not None:
        cy = (ctypes.c_int32 * 3)(*[int(x) for x in carry])
    _check(lib.jpgx_entropy_stats_gpu(d_coef.data_ptr(), nb_y, nb_c,
                                      ctypes.cast(cy, ctypes.c_void_p) if cy is not None else None,
                                      dc.data_ptr(), hist.data_ptr(), ws.data_ptr(), ws.numel(),
                                      _stream_ptr(stream)), "jpgx_entropy_stats_gpu")
    return dc, hist


def entropy_stats_gpu_batch(d_coef, nb_y: int, nb_c: int, stream=None):
    """The same over a frame batch d_coef [nframes][>= nb_y + 2 nb_c][64] (int16; each frame
    contiguous, frames d_coef.stride(0) elements apart, e.g. a slice of a padded batch):
    (dc int32 [nframes][nb_y + 2 nb_c], hist uint32 [nframes][4][257]), every frame from the image
    start."""
    import torch
    if d_coef.dtype != torch.int16 or d_coef.dim() < 2:
        raise ValueError("entropy_stats_gpu_batch: d_coef must be an int16 [nframes][...] tensor")
    if not d_coef[0].is_contiguous() or d_coef[0].numel() < (nb_y + 2 * nb_c) * 64:
        raise ValueError("entropy_stats_gpu_batch: each frame must be contiguous and hold nb_y + 2 nb_c blocks")
    if d_coef.data_ptr() % 16 or d_coef.stride(0) % 64:
        raise ValueError("entropy_stats_gpu_batch: 16-byte aligned frames, a stride of whole blocks")
    dev = d_coef.device
    nf = d_coef.shape[0]
    dc = torch.empty((nf, nb_y + 2 * nb_c), dtype=torch.int32, device=dev)
    hist = torch.empty((nf, 4, 257), dtype=torch.int32, device=dev)
    ws = torch.empty(max(int(lib.jpgx_entropy_workspace_size_batch(nb_y, nb_c, nf)), 8),
                     dtype=torch.uint8, device=dev)
    _check(lib.jpgx_entropy_stats_gpu_batch(d_coef.data_ptr(), d_coef.stride(0), nf, nb_y, nb_c, None,
                                            dc.data_ptr(), hist.data_ptr(), ws.data_ptr(), ws.numel(),
                                            _stream_ptr(stream)), "jpgx_entropy_stats_gpu_batch")
    return dc, hist


def split_sub(out, nb: int, nbc: int):
    """(Y [nb][64], CbCr [2][nbc][64]) views of one frame's FLAG_SUBSAMPLE output."""
    return out[:nb], out[nb:nb + 2 * nbc].reshape(2, nbc, 64)


def encode_blocks(rgb, quality: int, sample_ratio: int = 0, underflow: bytes | None = None,
                  flags: int = 0, device=None):
    """Convenience: one image (H,W,3 uint8 torch tensor on a GPU, or numpy on the host) ->
    int16 [3][nb][64] (with FLAG_SUBSAMPLE: [nb + 2 nbc][64], see split_sub).  Device tensors
    stay on the device; numpy goes through jpgx_blocks."""
    H, W = int(rgb.shape[0]), int(rgb.shape[1])
    nb = (H // 8) * (W // 8)
    nbc = chroma_blocks(W, 0, H // 8, sample_ratio, flags)
    shape = (nb + 2 * nbc, 64) if flags & FLAG_SUBSAMPLE else (3, nb, 64)
    if isinstance(rgb, np.ndarray):
        rgb = np.ascontiguousarray(rgb, np.uint8)
        p = default_params(W, H, quality, sample_ratio, underflow, flags)
        out = np.empty(shape, np.int16)
        dev = 0 if device is None else int(device)
        _check(lib.jpgx_blocks(rgb.ctypes.data, W, H, W * 3, ctypes.byref(p), out.ctypes.data,
                               dev), "jpgx_blocks")
        return out
    import torch
    H, W = int(rgb.shape[0]), int(rgb.shape[1])
    p = default_params(W, H, quality, sample_ratio, underflow, flags)
    _check(validate(W, H, p), "jpgx_validate")
    fr = frames(W, H)
    fr.out_frame_stride = shape[0] * 64 if flags & FLAG_SUBSAMPLE else 3 * nb * 64
    out = torch.empty(shape, dtype=torch.int16, device=rgb.device)
    ws = torch.empty(workspace_size(fr), dtype=torch.uint8, device=rgb.device)
    blocks_gpu(fr, p, rgb.contiguous(), out, ws)
    return out


def encode_blocks_multi(rgb: np.ndarray, quality: int, ngpus: int, sample_ratio: int = 0,
                        underflow: bytes | None = None, flags: int = 0) -> np.ndarray:
    """Host image -> host coefficients, block-row stripes over GPUs 0..ngpus-1."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    H, W = rgb.shape[:2]
    p = default_params(W, H, quality, sample_ratio, underflow, flags)
    nb = (H // 8) * (W // 8)
    nbc = chroma_blocks(W, 0, H // 8, sample_ratio, flags)
    out = np.empty((nb + 2 * nbc, 64) if flags & FLAG_SUBSAMPLE else (3, nb, 64), np.int16)
    _check(lib.jpgx_blocks_multi(rgb.ctypes.data, W, H, W * 3, ctypes.byref(p), out.ctypes.data,
                                 ngpus), "jpgx_blocks_multi")
    return out


class HostContext:
    """jpgx_host_ctx: `nshards` block-row shards of every image, shard k on GPU devices[k]
    (None: k modulo the device count), chunks of `chunk_rows` block rows (0: auto); device
    buffers, streams and pinned staging persist across calls until close()."""

    def __init__(self, nshards: int = 1, devices=None, chunk_rows: int = 0):
        self._h = ctypes.c_void_p()
        arr = None
        if devices is not None:
            devices = list(devices)
            if len(devices) != nshards:
                raise ValueError("one device per shard")
            arr = (ctypes.c_int * nshards)(*devices)
        self._lib = lib                           # the library that owns the handle
        _check(self._lib.jpgx_host_create(ctypes.byref(self._h), nshards,
                                    ctypes.cast(arr, ctypes.c_void_p) if arr is not None else None,
                                    chunk_rows), "jpgx_host_create")
        self.nshards = nshards

    def blocks(self, rgb: np.ndarray, quality: int, sample_ratio: int = 0, underflow=None,
               flags: int = 0, out: np.ndarray | None = None) -> np.ndarray:
        """Host (H, W, 3) uint8 -> host int16 coefficients (layout as encode_blocks)."""
        if rgb.dtype != np.uint8 or rgb.ndim != 3 or rgb.shape[2] != 3 or rgb.strides[1:] != (3, 1):
            raise ValueError("rgb must be (H, W, 3) uint8 with packed pixels")
        H, W = rgb.shape[:2]
        if rgb.strides[0] < 3 * W:                # flipped or overlapping rows: not a pitch
            raise ValueError("rgb rows must be laid out top-down with a pitch >= 3 * width")
        p = default_params(W, H, quality, sample_ratio, underflow, flags)
        nb = (H // 8) * (W // 8)
        nbc = chroma_blocks(W, 0, H // 8, sample_ratio, flags)
        shape = (nb + 2 * nbc, 64) if flags & FLAG_SUBSAMPLE else (3, nb, 64)
        if out is None:
            out = np.empty(shape, np.int16)
        elif out.shape != shape or out.dtype != np.int16 or not out.flags.c_contiguous:
            raise ValueError(f"out must be a contiguous int16 array of shape {shape}")
        _check(self._lib.jpgx_host_blocks(self._h, rgb.ctypes.data, W, H, rgb.strides[0],
                                    ctypes.byref(p), out.ctypes.data), "jpgx_host_blocks")
        return out

    def close(self) -> None:
        if self._h:
            self._lib.jpgx_host_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_register(a: np.ndarray) -> None:
    """Page-lock a numpy buffer (jpgx_host_register) so jpgx_host_blocks DMAs it directly."""
    _check(lib.jpgx_host_register(a.ctypes.data, a.nbytes), "jpgx_host_register")


def host_unregister(a: np.ndarray) -> None:
    _check(lib.jpgx_host_unregister(a.ctypes.data), "jpgx_host_unregister")
