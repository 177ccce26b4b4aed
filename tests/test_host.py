"""Host-side checks of the product library (no GPU compute): it loads, exports every symbol
include/jpgx.h declares, validates arguments like the reference's valid domain, and its
tables / underflow bytes / guard band agree with the oracle and with the analysis."""
import math
import os
import re

import numpy as np
import pytest

import jpgx
import oracle as O
from conftest import PKG, REPO
from test_oracle import CHR, LUM


def test_exports_every_declared_symbol():
    declared = []
    for h, names in (("jpgx.h", jpgx.EXPORTS), ("jpgx_compat.h", jpgx.COMPAT_EXPORTS)):
        hdr = open(os.path.join(REPO, "include", h)).read()
        hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)          # declarations only
        found = sorted(set(re.findall(r"\b(jpgx_[a-z_0-9]+)\s*\(", hdr)))
        assert found == sorted(names), h
        declared += found
    for name in declared:
        assert hasattr(jpgx.lib, name), name


def test_version_and_devices():
    assert "gfx950" in jpgx.version()
    assert jpgx.device_count() >= 0


def test_validate_codes():
    p = jpgx.default_params(64, 64, 50)
    assert jpgx.validate(64, 64, p) == jpgx.OK
    assert jpgx.validate(60, 64, p) == jpgx.EGEOMETRY
    assert jpgx.validate(64, 60, p) == jpgx.EGEOMETRY
    assert jpgx.validate(0, 64, p) == jpgx.EGEOMETRY
    for q in (0, -1, 98, 99, 100):
        assert jpgx.validate(64, 64, jpgx.default_params(64, 64, q)) == jpgx.EQUALITY
    assert jpgx.validate(64, 64, jpgx.default_params(64, 64, 50, 3)) == jpgx.ESAMPLE
    assert jpgx.validate(24, 16, jpgx.default_params(24, 16, 50, 1)) == jpgx.EGEOMETRY
    assert jpgx.validate(32, 16, jpgx.default_params(32, 16, 50, 1)) == jpgx.OK
    assert jpgx.validate(32, 24, jpgx.default_params(32, 24, 50, 2)) == jpgx.EGEOMETRY
    assert jpgx.validate(32, 32, jpgx.default_params(32, 32, 50, 2)) == jpgx.OK


def test_scale_tables_match_oracle():
    for q in range(1, 98):
        assert np.array_equal(jpgx.scale_table(0, q), O.scale_table(LUM, q)), q
        assert np.array_equal(jpgx.scale_table(1, q), O.scale_table(CHR, q)), q
    with pytest.raises(jpgx.JpgxError):
        jpgx.scale_table(0, 98)


@pytest.mark.parametrize("n,fs", [(64 * 64, 12426), (320 * 240, 230456), (512 * 512, None),
                                  (1920 * 1080, None), (3840 * 2160, None), (4096 * 2736, None),
                                  (4096 * 4096, None), (16384 * 16384, None), (8 * 8, None)])
def test_underflow_matches_oracle(n, fs):
    assert jpgx.glibc_underflow(n, fs) == bytes(O.glibc_underflow(n, fs))


def test_underflow_survey_values():
    # 4K -> 11 90 7e 00 ..; 16384^2 -> 02 10 00 10 ..
    assert jpgx.glibc_underflow(3840 * 2160).hex() == "11907e0000000000"
    assert jpgx.glibc_underflow(16384 * 16384).hex() == "0210001000000000"


def test_underflow_model_matches_real_mmap_bytes():
    """The mmap case of the model against the bytes the REAL reference read in front of its
    three planes (tests/golden/make_big_golden.py: the reference harness stopped after
    preprocess_jpeg for 4096^2 and 8192^2, and the full 16384^2 run)."""
    import json
    with open(os.path.join(REPO, "tests", "golden", "big_golden.json")) as f:
        g = json.load(f)
    cases = {int(s) ** 2: v for s, v in g["mmap_underflow"].items()}
    cases[16384 * 16384] = g["frame16k_q50_sr1"]["underflow"]
    assert len(cases) == 3
    for n, planes in cases.items():
        assert [bytes(p) for p in planes] == [jpgx.glibc_underflow(n)] * 3, n


def test_stripes_partition():
    for rows in (1, 7, 8, 135, 270, 2048):
        for n in (1, 2, 3, 4, 8):
            spans = [jpgx.stripe(rows, n, k) for k in range(n)]
            assert spans[0][0] == 0 and spans[-1][1] == rows
            for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
                assert b0 == a1
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_guard_band_sane():
    for q in (1, 10, 50, 75, 90, 97):
        w, lim = jpgx.guard_band(q)
        assert np.all(lim > 0.49) and np.all(lim < 0.5)
        assert np.all(w != 0)             # negative where the scaled DCT output carries -C2 (v or u = 6)
    # wider band at higher quality (smaller divisors)
    assert (0.5 - jpgx.guard_band(90)[1]).max() > (0.5 - jpgx.guard_band(50)[1]).max()


def test_kernel_cos_table_is_glibc():
    """The exact path's cosine doubles are those the reference's libm call returns:
    cos(((2x+1)*u*M_PI)/16) (src/dct.c:49-50)."""
    src = open(os.path.join(PKG, "csrc", "jx_consts.h")).read()
    assert "kCos[8][8] = JX_COS_INIT" in open(os.path.join(PKG, "csrc", "jpgx_kernels.hip")).read()
    body = src.split("#define JX_COS_INIT")[1].split("#define")[0]
    vals = [float.fromhex(t) for t in re.findall(r"-?0x[0-9a-f.]+p[+-]\d+", body)]
    assert len(vals) == 64
    for u in range(8):
        for x in range(8):
            assert vals[u * 8 + x] == math.cos(((2 * x + 1) * u * math.pi) / 16), (u, x)


def test_workspace_size():
    # every kernel keeps its exact-pass queue in LDS: no device workspace for any geometry
    for fr in (jpgx.frames(3840, 2160, nframes=8), jpgx.frames(64, 64, rows=(2, 5)),
               jpgx.frames(8, 8, nframes=1000), jpgx.frames(64, 64, rows=(3, 3))):
        assert jpgx.workspace_size(fr) == 0


@pytest.mark.parametrize("q", [10, 50, 75, 90, 97])
def test_mx_guard_band_holds_on_emulated_arithmetic(q):
    """k_mx's guard band (jpgx_plan.cpp jx_plan_tables_mx) on a host emulation of its fast
    path (acc_h exact, acc_l summed in fp32, R = fl(acc_h + 2^-12 acc_l), the FOps column pass and
    quantiser): no unflagged coefficient may round differently from the exact quotient, and
    the observed error must stay well inside the band."""
    import ctypes
    f = jpgx.lib.jx_selftest_mx
    f.restype = ctypes.c_longlong
    f.argtypes = [ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
    flagged, ratio = ctypes.c_longlong(), ctypes.c_double()
    assert f(600, 77 + q, q, ctypes.byref(flagged), ctypes.byref(ratio)) == 0
    assert ratio.value < 0.6
    assert flagged.value < 600 * 192 // 100          # well under 1% flagged


def test_mx_operands_make_the_hi_product_exact():
    """k_mx's B operands (jpgx_plan.cpp jx_mx_operands; v_mfma_f32_16x16x32_f16 layout: lane l
    holds B[k = 8 (l >> 4) + e][column l & 15]; k < 24 the pixel-row bytes, stored x 2^15 (A is
    the byte as the f16 subnormal b 2^-24), k = 24 the bias, stored x 2^-9 (A = 1.0), k > 24
    zero; operand 3 part + which, which 0 = Y | Cb columns, 1 = Cr in columns 0..7, 2 = Cr in
    columns 8..15, the other half zero): the hi part is a multiple of 2^-11 whose products with
    bytes 0..255 sum below 2^13 in every column (so the MFMA's hi accumulation is exact in fp32
    whatever its internal order), and hi + lo [+ lo2] reconstruct the colour x cosine matrix and
    the level-shift bias (-1024 for Y at u = 0, none for chroma) to the split's precision (the
    lo parts are stored scaled by 2^12)."""
    import ctypes
    import math
    parts_n = jpgx.lib.jx_mx_parts()
    assert parts_n in (2, 3)
    ops = np.zeros((3 * parts_n, 64, 8), np.uint16)
    f = jpgx.lib.jx_mx_operands
    f.restype = ctypes.c_int
    assert f(ops.ctypes.data_as(ctypes.c_void_p)) == 0
    vals = ops.view(np.float16).astype(np.float64)            # [3 part + which][lane][e]
    B = np.zeros((parts_n, 3, 32, 16))                        # [part][which][k][column]
    for lane in range(64):
        for e in range(8):
            B[:, :, 8 * (lane >> 4) + e, lane & 15] = vals.reshape(parts_n, 3, 64, 8)[:, :, lane, e]
    B[:, :, :24] *= 2.0 ** -15                                  # the encodings' scales
    B[:, :, 24] *= 2.0 ** 9
    assert not np.any(B[:, :, 25:, :])                          # K padding weighs 0
    assert not np.any(B[:, 1, :, 8:]) and not np.any(B[:, 2, :, :8])
    assert np.array_equal(B[:, 1, :, :8], B[:, 2, :, 8:])      # Cr of either set
    # plan columns n = 8c + u: Y|Cb from which 0, Cr from which 1
    M = np.concatenate([B[:, 0], B[:, 1, :, :8]], axis=2)      # [part][k][24]
    hi = M[0]
    lo = M[1:].sum(axis=0) * 2.0 ** -jpgx.lib.jx_mx_loexp()    # lo parts stored x 2^LOEXP
    assert np.all(hi * 2048 == np.round(hi * 2048))
    assert np.all(255 * np.abs(hi[:24]).sum(axis=0) + np.abs(hi[24]) < 8192)
    tol = 2 ** -30 if parts_n == 3 else 2 ** -23
    a = [(0.299, 0.587, 0.114), (-0.168736, 0.331264, -0.5), (0.5, -0.418688, -0.081312)]
    for c in range(3):
        for u in range(8):
            n = 8 * c + u
            for x in range(8):
                for p in range(3):
                    want = a[c][p] * math.cos((2 * x + 1) * u * math.pi / 16)
                    assert abs(hi[3 * x + p, n] + lo[3 * x + p, n] - want) < tol
            bias = -1024.0 if (u == 0 and c == 0) else 0.0
            assert abs(hi[24, n] + lo[24, n] - bias) < tol * 512


@pytest.mark.parametrize("q", [10, 50, 75, 90, 97])
def test_mx422_guard_band_holds_on_emulated_arithmetic(q):
    """k_mx422's chroma guard band (jpgx_plan.cpp jx_plan_tables_mx422: 48-byte rows of pixel
    pairs, two K = 32 products per lo part) on the host emulation of its fast path against the
    exact pair-averaged definition: no unflagged coefficient rounds differently."""
    import ctypes
    f = jpgx.lib.jx_selftest_mx422
    f.restype = ctypes.c_longlong
    f.argtypes = [ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
    flagged, ratio = ctypes.c_longlong(), ctypes.c_double()
    assert f(600, 91 + q, q, ctypes.byref(flagged), ctypes.byref(ratio)) == 0
    assert ratio.value < 0.6
    assert flagged.value < 600 * 128 // 100


@pytest.mark.parametrize("q", [10, 50, 75, 90, 97])
def test_mx420_guard_band_holds_on_emulated_arithmetic(q):
    """k_mx420's chroma guard band (jx_plan_tables_mx420: 96-byte rows = two pixel rows of an
    MCU, three K = 32 products per lo part) on the host emulation against the exact quad-averaged
    definition: no unflagged coefficient rounds differently."""
    import ctypes
    f = jpgx.lib.jx_selftest_mx420
    f.restype = ctypes.c_longlong
    f.argtypes = [ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
    flagged, ratio = ctypes.c_longlong(), ctypes.c_double()
    assert f(600, 53 + q, q, ctypes.byref(flagged), ctypes.byref(ratio)) == 0
    assert ratio.value < 0.6
    assert flagged.value < 600 * 128 // 100


def test_mx420_operands_reconstruct_the_quad_matrix():
    """k_mx420's B operands (jx_mx420_operands, [part][which][lane][e]): which 0 / 1 = k_mx422's Y
    columns; which 2 / 3 / 4 = the chroma matrix over k = 0..95 (k = 48 r + 3x + p, r = the MCU
    pixel row of the chroma row's pair): 0.25 a[c][p] cos((2 floor(x/2) + 1) u pi/16), stored x 2^15;
    the hi part exact-accumulating."""
    import ctypes
    import math
    parts_n = jpgx.lib.jx_mx_parts()
    ops = np.zeros((parts_n, 5, 64, 8), np.uint16)
    f = jpgx.lib.jx_mx420_operands
    f.restype = ctypes.c_int
    assert f(ops.ctypes.data_as(ctypes.c_void_p)) == 0
    vals = ops.view(np.float16).astype(np.float64)
    B = np.zeros((parts_n, 5, 32, 16))
    for lane in range(64):
        for e in range(8):
            B[:, :, 8 * (lane >> 4) + e, lane & 15] = vals[:, :, lane, e]
    ref422 = np.zeros((parts_n, 4, 64, 8), np.uint16)
    g = jpgx.lib.jx_mx422_operands
    g.restype = ctypes.c_int
    assert g(ref422.ctypes.data_as(ctypes.c_void_p)) == 0
    assert np.array_equal(ops[:, :2], ref422[:, :2])            # the same Y operands
    C = np.concatenate([B[:, 2], B[:, 3], B[:, 4]], axis=1) * 2.0 ** -15   # [part][k 0..95][16]
    hi, lo = C[0], C[1:].sum(axis=0) * 2.0 ** -jpgx.lib.jx_mx_loexp()
    assert np.all(hi * 2048 == np.round(hi * 2048))
    assert np.all(255 * np.abs(hi).sum(axis=0) < 8192)
    tol = 2 ** -30 if parts_n == 3 else 2 ** -23
    a = [(-0.168736, 0.331264, -0.5), (0.5, -0.418688, -0.081312)]
    for c in range(2):
        for u in range(8):
            n = 8 * c + u
            for r in range(2):
                for x in range(16):
                    for p in range(3):
                        k = 48 * r + 3 * x + p
                        want = 0.25 * a[c][p] * math.cos((2 * (x // 2) + 1) * u * math.pi / 16)
                        assert abs(hi[k, n] + lo[k, n] - want) < tol


def test_mx422_operands_reconstruct_the_pair_matrix():
    """k_mx422's B operands (jx_mx422_operands, [part][which][lane][e]): which 0 / 1 = k_mx's Y
    columns for set 0 (C columns 0..7) / set 1 (8..15), K = 25 used; which 2 / 3 = the chroma
    matrix over k = 0..31 / 32..63: 0.5 a[c][p] cos((2 floor(x/2) + 1) u pi/16) at k = 3x + p <
    48 (stored x 2^15, as k_mx's), zero from k = 48 on (chroma has no level-shift constant);
    column j = Cb (j < 8) / Cr u.  The hi part is exact-accumulating (multiple of 2^-11, products
    with bytes 0..255 below 2^13)."""
    import ctypes
    import math
    parts_n = jpgx.lib.jx_mx_parts()
    ops = np.zeros((parts_n, 4, 64, 8), np.uint16)
    f = jpgx.lib.jx_mx422_operands
    f.restype = ctypes.c_int
    assert f(ops.ctypes.data_as(ctypes.c_void_p)) == 0
    vals = ops.view(np.float16).astype(np.float64)
    B = np.zeros((parts_n, 4, 32, 16))
    for lane in range(64):
        for e in range(8):
            B[:, :, 8 * (lane >> 4) + e, lane & 15] = vals[:, :, lane, e]
    B[:, :2, :24] *= 2.0 ** -15                                 # Y: byte rows and bias row
    B[:, :2, 24] *= 2.0 ** 9
    B[:, 2:] *= 2.0 ** -15                                      # chroma: byte rows (k < 48)
    assert not np.any(B[:, 0, :, 8:]) and not np.any(B[:, 1, :, :8])
    assert np.array_equal(B[:, 0, :, :8], B[:, 1, :, 8:])
    assert not np.any(B[:, :2, 25:, :])
    C = np.concatenate([B[:, 2], B[:, 3]], axis=1)              # [part][k 0..63][16]
    assert not np.any(C[:, 48:, :])
    hi, lo = C[0], C[1:].sum(axis=0) * 2.0 ** -jpgx.lib.jx_mx_loexp()
    assert np.all(hi * 2048 == np.round(hi * 2048))
    assert np.all(255 * np.abs(hi[:48]).sum(axis=0) < 8192)
    tol = 2 ** -30 if parts_n == 3 else 2 ** -23
    a = [(-0.168736, 0.331264, -0.5), (0.5, -0.418688, -0.081312)]
    for c in range(2):
        for u in range(8):
            n = 8 * c + u
            for x in range(16):
                for p in range(3):
                    want = 0.5 * a[c][p] * math.cos((2 * (x // 2) + 1) * u * math.pi / 16)
                    assert abs(hi[3 * x + p, n] + lo[3 * x + p, n] - want) < tol


def test_table_builders_are_reentrant():
    """The plan's table and operand builders run once per device, on whichever host thread first
    launches there (jpgx_host_blocks runs one thread per shard): called from 8 threads at once
    (ctypes drops the GIL for the call) they return exactly the single-threaded results."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    parts_n = jpgx.lib.jx_mx_parts()
    shapes = {"jx_mx_operands": (3 * parts_n, 64, 8), "jx_mx422_operands": (parts_n, 4, 64, 8),
              "jx_mx420_operands": (parts_n, 5, 64, 8)}

    def run(name, q):
        f = getattr(jpgx.lib, name)
        f.restype = ctypes.c_int
        if name in shapes:
            ops = np.zeros(shapes[name], np.uint16)
            assert f(ops.ctypes.data_as(ctypes.c_void_p)) == 0
            return [ops]
        w, lim = np.zeros((24, 8), np.float32), np.zeros((24, 8), np.float32)
        qq = np.zeros((2, 64), np.int16)
        assert f(q, w.ctypes.data_as(ctypes.c_void_p), lim.ctypes.data_as(ctypes.c_void_p),
                 qq.ctypes.data_as(ctypes.c_void_p)) == 0
        return [w, lim, qq]

    jobs = [(n, q) for n in ("jx_mx_operands", "jx_mx422_operands", "jx_mx420_operands",
                             "jx_plan_tables_mx", "jx_plan_tables_mx422", "jx_plan_tables_mx420")
            for q in (50, 90)] * 3
    want = {j: run(*j) for j in set(jobs)}
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda j: run(*j), jobs))
    for j, g in zip(jobs, got):
        for a, b in zip(want[j], g):
            assert np.array_equal(a, b), j


def test_packed_transform_matches_scalar_bit_for_bit():
    """The packed-pair transform (xform_math.h: jx_fdct8_pk, PairOps) performs, lane by lane,
    the scalar operation sequence the guard band was derived for: identical fp32 row/column
    outputs and quantiser values on random, flat, two-level and ramp blocks (host evaluation,
    jpgx_plan.cpp jx_selftest_pk)."""
    import ctypes
    f = jpgx.lib.jx_selftest_pk
    f.restype = ctypes.c_longlong
    f.argtypes = [ctypes.c_longlong, ctypes.c_ulonglong]
    assert f(20000, 1) == 0
    assert f(20000, 0x9E3779B97F4A7C15) == 0


def test_product_entry_points_fail_loudly_without_a_gpu():
    """No CPU fallback: without a GPU every compute entry point returns JPGX_ENODEV (or the HIP
    error), never a result.  Skipped where a GPU is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import jpgx
    rgb = np.zeros((16, 16, 3), np.uint8)
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.encode_blocks(rgb, 50)
    assert e.value.rc == jpgx.ENODEV
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.encode_blocks_multi(rgb, 50, 1)
    assert e.value.rc == jpgx.ENODEV
    with pytest.raises(jpgx.JpgxError) as e:
        jpgx.HostContext(2)
    assert e.value.rc == jpgx.ENODEV
    assert jpgx.device_count() == 0


def test_launch_constant_division_is_exact(tmp_path):
    """jx_udiv_make (jpgx_internal.h): the multiply-high division a wave uses to find its frame,
    block-row and column (mx_seek) equals n / d for every divisor shape the launches use (frame
    and row block counts, powers of two, 1, the extremes) and random 32-bit numerators."""
    src = tmp_path / "udiv.cpp"
    src.write_text(r'''
#include <stdio.h>
#include "jpgx_internal.h"
static unsigned dv(unsigned n, jx_udiv d) {
    const unsigned t = (unsigned)(((unsigned long long)d.m * n) >> 32);
    return (t + ((n - t) >> d.s1)) >> d.s2;
}
int main() {
    unsigned long long x = 88172645463325252ull;
    const unsigned ds[] = {1, 2, 3, 7, 8, 9, 60, 240, 480, 2048, 4096, 129600, 259200, 8294400,
                           33554432, 0x7fffffffu, 0x80000000u, 0x80000001u, 0xffffffffu};
    int bad = 0;
    for (int k = 0; k < 20000; k++) {
        unsigned d;
        if (k < 19) d = ds[k];
        else { x ^= x << 13; x ^= x >> 7; x ^= x << 17; d = (unsigned)(x >> (x & 31)); if (!d) d = 1; }
        const jx_udiv D = jx_udiv_make(d);
        for (int i = 0; i < 200; i++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            unsigned n = (unsigned)x;
            if (i == 0) n = 0; else if (i == 1) n = 0xffffffffu; else if (i == 2) n = d - 1; else if (i == 3) n = d;
            if (dv(n, D) != n / d) bad++;
        }
    }
    printf("%d\n", bad);
    return bad != 0;
}
''')
    exe = tmp_path / "udiv"
    import subprocess
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(PKG, "csrc"), "-I" + os.path.join(REPO, "include"),
                    str(src), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout
