"""Minimal baseline-JPEG entropy decoder (test helper): parses the markers jpgx_write_jfif
emits (SOF0, or SOF1 with 16-bit DQT, DHT, DRI with RSTm markers, one interleaved SOS) and returns the quantised
zig-zag coefficients [ncomp][nblocks][64] (a list [Y, Cb, Cr] for 4:2:2 / 4:2:0) and the
DQT tables -- an independent check of the
writer, written from ITU-T T.81 (Annex C canonical codes, F.2.2 decoding, F.1.2.3 stuffing)."""
import numpy as np


def _u16(b, i):
    return b[i] << 8 | b[i + 1]


class _Bits:
    def __init__(self, data):
        self.d, self.i, self.acc, self.n = data, 0, 0, 0

    def bit(self):
        if self.n == 0:
            b = self.d[self.i]
            self.i += 1
            if b == 0xFF:
                nxt = self.d[self.i]
                assert nxt == 0x00, f"marker 0xFF{nxt:02X} inside entropy data"
                self.i += 1
            self.acc, self.n = b, 8
        self.n -= 1
        return (self.acc >> self.n) & 1

    def restart(self, m):
        """byte-align, then the RSTm marker (T.81 F.2.2.5)"""
        self.n = 0
        assert self.d[self.i] == 0xFF and self.d[self.i + 1] == 0xD0 + (m & 7), \
            f"expected RST{m & 7} at {self.i}"
        self.i += 2

    def bits(self, k):
        v = 0
        for _ in range(k):
            v = v << 1 | self.bit()
        return v


def _table(bits, vals):
    """canonical codes -> {(length, code): symbol}"""
    out, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            out[(ln, code)] = vals[k]
            code += 1
            k += 1
        code <<= 1
    return out


def _decode_sym(br, tab):
    code = 0
    for ln in range(1, 17):
        code = code << 1 | br.bit()
        if (ln, code) in tab:
            return tab[(ln, code)]
    raise ValueError("bad Huffman code")


def _extend(v, s):
    return v - (1 << s) + 1 if s and v < (1 << (s - 1)) else v


def decode(data: bytes):
    b = bytes(data)
    assert b[:2] == b"\xff\xd8", "no SOI"
    i = 2
    dqt, dht, comps, W, H, sof, ri = {}, {}, [], 0, 0, None, 0
    while True:
        assert b[i] == 0xFF
        m = b[i + 1]
        ln = _u16(b, i + 2)
        seg = b[i + 4:i + 2 + ln]
        if m == 0xDB:
            j = 0
            while j < len(seg):
                pq = seg[j] >> 4                       # 0: 8-bit, 1: 16-bit entries (T.81 B.2.4.1)
                if pq == 0:
                    dqt[seg[j] & 15] = list(seg[j + 1:j + 65])
                else:
                    dqt[seg[j] & 15] = [_u16(seg, j + 1 + 2 * k) for k in range(64)]
                j += 1 + 64 * (pq + 1)
        elif m == 0xC4:
            j = 0
            while j < len(seg):
                tc_th, bits = seg[j], list(seg[j + 1:j + 17])
                n = sum(bits)
                dht[tc_th] = _table(bits, list(seg[j + 17:j + 17 + n]))
                j += 17 + n
        elif m in (0xC0, 0xC1):                        # baseline / extended sequential, Huffman
            sof = m
            assert seg[0] == 8
            H, W = _u16(seg, 1), _u16(seg, 3)
            comps = [(seg[6 + 3 * k], seg[7 + 3 * k], seg[8 + 3 * k]) for k in range(seg[5])]
            assert all(c[1] == 0x11 for c in comps[1:]), "chroma must be sampled 1x1"
        elif m == 0xDD:                                # DRI (T.81 B.2.4.4)
            ri = _u16(seg, 0)
        elif m == 0xDA:
            ns = seg[0]
            sel = [(seg[1 + 2 * k], seg[2 + 2 * k]) for k in range(ns)]
            i += 2 + ln
            break
        i += 2 + ln
    hs, vs = comps[0][1] >> 4, comps[0][1] & 15       # luma sampling (1,1) (2,1) (2,2)
    bpr = W // 8
    nb = bpr * (H // 8)
    cpr, crows = bpr // hs, H // 8 // vs
    nbc = cpr * crows
    out = [np.zeros((nb, 64), np.int32)] + [np.zeros((nbc, 64), np.int32) for _ in sel[1:]]
    br = _Bits(b[i:])
    pred = [0] * len(sel)

    def block(c, tables, dst):
        dc_t, ac_t = dht[tables >> 4], dht[0x10 | (tables & 15)]
        s = _decode_sym(br, dc_t)
        pred[c] += _extend(br.bits(s), s)
        dst[0] = pred[c]
        k = 1
        while k < 64:
            rs = _decode_sym(br, ac_t)
            r, s = rs >> 4, rs & 15
            if s == 0:
                if r == 15:
                    k += 16
                    continue
                break                                      # EOB
            k += r
            dst[k] = _extend(br.bits(s), s)
            k += 1

    nmcu, nrst = 0, 0
    for my in range(crows):                            # MCUs (T.81 A.2.3)
        for mx in range(cpr):
            if ri and nmcu and nmcu % ri == 0:         # restart interval boundary
                br.restart(nrst)
                nrst += 1
                pred = [0] * len(sel)
            nmcu += 1
            for c, (_, tables) in enumerate(sel):
                if c == 0:
                    for dy in range(vs):
                        for dx in range(hs):
                            block(0, tables, out[0][(my * vs + dy) * bpr + mx * hs + dx])
                else:
                    block(c, tables, out[c][my * cpr + mx])
    if hs == vs == 1:
        out = np.stack(out)
    rest = br.d[br.i:]
    assert rest[-2:] == b"\xff\xd9", "no EOI after the scan"
    return {"width": W, "height": H, "coef": out, "dqt": dqt, "sof": sof,
            "qsel": [c[2] for c in comps], "sampling": (hs, vs), "restart_interval": ri,
            "restarts": nrst}
