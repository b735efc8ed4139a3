"""Test-side OpenEXR reader (TEST INFRASTRUCTURE, never imported by the product).

Reads scanline files with NO_COMPRESSION (igx's own writer, `host/exr.cpp`),
ZIPS/ZIP (zlib + byte predictor + interleave) and PIZ (Haar wavelet + Huffman)
compression, HALF / FLOAT / UINT channels.  The reference's evaluation images
(`scenes/evaluation/references/*.exr`) are PIZ (Mitsuba / Radiance exports) or
ZIP (Cycles exports); RunEvaluations.py reads them through simpleimageio, which
is not installed here, so this is a restatement of the published OpenEXR file
format and codecs:

* file layout: magic 20000630, version 2, attribute list, scanline offset
  table (one u64 per chunk), chunks `{i32 y, i32 size, data}`; a chunk whose
  size equals the uncompressed size is stored raw;
* ZIP: zlib inflate, undo the delta predictor (t[i] = t[i-1] + t[i] - 128),
  de-interleave the two byte halves; 1 (ZIPS) or 16 (ZIP) scanlines per chunk;
* PIZ: 32 scanlines per chunk; bitmap of the used 16-bit values and its
  reverse LUT; canonical Huffman code (6-bit code lengths with zero-run codes
  59..63, the last symbol `iM` being the run-length escape with an 8-bit
  repeat count); per channel (FLOAT = two 16-bit planes) the inverse 2D Haar
  wavelet `wav2Decode` with the 14-bit or the modulo-2^16 lifting step; the
  LUT expansion; per scanline re-interleaving of the channels.

Pure numpy; a 256x256 RGB PIZ image decodes in about a second.
"""
import struct
import zlib

import numpy as np

_PIXEL_BYTES = {0: 4, 1: 2, 2: 4}  # UINT, HALF, FLOAT
_PIXEL_DTYPE = {0: np.uint32, 1: np.float16, 2: np.float32}
_LINES_PER_CHUNK = {0: 1, 1: 1, 2: 1, 3: 16, 4: 32}


def _parse_header(data):
    magic, version = struct.unpack_from("<II", data, 0)
    assert magic == 20000630 and (version & 0xFF) == 2, (magic, version)
    assert not (version & 0x200), "tiled EXR not supported"
    pos = 8
    attrs = {}
    while data[pos] != 0:
        end = data.index(b"\0", pos)
        name = data[pos:end].decode()
        pos = end + 1
        end = data.index(b"\0", pos)
        typ = data[pos:end].decode()
        pos = end + 1
        (size,) = struct.unpack_from("<i", data, pos)
        pos += 4
        attrs[name] = (typ, data[pos:pos + size])
        pos += size
    return attrs, pos + 1


def _channels(raw):
    chans = []
    p = 0
    while raw[p] != 0:
        end = raw.index(b"\0", p)
        nm = raw[p:end].decode()
        ptype, _plin, xs, ys = struct.unpack_from("<iiii", raw, end + 1)
        assert xs == 1 and ys == 1, "subsampled channels not supported"
        chans.append((nm, ptype))
        p = end + 1 + 16
    return chans


# ---------------------------------------------------------------- ZIP codec
def _unzip(buf, out_size):
    t = np.frombuffer(zlib.decompress(buf), np.uint8)
    assert t.size == out_size, (t.size, out_size)
    # predictor: t[i] = t[i-1] + t[i] - 128  (mod 256)  == running sum
    d = t.astype(np.int64)
    d[1:] -= 128
    t = (np.cumsum(d) & 0xFF).astype(np.uint8)
    half = (out_size + 1) // 2
    out = np.empty(out_size, np.uint8)
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out.tobytes()


# ---------------------------------------------------------------- PIZ codec
_HUF_ENCSIZE = 65537
_SHORT_ZEROCODE_RUN = 59
_LONG_ZEROCODE_RUN = 63
_SHORTEST_LONG_RUN = 2 + _LONG_ZEROCODE_RUN - _SHORT_ZEROCODE_RUN


class _BitReader:
    """MSB-first bit reader over a byte string (OpenEXR's getBits)."""

    def __init__(self, buf, pos):
        self.buf, self.pos, self.c, self.lc = buf, pos, 0, 0

    def get(self, n):
        while self.lc < n:
            self.c = ((self.c << 8) | self.buf[self.pos]) & ((1 << 64) - 1)
            self.pos += 1
            self.lc += 8
        self.lc -= n
        return (self.c >> self.lc) & ((1 << n) - 1)


def _huf_code_lengths(buf, pos, im, iM):
    """Packed code-length table -> (lengths[65537], byte position after it)."""
    lens = np.zeros(_HUF_ENCSIZE, np.int64)
    br = _BitReader(buf, pos)
    i = im
    while i <= iM:
        l = br.get(6)
        if l == _LONG_ZEROCODE_RUN:
            run = br.get(8) + _SHORTEST_LONG_RUN
            assert i + run <= iM + 1, "corrupt Huffman table"
            i += run
        elif l >= _SHORT_ZEROCODE_RUN:
            run = l - _SHORT_ZEROCODE_RUN + 2
            assert i + run <= iM + 1, "corrupt Huffman table"
            i += run
        else:
            lens[i] = l
            i += 1
    return lens, br.pos


def _huf_canonical(lens):
    """Canonical codes: symbols of a length are numbered in index order, and
    longer codes take the numerically smaller prefixes (hufCanonicalCodeTable)."""
    n = np.bincount(lens, minlength=59)[:59].astype(np.int64)
    start = np.zeros(59, np.int64)
    c = 0
    for l in range(58, 0, -1):
        nc = (c + n[l]) >> 1
        start[l] = c
        c = nc
    codes = np.zeros_like(lens)
    syms = np.flatnonzero(lens > 0)
    # within one length, consecutive codes in symbol order
    for l in np.unique(lens[syms]):
        s = syms[lens[syms] == l]
        codes[s] = start[l] + np.arange(s.size)
    return codes


def _huf_decode(buf, pos, nbytes, n_out):
    im, iM, _tlen, nbits, _ = struct.unpack_from("<5i", buf, pos)
    lens, p = _huf_code_lengths(buf, pos + 20, im, iM)
    codes = _huf_canonical(lens)
    syms = np.flatnonzero(lens > 0)
    lmax = int(lens.max())
    assert 0 < lmax <= 24, lmax
    # full lookup table over lmax-bit windows: window -> (symbol, length)
    tab_sym = np.full(1 << lmax, -1, np.int64)
    tab_len = np.zeros(1 << lmax, np.int64)
    for s in syms:
        l = int(lens[s])
        lo = int(codes[s]) << (lmax - l)
        tab_sym[lo:lo + (1 << (lmax - l))] = s
        tab_len[lo:lo + (1 << (lmax - l))] = l
    end = pos + nbytes
    bits = np.unpackbits(np.frombuffer(buf[p:end], np.uint8))[:nbits]
    pad = np.concatenate([bits, np.zeros(lmax, np.uint8)]).astype(np.int64)
    win = np.zeros(nbits, np.int64)
    for k in range(lmax):
        win = (win << 1) | pad[k:k + nbits]
    sym_at = tab_sym[win].tolist()
    len_at = tab_len[win].tolist()
    out = np.empty(n_out, np.uint16)
    o = 0
    b = 0
    while b < nbits:
        s = sym_at[b]
        l = len_at[b]
        assert s >= 0 and b + l <= nbits, "corrupt Huffman stream"
        b += l
        if s == iM:  # run-length escape: repeat the previous symbol
            cs = 0
            for _ in range(8):
                cs = (cs << 1) | int(bits[b])
                b += 1
            assert o > 0 and o + cs <= n_out
            out[o:o + cs] = out[o - 1]
            o += cs
        else:
            out[o] = s
            o += 1
    assert o == n_out, (o, n_out)
    return out


def _wdec14(l, h):
    ls = l.astype(np.uint16).view(np.int16).astype(np.int32)
    hi = h.astype(np.uint16).view(np.int16).astype(np.int32)
    ai = ls + (hi & 1) + (hi >> 1)
    return ai & 0xFFFF, (ai - hi) & 0xFFFF


def _wdec16(l, h):
    m = l.astype(np.int32)
    d = h.astype(np.int32)
    bb = (m - (d >> 1)) & 0xFFFF
    aa = (d + bb - 32768) & 0xFFFF
    return aa, bb


def _wav2_decode(a, mx):
    """In-place inverse Haar wavelet of a 2D uint16 plane (ny, nx) (ImfWav wav2Decode)."""
    ny, nx = a.shape
    dec = _wdec14 if mx < (1 << 14) else _wdec16
    n = min(nx, ny)
    p = 1
    while p <= n:
        p <<= 1
    p >>= 1
    p2 = p
    p >>= 1
    v = a.astype(np.int32)
    while p >= 1:
        ys = np.arange(0, ny - p2 + 1, p2)
        xs = np.arange(0, nx - p2 + 1, p2)
        Y, X = np.ix_(ys, xs)
        i00, i10 = dec(v[Y, X], v[Y + p, X])
        i01, i11 = dec(v[Y, X + p], v[Y + p, X + p])
        v[Y, X], v[Y, X + p] = dec(i00, i01)
        v[Y + p, X], v[Y + p, X + p] = dec(i10, i11)
        if nx & p:  # odd column
            xl = xs[-1] + p2 if xs.size else 0
            i00, v[ys + p, xl] = dec(v[ys, xl], v[ys + p, xl])
            v[ys, xl] = i00
        if ny & p:  # odd line
            yl = ys[-1] + p2 if ys.size else 0
            i00, v[yl, xs + p] = dec(v[yl, xs], v[yl, xs + p])
            v[yl, xs] = i00
        p2 = p
        p >>= 1
    a[...] = v.astype(np.uint16)


def _unpiz(buf, w, nlines, chans):
    pos = 0
    mn, mx_nz = struct.unpack_from("<HH", buf, pos)
    pos += 4
    assert mx_nz < 8192
    bitmap = np.zeros(8192, np.uint8)
    if mn <= mx_nz:
        bitmap[mn:mx_nz + 1] = np.frombuffer(buf, np.uint8, mx_nz - mn + 1, pos)
        pos += mx_nz - mn + 1
    used = np.unpackbits(bitmap, bitorder="little").astype(bool)
    used[0] = True
    lut = np.flatnonzero(used).astype(np.uint16)
    max_value = lut.size - 1
    (length,) = struct.unpack_from("<i", buf, pos)
    pos += 4
    sizes = [_PIXEL_BYTES[t] // 2 for _, t in chans]
    n_total = sum(w * nlines * s for s in sizes)
    tmp = _huf_decode(buf, pos, length, n_total)
    planes = []
    off = 0
    for s in sizes:
        pl = tmp[off:off + w * nlines * s].reshape(nlines, w, s)
        for j in range(s):
            sub = np.ascontiguousarray(pl[:, :, j])
            _wav2_decode(sub, max_value)
            pl[:, :, j] = sub
        planes.append(lut[pl.reshape(nlines, w * s)])
        off += w * nlines * s
    # scanline-interleaved: for each line, each channel's w*s values
    return np.concatenate(planes, axis=1).tobytes()


# ---------------------------------------------------------------- reader
def read_exr(path):
    """-> ({channel name: float32 (h, w) array}, attributes)."""
    data = open(path, "rb").read()
    attrs, pos = _parse_header(data)
    chans = _channels(attrs["channels"][1])
    comp = attrs["compression"][1][0]
    assert comp in _LINES_PER_CHUNK, f"compression {comp} not supported"
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    lpc = _LINES_PER_CHUNK[comp]
    nchunks = (h + lpc - 1) // lpc
    offsets = struct.unpack_from(f"<{nchunks}Q", data, pos)
    line_bytes = sum(w * _PIXEL_BYTES[t] for _, t in chans)
    img = {nm: np.zeros((h, w), np.float32) for nm, _ in chans}
    for off in offsets:
        y, size = struct.unpack_from("<ii", data, off)
        nlines = min(lpc, y1 - y + 1)
        raw_size = nlines * line_bytes
        buf = data[off + 8:off + 8 + size]
        if size >= raw_size or comp == 0:
            raw = buf
        elif comp in (2, 3):
            raw = _unzip(buf, raw_size)
        else:
            raw = _unpiz(buf, w, nlines, chans)
        assert len(raw) == raw_size
        p = 0
        for ln in range(nlines):
            for nm, t in chans:
                n = w * _PIXEL_BYTES[t]
                img[nm][y - y0 + ln] = np.frombuffer(raw, _PIXEL_DTYPE[t], w, p).astype(np.float32)
                p += n
    return img, attrs


def read_rgb(path):
    """-> float32 (h, w, 3) linear RGB."""
    img, _ = read_exr(path)
    return np.stack([img["R"], img["G"], img["B"]], axis=-1)
