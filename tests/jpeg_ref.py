"""TEST INFRASTRUCTURE: a numpy restatement of the pixel half of the JPEG
decode peer, from the packed coefficient image the host half produces
(uphip_jpeg_entropy_decode, layout csrc/jpeg.h), with libjpeg's default
arithmetic:

- jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2, 64-bit products,
  the IDCT range-limit table of jdmaster.c prepare_range_limit_table);
- jdsample.c h2v1 / h2v2 / h1v2 fancy upsampling (box replication when the
  downsampled width is <= 2, as jinit_upsampler picks);
- jdcolor.c ycc_rgb_convert (SCALEBITS 16 tables).

The CPU tests pin the host entropy decoder plus this arithmetic against PIL's
libjpeg-turbo; the GPU tests pin the device kernels (kernels_jpeg.hip) against
PIL directly.  Never imported by the product."""
import ctypes as C

import numpy as np

NATURAL = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], np.int64)


class JpegComp(C.Structure):
    _fields_ = [("h", C.c_int32), ("v", C.c_int32), ("bw", C.c_int32), ("bh", C.c_int32),
                ("dw", C.c_int32), ("dh", C.c_int32), ("plane_off", C.c_int64),
                ("pitch", C.c_int32), ("qzz", C.c_uint16 * 64)]


class JpegScan(C.Structure):
    _fields_ = [("ncomp", C.c_int32), ("comp", C.c_int32 * 4), ("mcus_x", C.c_int32),
                ("mcus_y", C.c_int32), ("blocks_per_mcu", C.c_int32),
                ("first_block", C.c_int64), ("first_group", C.c_int32)]


class JpegHeader(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("ncomp", C.c_int32),
                ("color", C.c_int32), ("hmax", C.c_int32), ("vmax", C.c_int32),
                ("comp", JpegComp * 3), ("nscans", C.c_int32), ("scan", JpegScan * 8),
                ("nblocks", C.c_int64), ("ngroups", C.c_int64), ("counts_off", C.c_int64),
                ("groups_off", C.c_int64), ("coefs_off", C.c_int64), ("total_bytes", C.c_int64),
                ("scratch_bytes", C.c_int64)]


def entropy_decode(lib, data: bytes):
    n = lib.uphip_jpeg_entropy_decode(data, len(data), None, 0)
    if n < 0:
        raise RuntimeError(lib.uphip_last_error().decode())
    buf = np.zeros(n, np.uint8)
    assert lib.uphip_jpeg_entropy_decode(data, len(data), buf.ctypes.data, n) == n
    return buf


def unpack(buf):
    h = JpegHeader.from_buffer_copy(buf[:C.sizeof(JpegHeader)].tobytes())
    counts = buf[h.counts_off:h.counts_off + h.nblocks].astype(np.int64)
    groups = buf[h.groups_off:h.groups_off + 4 * (h.ngroups + 1)].view(np.uint32).astype(np.int64)
    ncoef = (h.total_bytes - h.coefs_off) // 2
    coefs = buf[h.coefs_off:h.coefs_off + 2 * ncoef].view(np.int16).astype(np.int64)
    return h, counts, groups, coefs


def block_positions(h):
    """(comp, bx, by) of every block in decode order."""
    comp = np.zeros(h.nblocks, np.int64)
    bx = np.zeros(h.nblocks, np.int64)
    by = np.zeros(h.nblocks, np.int64)
    for s in range(h.nscans):
        S = h.scan[s]
        nb = S.mcus_x * S.mcus_y * S.blocks_per_mcu
        l = np.arange(nb)
        mcu, k = l // S.blocks_per_mcu, l % S.blocks_per_mcu
        mx, my = mcu % S.mcus_x, mcu // S.mcus_x
        sl = slice(S.first_block, S.first_block + nb)
        if S.ncomp == 1:
            comp[sl], bx[sl], by[sl] = S.comp[0], mx, my
            continue
        c_, x_, y_ = np.zeros(nb, np.int64), np.zeros(nb, np.int64), np.zeros(nb, np.int64)
        start = 0
        for i in range(S.ncomp):
            cc = h.comp[S.comp[i]]
            m = (k >= start) & (k < start + cc.h * cc.v)
            kk = k[m] - start
            c_[m] = S.comp[i]
            x_[m] = mx[m] * cc.h + kk % cc.h
            y_[m] = my[m] * cc.v + kk // cc.h
            start += cc.h * cc.v
        comp[sl], bx[sl], by[sl] = c_, x_, y_
    return comp, bx, by


def _idct_pass(d, shift):
    """jpeg_idct_islow's 8-point pass along the last axis (int64)."""
    z2, z3 = d[..., 2], d[..., 6]
    z1 = (z2 + z3) * 4433
    tmp2 = z1 + z3 * -15137
    tmp3 = z1 + z2 * 6270
    tmp0 = (d[..., 0] + d[..., 4]) * 8192
    tmp1 = (d[..., 0] - d[..., 4]) * 8192
    t10, t13, t11, t12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
    tmp0, tmp1, tmp2, tmp3 = d[..., 7], d[..., 5], d[..., 3], d[..., 1]
    z1, z2, z3, z4 = tmp0 + tmp3, tmp1 + tmp2, tmp0 + tmp2, tmp1 + tmp3
    z5 = (z3 + z4) * 9633
    tmp0, tmp1, tmp2, tmp3 = tmp0 * 2446, tmp1 * 16819, tmp2 * 25172, tmp3 * 12299
    z1, z2, z3, z4 = z1 * -7373, z2 * -20995, z3 * -16069 + z5, z4 * -3196 + z5
    tmp0 = tmp0 + z1 + z3
    tmp1 = tmp1 + z2 + z4
    tmp2 = tmp2 + z2 + z3
    tmp3 = tmp3 + z1 + z4
    half = 1 << (shift - 1)
    out = np.stack([t10 + tmp3, t11 + tmp2, t12 + tmp1, t13 + tmp0,
                    t13 - tmp0, t12 - tmp1, t11 - tmp2, t10 - tmp3], axis=-1)
    return (out + half) >> shift


def idct_islow(nat):
    """nat: (n, 64) dequantised coefficients, natural order -> (n, 8, 8) samples."""
    blk = nat.reshape(-1, 8, 8)
    ws = _idct_pass(np.swapaxes(blk, 1, 2), 11)          # columns
    ws = np.swapaxes(ws, 1, 2).astype(np.int32).astype(np.int64)  # (int) workspace
    out = _idct_pass(ws, 18)                             # rows
    s = out & 1023
    s = np.where(s >= 512, s - 1024, s) + 128
    return np.clip(s, 0, 255).astype(np.uint8)


def planes(buf):
    h, counts, groups, coefs = unpack(buf)
    off = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    zz = np.zeros((h.nblocks, 64), np.int64)
    for k in range(64):
        m = counts > k
        zz[m, k] = coefs[off[m] + k]
    comp, bx, by = block_positions(h)
    q = np.array([[h.comp[c].qzz[k] for k in range(64)] for c in range(h.ncomp)], np.int64)
    nat = np.zeros_like(zz)
    nat[:, NATURAL] = zz * q[comp]
    pix = idct_islow(nat)
    out = []
    for c in range(h.ncomp):
        cc = h.comp[c]
        P = np.zeros((cc.bh * 8, cc.bw * 8), np.uint8)
        m = comp == c
        for b, x, y in zip(np.nonzero(m)[0], bx[m], by[m]):
            P[y * 8:y * 8 + 8, x * 8:x * 8 + 8] = pix[b]
        out.append(P)
    return h, out, (counts, groups, off)


def upsample(h, c, P):
    cc = h.comp[c]
    rh, rv = h.hmax // cc.h, h.vmax // cc.v
    W, H = h.width, h.height
    dw, dh = cc.dw, cc.dh
    x = np.arange(W)
    y = np.arange(H)
    if rh == 1 and rv == 1:
        return P[:H, :W].astype(np.int64)
    if rv == 1:
        rows = P[:H].astype(np.int64)
        cx = x >> 1
        if dw <= 2:
            return rows[:, cx]
        v3 = 3 * rows[:, cx]
        prv = rows[:, np.maximum(cx - 1, 0)]
        nxt = rows[:, np.minimum(cx + 1, dw - 1)]
        even = np.where(cx == 0, rows[:, cx], (v3 + prv + 1) >> 2)
        odd = np.where(cx == dw - 1, rows[:, cx], (v3 + nxt + 2) >> 2)
        return np.where((x & 1) == 0, even, odd)
    cy = y >> 1
    ny = np.where(y & 1, np.minimum(cy + 1, dh - 1), np.maximum(cy - 1, 0))
    if rh == 1:
        bias = np.where(y & 1, 2, 1)[:, None]
        return (3 * P[cy][:, :W].astype(np.int64) + P[ny][:, :W] + bias) >> 2
    cx = x >> 1
    if dw <= 2:
        return P[cy][:, cx].astype(np.int64)
    cs = 3 * P[cy].astype(np.int64) + P[ny]           # column sums per output row
    this = cs[:, cx]
    prv = cs[:, np.maximum(cx - 1, 0)]
    nxt = cs[:, np.minimum(cx + 1, dw - 1)]
    even = np.where(cx == 0, (this * 4 + 8) >> 4, (this * 3 + prv + 8) >> 4)
    odd = np.where(cx == dw - 1, (this * 4 + 7) >> 4, (this * 3 + nxt + 7) >> 4)
    return np.where((x & 1) == 0, even, odd)


def decode(lib, data: bytes):
    """Pixels (H, W) uint8 or (H, W, 3) uint8 as the device path makes them."""
    return decode_packed(entropy_decode(lib, data))


def decode_packed(buf):
    """Pixels from a packed coefficient image (jpeg.h layout)."""
    h, P, _ = planes(buf)
    if h.ncomp == 1:
        return P[0][:h.height, :h.width].copy()
    c0, c1, c2 = (upsample(h, c, P[c]) for c in range(3))
    if h.color == 2:
        return np.stack([c0, c1, c2], axis=2).astype(np.uint8)
    cb, cr = c1 - 128, c2 - 128
    r = c0 + ((91881 * cr + 32768) >> 16)
    g = c0 + ((-22554 * cb + 32768 + -46802 * cr) >> 16)
    b = c0 + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], axis=2), 0, 255).astype(np.uint8)
