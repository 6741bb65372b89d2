"""Minimal PNG writer for the offline-replay tests (TEST INFRASTRUCTURE): grey / RGB / RGBA, 8 or
16 bit, every scanline filter type (rows cycle through `filters`), zlib via the standard library."""
import struct
import zlib

import numpy as np


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def write_png(path, img, filters=(0, 1, 2, 3, 4)):
    img = np.asarray(img)
    depth = 16 if img.dtype == np.uint16 else 8
    chans = 1 if img.ndim == 2 else img.shape[2]
    ctype = {1: 0, 3: 2, 4: 6}[chans]
    H, W = img.shape[:2]
    if depth == 16:
        rows = img.reshape(H, W * chans).astype(">u2").view(np.uint8).reshape(H, -1)
    else:
        rows = img.reshape(H, W * chans).astype(np.uint8)
    bpp = chans * depth // 8
    out = bytearray()
    prev = np.zeros(rows.shape[1], np.int64)
    for y in range(H):
        x = rows[y].astype(np.int64)
        a = np.concatenate([np.zeros(bpp, np.int64), x[:-bpp]])
        c = np.concatenate([np.zeros(bpp, np.int64), prev[:-bpp]])
        ft = filters[y % len(filters)]
        f = {0: x, 1: x - a, 2: x - prev, 3: x - ((a + prev) >> 1), 4: x - _paeth(a, prev, c)}[ft]
        out.append(ft)
        out += (f & 0xFF).astype(np.uint8).tobytes()
        prev = x

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    with open(path, "wb") as fh:
        fh.write(b"\x89PNG\r\n\x1a\n")
        fh.write(chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, depth, ctype, 0, 0, 0)))
        fh.write(chunk(b"IDAT", zlib.compress(bytes(out), 6)))
        fh.write(chunk(b"IEND", b""))


def se3_from_matrix(m):
    """SE3<float>(Eigen::Matrix<float, 3, 4>) (lie_group.cuh:18-19): Eigen's rotation-matrix ->
    quaternion (trace method) in float32, the same operation order as host/tsdf_types.h."""
    f = np.float32
    M = lambda i, j: f(m[i][j])
    q = [f(0)] * 4  # x y z w
    t = M(0, 0) + (M(1, 1) + M(2, 2))
    if t > 0:
        t = np.sqrt(t + f(1.0))
        w = f(0.5) * t
        t = f(0.5) / t
        q = [(M(2, 1) - M(1, 2)) * t, (M(0, 2) - M(2, 0)) * t, (M(1, 0) - M(0, 1)) * t, w]
    else:
        i = 0
        if M(1, 1) > M(0, 0):
            i = 1
        if M(2, 2) > M(i, i):
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(M(i, i) - M(j, j) - M(k, k) + f(1.0))
        cc = [f(0)] * 3
        cc[i] = f(0.5) * t
        t = f(0.5) / t
        w = (M(k, j) - M(j, k)) * t
        cc[j] = (M(j, i) + M(i, j)) * t
        cc[k] = (M(k, i) + M(i, k)) * t
        q = [cc[0], cc[1], cc[2], w]
    qi = [f(0), f(0), f(0), f(1)]  # identity extrinsics * SE3(m): SSE quaternion product order
    a, b = qi, q
    r = [(a[0] * b[3] - a[2] * b[1]) + (a[1] * b[2] + a[3] * b[0]),
         (a[1] * b[3] - a[0] * b[2]) + (a[2] * b[0] + a[3] * b[1]),
         (a[2] * b[3] - a[1] * b[0]) + (a[0] * b[1] + a[3] * b[2]),
         (a[3] * b[3] - a[0] * b[0]) - (a[2] * b[2] + a[1] * b[1])]
    tt = [M(0, 3), M(1, 3), M(2, 3)]  # rotate(identity, t) + 0 == t
    return np.array(r, np.float32), np.array(tt, np.float32)
