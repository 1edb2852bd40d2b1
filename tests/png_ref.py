"""Reference PNG filter/encoder in numpy (test infrastructure only): the
per-row filter choice that libicx's icx_png_encode must reproduce.

The reference writes PNG through the JDK's PNGImageWriter
(ImageCompressionPng.java:70).  Restated from OpenJDK's published
com.sun.imageio.plugins.png sources (not in /root/reference, no JDK here:
SURVEY.md §8c): RowFilter.filterRow costs None as the sum of the row's
unsigned bytes and Sub / Up / Average / Paeth as the sum of |curr -
predictor| over ints (the unwrapped difference), keeping the first strictly
smallest (ties: the lower type); PNGImageWriter deflates at its default level
4 and IDATOutputStream cuts the stream into 32768-byte IDAT chunks.  The
deflate bytes are not pinned (they depend on the JDK's zlib) — parity for PNG
is on decoded pixels, dimensions, colour type and bit depth, plus the filter
choice row for row.
"""
import struct
import zlib

import numpy as np


def _chunk(tag, data):
    c = struct.pack(">I", len(data)) + tag + data
    return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def filter_rows(raw: np.ndarray, bpp: int) -> np.ndarray:
    """raw (h, rowbytes) u8 -> (h, 1 + rowbytes) u8 with RowFilter.filterRow's
    per-row choice (None: sum of unsigned bytes; the others: sum of |int
    difference|; ties: the lower filter type)."""
    h, n = raw.shape
    x = raw.astype(np.int16)
    a = np.zeros_like(x)
    a[:, bpp:] = x[:, :-bpp]                  # left
    b = np.zeros_like(x)
    b[1:] = x[:-1]                            # up
    c = np.zeros_like(x)
    c[1:, bpp:] = x[:-1, :-bpp]               # up-left
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    paeth = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))
    best_cost = None
    out = np.empty((h, n + 1), np.uint8)
    for ftype, pred in enumerate((None, a, b, (a + b) >> 1, paeth)):
        diff = x if pred is None else x - pred            # int16: the unwrapped difference
        res = diff.astype(np.uint8)                       # the residual byte (mod 256)
        cost = np.abs(diff.astype(np.int32)).sum(axis=1)  # None: x >= 0, the unsigned bytes
        if best_cost is None:
            best_cost = cost
            out[:, 1:] = res
            out[:, 0] = 0
            continue
        take = cost < best_cost
        if take.any():
            out[take, 1:] = res[take]
            out[take, 0] = ftype
            best_cost = np.where(take, cost, best_cost)
    return out


def encode_png(img: np.ndarray, level: int = 4) -> bytes:
    """img: (H, W, 3) BGR, (H, W, 4) ABGR, (H, W) grey uint8 or (H, W) grey
    uint16 (TYPE_USHORT_GRAY: a 16-bit PNG)."""
    depth = 16 if img.dtype == np.uint16 else 8
    if img.ndim == 2:
        ctype, bpp = 0, depth // 8
        rgb = img.astype(">u2").view(np.uint8) if depth == 16 else img
    else:
        bpp = img.shape[2]
        rgb, ctype = np.ascontiguousarray(img[:, :, ::-1]), 2 if bpp == 3 else 6
    h, w = img.shape[:2]
    raw = filter_rows(np.ascontiguousarray(rgb).reshape(h, -1), bpp)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0)
    z = zlib.compress(raw.tobytes(), level)
    idat = b"".join(_chunk(b"IDAT", z[i:i + 32768]) for i in range(0, len(z), 32768))
    return b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) + idat + _chunk(b"IEND", b"")


def write_png(path, img: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(encode_png(img))
