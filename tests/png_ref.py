"""Reference PNG filter/encoder in numpy (test infrastructure only): the
per-row filter choice that libicx's icx_png_encode must reproduce.

The reference writes PNG through the JDK's PNGImageWriter
(ImageCompressionPng.java:70): per row it picks the filter (None, Sub, Up,
Average, Paeth) with the smallest sum of |filtered byte as signed|, then
deflates.  This writer uses the same row-filter heuristic (vectorised over the
whole image) and zlib; the deflate bytes themselves are not pinned (no JDK
here) — parity for PNG is on decoded pixels and dimensions.
"""
import struct
import zlib

import numpy as np


def _chunk(tag, data):
    c = struct.pack(">I", len(data)) + tag + data
    return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def filter_rows(raw: np.ndarray, bpp: int) -> np.ndarray:
    """raw (h, rowbytes) u8 -> (h, 1 + rowbytes) u8 with the per-row filter of
    minimum sum of absolute signed residuals (ties: the lower filter type)."""
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
        res = (x if pred is None else x - pred).astype(np.uint8)  # mod 256
        cost = np.abs(res.view(np.int8).astype(np.int32)).sum(axis=1)
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


def encode_png(img: np.ndarray, level: int = 6) -> bytes:
    """img: (H, W, 3) BGR, (H, W, 4) ABGR or (H, W) grey uint8."""
    if img.ndim == 2:
        rgb, ctype, bpp = img, 0, 1
    else:
        bpp = img.shape[2]
        rgb, ctype = np.ascontiguousarray(img[:, :, ::-1]), 2 if bpp == 3 else 6
    h, w = rgb.shape[:2]
    raw = filter_rows(rgb.reshape(h, -1), bpp)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) +
            _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + _chunk(b"IEND", b""))


def write_png(path, img: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(encode_png(img))
