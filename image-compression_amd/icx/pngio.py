"""Minimal PNG writer (zlib deflate, filter type 0) for the PNG path's output.

The reference writes PNG through the JDK's PNGImageWriter
(ImageCompressionPng.java:70); its deflate bytes are out of scope
(SURVEY.md §8f rank 2).  Parity for PNG is on decoded pixels and dimensions.
"""
import struct
import zlib

import numpy as np


def _chunk(tag, data):
    c = struct.pack(">I", len(data)) + tag + data
    return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_png(img: np.ndarray, level: int = 6) -> bytes:
    """img: (H, W, 3) BGR or (H, W) grey uint8."""
    if img.ndim == 2:
        rgb, ctype = img, 0
    else:
        rgb, ctype = np.ascontiguousarray(img[:, :, ::-1]), 2
    h, w = rgb.shape[:2]
    raw = np.empty((h, 1 + rgb[0].size), np.uint8)
    raw[:, 0] = 0
    raw[:, 1:] = rgb.reshape(h, -1)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr) +
            _chunk(b"IDAT", zlib.compress(raw.tobytes(), level)) + _chunk(b"IEND", b""))


def write_png(path, img: np.ndarray) -> None:
    with open(path, "wb") as f:
        f.write(encode_png(img))
