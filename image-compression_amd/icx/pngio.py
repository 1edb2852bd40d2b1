"""PNG writer of the PNG path: libicx's icx_png_encode (C++ on the calling
host thread; ctypes releases the GIL, so the batch driver's writer pool
encodes one image per thread).

Reference: ImageCompressionPng.java:70, ImageIO.write(img, "png", file).
The JDK writer's row-filter choice (RowFilter.filterRow), default deflate
level (4) and 32 KiB IDAT chunks are restated (icx_png.cpp); its deflate
bytes depend on the JDK's zlib and are not pinnable here (no JDK, SURVEY.md
§8c): parity is on decoded pixels, dimensions, colour type and bit depth,
and the per-row filter choice is checked against tests/png_ref.py.
"""
import ctypes

import numpy as np

from . import _native as N


def encode_png(img, fmt=None, level: int = -1) -> bytes:
    """img: host (H, W) grey, (H, W, 3) BGR or (H, W, 4) ABGR uint8 array,
    (H, W) uint16 grey (TYPE_USHORT_GRAY, a 16-bit PNG), an IndexedImage
    (TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY: a palette or 1-bit grey PNG, as
    PNGMetadata.initialize picks for its colour map), or another icx_fmt
    given explicitly -> PNG file bytes.  level -1 = PNGImageWriter's default."""
    from .core import IndexedImage, _image_struct
    lib = N.load()
    im, keep = _image_struct(img if isinstance(img, IndexedImage) else np.ascontiguousarray(img), fmt)
    cap = lib.icx_png_bound(ctypes.byref(im))
    if cap == 0:
        raise N.IcxError(N.E_UNSUPPORTED, "image too large for one IDAT chunk")
    out = np.empty(cap, np.uint8)
    n = ctypes.c_size_t()
    st = lib.icx_png_encode(ctypes.byref(im), int(level), out.ctypes.data, cap, ctypes.byref(n))
    if st != N.OK:
        raise N.IcxError(st, f"icx_png_encode: {lib.icx_status_string(st).decode()}")
    return out[:n.value].tobytes()


def write_png(path, img, fmt=None) -> None:
    data = encode_png(img, fmt)
    with open(path, "wb") as f:
        f.write(data)
