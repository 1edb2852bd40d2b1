"""C-ABI boundary checks that need no GPU: libicx.so loads, exports every
symbol include/icx.h declares, and its pure host helpers agree with the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

import icx
from icx import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "icx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(icx_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_all_header_symbols():
    lib = ctypes.CDLL(N.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(N.EXPORTS) == syms


def test_abi_version_and_status_strings():
    lib = N.load()
    assert lib.icx_abi_version() == 5
    assert lib.icx_status_string(N.E_BUFFER) == b"output buffer too small"
    assert b"refuses" in lib.icx_status_string(N.E_REFUSED)
    assert lib.icx_jpeg_header_size(N.BGR24) == 623 and lib.icx_jpeg_header_size(N.GRAY8) == 328
    assert lib.icx_jpeg_header_size_layout(N.BGR24, N.TABLES_GROUPED) == 607
    assert lib.icx_jpeg_header_size_layout(N.GRAY8, N.TABLES_GROUPED) == 324
    assert lib.icx_jpeg_header_size_layout(N.BGR24, N.TABLES_SEPARATE) == 623


def test_quality_tables_match_oracle(oracle):
    qs = [0.0, -1.0, 0.001, 0.01, 0.015625, 0.0078125, 0.1, 0.125, 0.2421875, 0.25, 0.3, 0.33, 0.49999, 0.5,
          0.51, 0.75, 0.95, 0.99, 1.0, 1.5]
    qs += list(np.random.default_rng(1).uniform(0, 1, 200))
    for q in qs:
        assert icx.quality_tables(q) == oracle.qtables(q), q


def test_host_helpers_match_oracle(oracle):
    rng = np.random.default_rng(2)
    for _ in range(300):
        w, h = int(rng.integers(1, 40000)), int(rng.integers(1, 40000))
        assert icx.subsampling_factor(w, h) == oracle.subsampling(w, h)
        s = float(rng.uniform(0.01, 1.0))
        assert icx.scaled_dims(w, h, s) == oracle.scaled_dims(w, h, s)
    key = N.SimilarityKey()
    N.load().icx_create_key(3840, 2160, 5 * 1024 * 1024 + 7, ctypes.byref(key))
    assert (key.width_bucket, key.height_bucket, key.size_bucket) == oracle.create_key(3840, 2160, 5 * 1024 * 1024 + 7)


def test_num_blocks():
    lib = N.load()
    assert lib.icx_num_blocks(3840, 2160, N.BGR24) == 194400
    assert lib.icx_num_blocks(1920, 1080, N.BGR24) == 120 * 68 * 6
    assert lib.icx_num_blocks(37, 29, N.GRAY8) == 5 * 4


def test_null_arguments_rejected_without_gpu():
    lib = N.load()
    assert lib.icx_create(0, None) == N.E_NULL
    assert lib.icx_compress_jpg_to_stream(None, None, 0.25, None, 0, None) == N.E_NULL
    assert lib.icx_compress_jpg_batch(None, None, 0) == N.E_NULL


def test_pool_arguments_rejected_without_gpu():
    """icx_pool_* validates its arguments before touching a device."""
    lib = N.load()
    p = ctypes.c_void_p()
    assert lib.icx_pool_create(None, 1, ctypes.byref(p)) == N.E_NULL
    devs = (ctypes.c_int32 * 1)(0)
    assert lib.icx_pool_create(devs, 0, ctypes.byref(p)) == N.E_INVALID
    assert lib.icx_pool_create(devs, 1, None) == N.E_NULL
    assert lib.icx_pool_size(None) == 0 and not lib.icx_pool_context(None, 0)
    assert lib.icx_pool_compress_jpg_batch(None, None, 0) == N.E_NULL
    assert lib.icx_pool_decode_jpg_batch(None, None, 0) == N.E_NULL
    assert lib.icx_pool_png_fit_batch(None, None, 0) == N.E_NULL
    lib.icx_pool_destroy(None)


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setattr(N, "LIB_PATH", "/nonexistent/libicx.so")
    with pytest.raises(N.NativeLibraryError):
        N.load()


def test_self_check_vectors_match_oracle(oracle):
    """icx_create's device self-check compares two known-answer files with
    what the context's GPU encodes; the known answers (length, FNV-1a 64)
    are the CPU oracle's files for the same images at q = 0.75."""
    L = N.load()

    def fnv(b):
        h = 0xcbf29ce484222325
        for x in b:
            h = ((h ^ x) * 0x100000001b3) & 0xffffffffffffffff
        return h

    for grey in (0, 1):
        px = np.zeros((16, 16) if grey else (16, 16, 3), np.uint8)
        dig, n = ctypes.c_uint64(), ctypes.c_int64()
        L.icx_debug_self_check_image(grey, px.ctypes.data, ctypes.byref(dig), ctypes.byref(n))
        assert len(np.unique(px)) > 64  # busy content: many AC codes
        data = oracle.encode(px, 0.75)
        assert (len(data), fnv(data)) == (n.value, dig.value), grey
