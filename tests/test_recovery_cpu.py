"""The oracle's decode of damaged and 6b-only JPEGs,
pinned by libjpeg-turbo fixtures (tests/golden/gen_recovery_golden.py).

The reference reads through the JDK's IJG 6b reader
(ImageCompression.java:113-155), which recovers from damaged entropy data
with warnings only - a fake EOI at end of file, zero-filled MCUs after
insufficient data, symbol 0 for a bad Huffman code, jdmarker.c's restart
resynchronisation - so such files are compressed, not failed (:94-96).
Bit-exact: every pixel of each fixture (the luma plane only for 4:4:0 and
4:1:1, whose chroma upsampling libjpeg-turbo does differently)."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def recovery():
    z = np.load(os.path.join(HERE, "golden", "recovery_golden.npz"))
    with open(os.path.join(HERE, "golden", "recovery_golden.json")) as f:
        meta = json.load(f)
    return meta, z


def test_oracle_matches_every_recovery_fixture(oracle, recovery):
    meta, z = recovery
    kinds = set()
    errors = 0
    for name, m in sorted(meta["cases"].items()):
        data = z[f"jpg:{name}"].tobytes()
        if m["pinned"] == "error":  # libjpeg throws (after the scan: jpeg_finish_decompress)
            assert oracle.jpeg_decode(data)[0] == 6, name
            errors += 1
            continue
        exp = z[f"px:{name}"]
        rc, got = oracle.jpeg_decode_luma(data) if m["pinned"] == "luma" else oracle.jpeg_decode(data)
        assert rc == 0, name
        assert np.array_equal(got, exp), name
        kinds.add(name.rsplit("_", 1)[-1])
    assert len(meta["cases"]) >= 220 and errors >= 27
    for k in ("intact", "cut300", "ff", "eoi", "badcode", "missing", "dup", "wrong", "skip1", "garbage"):
        assert any(x.endswith(k) for x in kinds), k


def test_truncated_scan_leaves_later_mcus_grey(oracle, recovery):
    """After the MCU in which the data runs out, the rest of the (only)
    segment is zero coefficients: uniform 128 (jdhuff.c insufficient_data)."""
    meta, z = recovery
    data = z["jpg:c420_200x136_cut600"].tobytes()
    rc, px = oracle.jpeg_decode(data)
    assert rc == 0
    assert (px[-16:] == 128).all()
    coefs = oracle.jpeg_coefs(data)
    nz = np.flatnonzero(np.abs(coefs).sum(1))
    assert nz.size and (coefs[nz[-1] + 1:] == 0).all() and nz[-1] + 1 < len(coefs)


def test_refused_flavours(oracle):
    """Arithmetic coding, hierarchical and 12-bit files: the JDK reader's
    read() throws (status 8 -> FAILED_IO_ERROR); lossless (SOF3) and 8-bit
    progressive are read by another reader (status 5)."""
    import io
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.zeros((16, 24, 3), np.uint8)).save(buf, "JPEG", quality=90)
    base = bytearray(buf.getvalue())
    sof = base.index(b"\xff\xc0")
    for marker, rc in ((0xC9, 8), (0xCA, 8), (0xCB, 8), (0xC5, 8), (0xCD, 8), (0xC3, 5), (0xC2, 5)):
        f = bytearray(base)
        f[sof + 1] = marker
        got, w, h, n = oracle.jpeg_info(bytes(f))
        assert (got, w, h, n) == (rc, 24, 16, 3), hex(marker)
    f = bytearray(base)
    f[sof + 4] = 12  # sample precision
    assert oracle.jpeg_info(bytes(f))[:3] == (8, 24, 16)


def test_host_recovery_decode_equals_oracle(oracle, recovery):
    """libicx's host entropy decode with 6b recovery (icx_seqdecode.cpp, the
    route of the files the device decode flags) gives the oracle's
    coefficients on every fixture (no GPU: icx_debug_recovery_coefs)."""
    from icx.core import recovery_coefs
    meta, z = recovery
    import icx
    for name, m in sorted(meta["cases"].items()):
        data = z[f"jpg:{name}"].tobytes()
        if m["pinned"] == "error":
            assert oracle.jpeg_coefs(data) is None
            with pytest.raises(icx.IcxError) as e:
                recovery_coefs(data)
            assert e.value.status == icx.core.N.E_CORRUPT, name
            continue
        assert np.array_equal(recovery_coefs(data), oracle.jpeg_coefs(data)), name


def test_host_recovery_decode_fuzz(oracle):
    """Random damage (cuts, byte flips, planted 0xFF runs, RSTn removed or
    renumbered) on small files of every sampling layout: the host recovery
    decode equals the oracle bit for bit."""
    import io
    from PIL import Image
    from icx.core import recovery_coefs
    from tests.oracle_ffi import noise, smooth
    rng = np.random.default_rng(2026)
    n = 0
    for i in range(300):
        h, w = int(rng.integers(8, 90)), int(rng.integers(8, 90))
        img = smooth(h, w, i) if i % 2 else noise(h, w, i)
        kw = dict(quality=int(rng.integers(30, 100)), subsampling=int(rng.integers(0, 3)))
        if i % 3 == 0:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        buf = io.BytesIO()
        Image.fromarray(img if i % 5 else img[:, :, 0]).save(buf, "JPEG", **kw)
        d = bytearray(buf.getvalue())
        s0 = d.index(b"\xff\xda") + 2 + int.from_bytes(d[d.index(b"\xff\xda") + 2:d.index(b"\xff\xda") + 4], "big")
        for _ in range(int(rng.integers(1, 4))):
            op = int(rng.integers(0, 5))
            if op == 0:
                d = d[:int(rng.integers(s0, len(d)))]
            elif op == 1 and len(d) > s0 + 1:
                d[int(rng.integers(s0, len(d)))] = int(rng.integers(0, 256))
            elif op == 2 and len(d) > s0 + 8:
                a = int(rng.integers(s0, len(d) - 6))
                d[a:a + 6] = b"\xff\x00" * 3
            elif op == 3:
                r = [k for k in range(s0, len(d) - 1) if d[k] == 0xFF and 0xD0 <= d[k + 1] <= 0xD7]
                if r:
                    k = r[int(rng.integers(0, len(r)))]
                    d = d[:k] + d[k + 2:] if rng.random() < 0.5 else d[:k + 1] + bytes([0xD0 + int(rng.integers(0, 8))]) + d[k + 2:]
            else:
                a = int(rng.integers(s0, len(d) + 1))
                d = d[:a] + bytes(rng.integers(0, 256, int(rng.integers(1, 5)), dtype=np.uint8)) + d[a:]
        data = bytes(d)
        ref = oracle.jpeg_coefs(data)
        if ref is None:  # the JDK reader throws (a marker after the scan it cannot take)
            import icx
            with pytest.raises(icx.IcxError):
                recovery_coefs(data)
            continue
        assert np.array_equal(recovery_coefs(data), ref), (i, kw)
        n += 1
    assert n >= 200
