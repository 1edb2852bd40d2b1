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
    for name, m in sorted(meta["cases"].items()):
        data = z[f"jpg:{name}"].tobytes()
        exp = z[f"px:{name}"]
        rc, got = oracle.jpeg_decode_luma(data) if m["pinned"] == "luma" else oracle.jpeg_decode(data)
        assert rc == 0, name
        assert np.array_equal(got, exp), name
        kinds.add(name.rsplit("_", 1)[-1])
    assert len(meta["cases"]) >= 170
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
