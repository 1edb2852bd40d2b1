"""Pins the CPU decode oracle (row A11) against the committed golden vectors:
libjpeg-turbo 3.1.4 decodes of Pillow-encoded files (tests/golden/
gen_decode_golden.py), and against this repo's own encoder through the
coefficient domain."""
import numpy as np
import pytest

from tests.oracle_ffi import load_decode_golden, smooth


@pytest.fixture(scope="module")
def dgolden():
    return load_decode_golden()


def test_decode_matches_golden(oracle, dgolden):
    meta, jpgs, pxs = dgolden
    n = 0
    for name, data in jpgs.items():
        rc, img = oracle.jpeg_decode(data)
        if meta["cases"][name].get("unsupported"):
            assert rc == 5, name
            continue
        assert rc == 0, (name, rc)
        assert img.shape == pxs[name].shape and np.array_equal(img, pxs[name]), name
        n += 1
    assert n == 111


@pytest.mark.parametrize("s", [2, 3, 4])
def test_decode_source_subsampling(oracle, dgolden, s):
    """ImageReadParam.setSourceSubsampling(s, s, 0, 0) keeps pixels (x*s, y*s)
    (ImageCompression.java:150-153)."""
    meta, jpgs, pxs = dgolden
    for name in ("c130x250_s2_q95", "c66x130_s1_q50", "g47x61_q90", "rst7_130x250_444"):
        rc, img = oracle.jpeg_decode(jpgs[name], s)
        assert rc == 0
        assert np.array_equal(img, pxs[name][::s, ::s]), (name, s)


def test_info_and_refusals(oracle, dgolden):
    meta, jpgs, _ = dgolden
    for name, data in jpgs.items():
        rc, w, h, n = oracle.jpeg_info(data)
        c = meta["cases"][name]
        assert (w, h, n) == (c["w"], c["h"], c["ncomp"]), name
        assert rc == (5 if c.get("unsupported") else 0)
    assert oracle.jpeg_info(b"\x00\x01garbage")[0] == 6
    good = jpgs["c48x64_s2_q95"]
    assert oracle.jpeg_decode(good[: len(good) // 3])[0] in (0, 6)  # truncated: never crashes


def test_coefficients_of_own_encodes(oracle):
    """decode(encode(img, q)) coefficients == quantised FDCT of img: the two
    restatements (encoder and decoder) agree in the coefficient domain."""
    for (h, w), q in [((48, 64), 0.25), ((37, 53), 0.9), ((16, 16), 1.0)]:
        img = smooth(h, w, h * w)
        data = oracle.encode(img, q)
        co = oracle.jpeg_coefs(data)
        raw = oracle.fdct(img).astype(np.int32)  # zig-zag, x8 scale
        lum, chrom = oracle.qtables(q)
        zz = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34,
                       27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44,
                       51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
        qt = np.array([lum if (b % 6) < 4 else chrom for b in range(raw.shape[0])])[:, zz] * 8
        quant = np.sign(raw) * ((np.abs(raw) + qt // 2) // qt)
        assert np.array_equal(co[:, zz], quant), (h, w, q)


def test_libicx_header_colour_rules_match_oracle(oracle, dgolden):
    """libicx's header parse (icx_jpeg_info, host code, no GPU) settles the
    colour-space cases as the oracle does: the JDK's Adobe override also next
    to a JFIF marker, IS_EXIF = the first saved COM/APPn marker is an APP1
    (imageioJPEG.c); pixels of the supported ones are checked on the GPU."""
    from icx.core import jpeg_info
    meta, jpgs, _ = dgolden
    n = 0
    for name, data in jpgs.items():
        c = meta["cases"][name]
        if not c.get("colour"):
            continue
        st = jpeg_info(data)[0]
        if c.get("progressive"):
            assert st == 0, name  # progressive files are the device path's too
        else:
            assert st == (5 if c.get("unsupported") else 0), (name, st)
        n += 1
    assert n == 11
