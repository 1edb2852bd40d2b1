"""The device decoder on damaged and 6b-only JPEGs (row A11), through the C
ABI: the JDK's IJG 6b reader recovers from truncated scans, bad Huffman codes
and restart markers out of sequence with warnings only
(ImageCompression.java:113-155), so libicx decodes such files as it does -
the device flags every departure from the clean case and the file is
entropy-decoded with 6b's recovery on a host thread (icx_seqdecode.cpp), its
IDCT, upsampling and colour on the device.  Bit-exact against the
libjpeg-turbo fixtures (tests/golden/gen_recovery_golden.py) and the oracle;
4:4:0 / 4:1:1 colour against the oracle's int_upsample (turbo upsamples h1v2
differently: its luma plane pins the rest)."""
import json
import os

import numpy as np
import pytest

from icx import _native as N
from tests.oracle_ffi import noise, smooth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def recovery():
    z = np.load(os.path.join(HERE, "golden", "recovery_golden.npz"))
    with open(os.path.join(HERE, "golden", "recovery_golden.json")) as f:
        meta = json.load(f)
    return meta, {k: z[f"jpg:{k}"].tobytes() for k in meta["cases"]}, z


def test_recovery_fixtures_in_one_batch(codec, oracle, recovery):
    """Every fixture (intact, truncated at 3..99.9 %, cut after a 0xFF or
    around an RSTn, EOI missing, bad codes, RSTn missing / duplicated /
    renumbered / after garbage, bad markers after the scan) in one batch."""
    meta, jpgs, z = recovery
    names = sorted(jpgs)
    res = codec.decode_jpg_batch([jpgs[k] for k in names], subsampling=1)
    n_ok = 0
    for name, (st, img) in zip(names, res):
        m = meta["cases"][name]
        if m["pinned"] == "error":
            assert st == N.E_CORRUPT, (name, st)
            continue
        assert st == N.OK, (name, st)
        rc, ref = oracle.jpeg_decode(jpgs[name])
        assert rc == 0 and np.array_equal(img, ref), name
        if m["pinned"] == "pixels":
            assert np.array_equal(img, z[f"px:{name}"]), name
        n_ok += 1
    assert n_ok >= 190


def test_recovery_coefficients_match_oracle(codec, oracle, recovery):
    meta, jpgs, _ = recovery
    for name in sorted(jpgs):
        if meta["cases"][name]["pinned"] == "error":
            continue
        ref = oracle.jpeg_coefs(jpgs[name])
        got = codec.debug_decode_coefs(jpgs[name])
        assert got.shape == ref.shape and np.array_equal(got, ref), name


def _damage(data, rng):
    s0 = data.index(b"\xff\xda")
    s0 += 2 + int.from_bytes(data[s0 + 2:s0 + 4], "big")
    n = len(data) - 2 - s0
    rst = [k for k in range(s0, len(data) - 1) if data[k] == 0xFF and 0xD0 <= data[k + 1] <= 0xD7]
    out = {"cut50": data[:s0 + n // 2], "cut97": data[:s0 + n * 97 // 100], "no_eoi": data[:-2]}
    bad = bytearray(data)
    a = s0 + int(rng.integers(n // 4, 3 * n // 4))
    bad[a:a + 8] = b"\xff\x00" * 4
    out["badcode"] = bytes(bad)
    if rst:
        k = rst[len(rst) // 3]
        out["rst_missing"] = data[:k] + data[k + 2:]
        out["rst_garbage"] = data[:k] + b"\x11\x22\x33" + data[k:]
    return out


@pytest.mark.parametrize("kind", ["smooth", "noise"])
def test_recovery_4k_matches_oracle(codec, oracle, kind):
    """4K q95 frames (the e2e leg's sources) damaged, with and without DRI:
    the device decode equals the oracle's, a whole batch at once."""
    import io
    from PIL import Image
    rng = np.random.default_rng(5)
    img = (smooth if kind == "smooth" else noise)(2160, 3840, 17)
    datas = []
    for kw in ({}, {"restart_marker_rows": 2}):
        buf = io.BytesIO()
        Image.fromarray(img[:, :, ::-1]).save(buf, "JPEG", quality=95, subsampling=2, **kw)
        datas += list(_damage(buf.getvalue(), rng).values())
    res = codec.decode_jpg_batch(datas, subsampling=1)
    for i, (d, (st, px)) in enumerate(zip(datas, res)):
        rc, ref = oracle.jpeg_decode(d)
        assert st == N.OK and rc == 0 and np.array_equal(px, ref), i


def test_recovery_device_inputs_and_subsampling(codec, oracle, recovery):
    """Damaged files resident in HBM (a CUDA tensor, a libicx buffer) and
    source subsampling s = 2, 3 on the recovery route."""
    import torch

    import icx
    meta, jpgs, _ = recovery
    names = ["c420_200x136_cut600", "rst_c420_136x200_rst_missing", "c444_noise_80x96_badcode",
             "grey_88x120_cut_after_ff", "c440_66x130_cut300", "rst_grey_88x120_rst_skip1"]
    for s in (1, 2, 3):
        for name in names:
            rc, ref = oracle.jpeg_decode(jpgs[name], s)
            assert rc == 0
            t_in = torch.from_numpy(np.frombuffer(jpgs[name], np.uint8).copy()).cuda()
            assert np.array_equal(codec.decode_jpg(t_in, subsampling=s), ref), (name, s)
            dev_in = icx.DeviceImage.from_host(codec, jpgs[name])
            img = codec.decode_jpg(dev_in, subsampling=s, device_out=True)
            assert np.array_equal(img.numpy(), ref), (name, s)


def test_440_and_411_decode_on_the_device(codec, oracle, recovery):
    """4:4:0 and 4:1:1 files (int_upsample replication in 6b) decode on the
    device, intact and damaged, at s = 1 and 2: equal to the oracle, whose
    luma plane libjpeg-turbo pins (test_recovery_cpu.py)."""
    meta, jpgs, _ = recovery
    names = [k for k, m in meta["cases"].items() if m["pinned"] == "luma"]
    assert len(names) >= 12
    for s in (1, 2):
        res = codec.decode_jpg_batch([jpgs[k] for k in names], subsampling=s)
        for name, (st, img) in zip(names, res):
            rc, ref = oracle.jpeg_decode(jpgs[name], s)
            assert st == N.OK and rc == 0 and np.array_equal(img, ref), (name, s)


def test_refused_flavours_on_the_device(codec):
    """Arithmetic / hierarchical / 12-bit: ICX_E_REFUSED with the SOF's
    dimensions (the reference's reader throws at read())."""
    import io
    from PIL import Image
    from icx.core import jpeg_info
    buf = io.BytesIO()
    Image.fromarray(noise(40, 56, 3)).save(buf, "JPEG", quality=90)
    base = buf.getvalue()
    sof = base.index(b"\xff\xc0")
    datas = []
    for m in (0xC9, 0xCA, 0xCB, 0xC5, 0xCD):
        d = bytearray(base)
        d[sof + 1] = m
        datas.append(bytes(d))
    d = bytearray(base)
    d[sof + 4] = 12
    datas.append(bytes(d))
    res = codec.decode_jpg_batch(datas + [base], subsampling=1)
    for d, (st, img) in zip(datas, res):
        assert st == N.E_REFUSED and jpeg_info(d) == (N.E_REFUSED, 56, 40, 3)
    assert res[-1][0] == N.OK
