"""4-component (CMYK / YCCK) JPEG decode, SURVEY §8f rank 4 (the reference reads
them through TwelveMonkeys, ImageCompression.java:32-35, 113-157).  CPU
checks: the oracle's decode equals libjpeg-turbo's CMYK samples for
Pillow-written CMYK files, their YCCK twins (Adobe transform 2: jdcolor.c
ycck_cmyk_convert) and a file without an Adobe marker; its BGR equals the
RGB step the build restates (Pillow's Adobe-inverted CMYK + cmyk2rgb;
TwelveMonkeys' ICC conversion: parity unpinned); the product's header parse
accepts them for the device decoder, and the device state machine (CPU
emulator) reproduces the oracle's coefficients."""
import os

import numpy as np

from icx import _native as N
from icx.core import jpeg_info
from tests.oracle_ffi import ROOT
from tests.test_decode_emu import emu, run  # noqa: F401  (the emulator fixture)

GOLD = os.path.join(ROOT, "tests", "golden", "cmyk_golden.npz")


def cmyk_golden():
    z = np.load(GOLD)  # allow_pickle=False: plain arrays
    names = sorted(k[:-4] for k in z.files if k.endswith(".jpg"))
    return {n: (z[n + ".jpg"].tobytes(), z[n + ".cmyk"], z[n + ".bgr"]) for n in names}


def test_oracle_cmyk_decode_matches_libjpeg_turbo(oracle):
    g = cmyk_golden()
    assert {n.split("_")[0] for n in g} == {"cmyk", "ycck", "noadobe"}
    for name, (data, cmyk, bgr) in g.items():
        rc, w, h, nc = oracle.jpeg_info(data)
        assert rc == 0 and nc == 4 and (h, w) == cmyk.shape[:2], name
        rc, got = oracle.jpeg_decode_cmyk(data)
        assert rc == 0 and np.array_equal(got, cmyk), name
        rc, px = oracle.jpeg_decode(data)
        assert rc == 0 and np.array_equal(px, bgr), name
        for s in (2, 3):
            rc, px = oracle.jpeg_decode(data, s)
            assert rc == 0 and np.array_equal(px, bgr[::s, ::s]), (name, s)


def test_ycck_twin_differs_and_product_parser_accepts(oracle):
    g = cmyk_golden()
    assert not np.array_equal(g["cmyk_64x48"][1], g["ycck_64x48"][1])  # the transform really runs
    for name, (data, cmyk, _) in g.items():
        st, w, h, nc = jpeg_info(np.frombuffer(data, np.uint8))
        assert st == N.OK and nc == 4 and (h, w) == cmyk.shape[:2], name
        assert oracle.jpeg_coefs(data).shape == (-(-w // 8) * -(-h // 8) * 4, 64), name


def test_cmyk_device_state_machine_matches_oracle(oracle, emu):
    """The device decoder's entropy stage (tests/dec_emu.cpp: the product's
    state machine, four one-block components per MCU, DC predictors per
    component reset at every restart interval, symbol pairs) against the
    oracle, and the lean walkers against the spec walkers from random
    states."""
    import ctypes
    emu.dec_emu_lean_check.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    emu.dec_emu_lean_check.restype = ctypes.c_long
    for k, (name, (data, _, _)) in enumerate(cmyk_golden().items()):
        ref = oracle.jpeg_coefs(data)
        for sub in (32, 160, 1024):
            rc, got, _ = run(emu, data, ref.shape[0], seed=k + 1, sub=sub)
            assert rc == 0 and np.array_equal(got, ref), (name, sub)
        buf = np.frombuffer(data, np.uint8)
        assert emu.dec_emu_lean_check(buf.ctypes.data, buf.size, 32, 300, k + 7) == 0, name
