"""The progressive (SOF2) entropy decode of the device decoder's progressive
path (icx_progressive.cpp, host C++ in libicx: jdphuff.c semantics), checked
on the CPU through icx_debug_progressive_coefs.

Pin: a progressive file and a baseline file that Pillow encodes from the same
pixels with the same tables hold the same quantised coefficients (the encoder
runs one FDCT + quantisation, then writes either scan script), so the
progressive decode must equal the baseline oracle's (oracle/icx_oracle_decode.c,
itself pinned by tests/golden/decode_golden.*) block for block — DC
successive approximation, AC spectral selection, refinement scans, EOB runs
and restart intervals included."""
import io

import numpy as np
import pytest
from PIL import Image

from icx import _native as N
from icx.core import jpeg_info, progressive_coefs
from tests.oracle_ffi import load_decode_golden, noise, smooth


def _twins(img, **kw):
    pil = Image.fromarray(np.ascontiguousarray(img[:, :, ::-1]) if img.ndim == 3 else img)
    a, b = io.BytesIO(), io.BytesIO()
    pil.save(a, "JPEG", **kw)
    pil.save(b, "JPEG", progressive=True, **kw)
    return a.getvalue(), b.getvalue()


CASES = [((64, 64), 2, 95), ((137, 251), 2, 90), ((100, 77), 0, 75), ((99, 130), 1, 85), ((33, 1), 2, 80),
         ((1, 17), 0, 50), ((16, 16), 2, 100), ((40, 72), 2, 1), ((720, 1280), 2, 95)]


@pytest.mark.parametrize("shape,sub,q", CASES)
def test_progressive_coefficients_equal_baseline_twin(oracle, shape, sub, q):
    h, w = shape
    img = (noise if (h * w) % 2 else smooth)(h, w, h + w)
    base, prog = _twins(img, quality=q, subsampling=sub)
    assert np.array_equal(progressive_coefs(prog), oracle.jpeg_coefs(base))


@pytest.mark.parametrize("shape,q", [((121, 83), 95), ((1, 1), 75), ((66, 130), 30)])
def test_progressive_grey_equals_baseline_twin(oracle, shape, q):
    img = smooth(*shape, 11)[:, :, 1].copy()
    base, prog = _twins(img, quality=q)
    assert np.array_equal(progressive_coefs(prog), oracle.jpeg_coefs(base))


@pytest.mark.parametrize("rst", [dict(restart_marker_blocks=1), dict(restart_marker_blocks=3),
                                 dict(restart_marker_rows=1)])
def test_progressive_restart_intervals(oracle, rst):
    img = noise(77, 133, 9)
    base, prog = _twins(img, quality=90, subsampling=2, **rst)
    assert b"\xff\xdd" in prog and b"\xff\xd0" in prog
    assert np.array_equal(progressive_coefs(prog), oracle.jpeg_coefs(base))


def test_golden_progressive_files_parse_and_decode():
    meta, jpgs, pxs = load_decode_golden()
    names = [k for k in jpgs if meta["cases"][k].get("progressive")]
    assert len(names) >= 10
    for k in names:
        st, w, h, n = jpeg_info(jpgs[k])
        c = meta["cases"][k]
        assert st == N.OK and (w, h, n) == (c["w"], c["h"], c["ncomp"]), k
        assert progressive_coefs(jpgs[k]).shape[1] == 64


def _sos_offsets(data):
    return [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]


def test_truncated_scan_script_is_left_to_the_host():
    """A file whose scans stop before AC 1..5 are fully refined is what the
    JDK would block-smooth (jdcoefct.c smoothing_ok): unsupported, the
    pipeline decodes it on the host."""
    _, prog = _twins(smooth(64, 96, 5), quality=90, subsampling=2)
    sos = _sos_offsets(prog)
    assert len(sos) == 10  # libjpeg's simple progression for YCbCr
    for k in (1, 5, 9):
        cut = prog[:sos[k]] + b"\xff\xd9"
        with pytest.raises(N.IcxError) as e:
            progressive_coefs(cut)
        assert e.value.status == N.E_UNSUPPORTED, k


def test_progressive_refusals():
    base, prog = _twins(noise(48, 64, 3), quality=90, subsampling=2)
    sos = _sos_offsets(prog)
    with pytest.raises(N.IcxError) as e:  # cut inside a scan: the scan runs out of data
        progressive_coefs(prog[:sos[3] + 40])
    assert e.value.status == N.E_CORRUPT
    with pytest.raises(N.IcxError) as e:  # no EOI after the last scan
        progressive_coefs(prog[:-2])
    assert e.value.status == N.E_CORRUPT
    with pytest.raises(N.IcxError) as e:  # a sequential file is not this entry's
        progressive_coefs(base)
    assert e.value.status == N.E_INVALID
    bad = bytearray(prog)
    bad[sos[2] + 30] ^= 0x5A  # flipped entropy byte: never a crash, any of these statuses
    try:
        progressive_coefs(bytes(bad))
    except N.IcxError as x:
        assert x.status in (N.E_CORRUPT, N.E_UNSUPPORTED)
