"""Device decode of 4-component (CMYK / YCCK) JPEGs (SURVEY §8f rank 4,
ImageCompression.java:32-35, 113-157), libicx through the C ABI: quantised
coefficients equal the oracle's, CMYK samples equal libjpeg-turbo's
(tests/golden/gen_cmyk_golden.py: Pillow-written CMYK, their YCCK twins,
no Adobe marker), and the BGR frames the encoder gets equal the restated
RGB step (Pillow's Adobe-inverted CMYK + cmyk2rgb; TwelveMonkeys' ICC
conversion is parity unpinned) at source subsampling 1, 2, 3, alone and in
a batch with YCbCr files, into host and device memory."""
import numpy as np
import pytest

from icx import _native as N
from tests.oracle_ffi import smooth
from tests.test_cmyk_cpu import cmyk_golden

pytestmark = pytest.mark.gpu


def test_cmyk_coefficients_samples_and_pixels(codec, oracle):
    for name, (data, cmyk, bgr) in cmyk_golden().items():
        assert np.array_equal(codec.debug_decode_coefs(data), oracle.jpeg_coefs(data)), name
        assert np.array_equal(codec.debug_decode_cmyk(data), cmyk), name
        assert np.array_equal(codec.decode_jpg(data, subsampling=1), bgr), name
        for s in (2, 3):
            assert np.array_equal(codec.decode_jpg(data, subsampling=s), bgr[::s, ::s]), (name, s)


def test_cmyk_in_a_mixed_batch_to_device(codec, oracle):
    import io
    from PIL import Image
    g = cmyk_golden()
    ycc = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(smooth(70, 90, 3)[:, :, ::-1])).save(ycc, "JPEG", quality=95)
    datas = [g["ycck_130x66_rst"][0], ycc.getvalue(), g["cmyk_37x23"][0], g["noadobe_64x48"][0]]
    res = codec.decode_jpg_batch(datas, subsampling=0, device_out=True)
    for d, (st, img) in zip(datas, res):
        assert st == N.OK
        rc, ref = oracle.jpeg_decode(d)
        assert rc == 0 and np.array_equal(img.numpy(), ref)
