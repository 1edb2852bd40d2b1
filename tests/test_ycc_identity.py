"""Exhaustive check of the colour conversion form k_fdct_color uses
(icx_kernels.hip rgb_ycc) against jccolor.c's rgb_ycc_convert (IJG 6b,
16-bit fixed point): over e = r - g and d = b - g the same integers come out
for every one of the 2^24 inputs, because each output's weights sum to a
power of two (19595 + 38470 + 7471 = 65536; 11059 + 21709 = 27439 + 5329 =
32768)."""
import numpy as np


def test_difference_form_equals_rgb_ycc_convert():
    v = np.arange(256, dtype=np.int32)
    g, b = np.meshgrid(v, v, indexing="ij")
    g, b = g.ravel(), b.ravel()
    for r in range(256):  # 64 Ki (g, b) pairs per r: small int32 arrays
        y = (19595 * r + 38470 * g + 7471 * b + 32768) >> 16
        cb = (-11059 * r - 21709 * g + 32768 * b + (128 << 16) + 32767) >> 16
        cr = (32768 * r - 27439 * g - 5329 * b + (128 << 16) + 32767) >> 16
        e, d = r - g, b - g
        y128 = g + ((19595 * e + 7471 * d + 32768 - (128 << 16)) >> 16)
        cb2 = ((d << 15) - 11059 * e + (128 << 16) + 32767) >> 16
        cr2 = ((e << 15) - 5329 * d + (128 << 16) + 32767) >> 16
        assert np.array_equal(y - 128, y128), r
        assert np.array_equal(cb, cb2), r
        assert np.array_equal(cr, cr2), r
