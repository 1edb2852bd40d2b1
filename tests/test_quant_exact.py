"""Exhaustive proof of the float quantiser used by k_huff (icx_kernels.hip
quant / the AC loop) against jcdctmgr.c's integer division.

For divisor d = q<<3 (q = 1..255) and every |c| <= 32767 (int16 FDCT output):
  * |c| >= thr          <=>  (|c| + d/2) // d != 0   (the FDCT's candidate test)
  * floor(fma(|c|, frcp, fbias)) == (|c| + d/2) // d  for every |c|, zero
    quotients included, so k_huff's nonzero test fma(...) >= 1 is exact
  * frexp exponent of that fma result == bit length of the quotient
with thr/frcp/fbias computed exactly as make_node (icx_runtime.cpp) does, in
IEEE float32.  fma is emulated exactly: the float64 product of two float32
values is exact and the sum spans < 53 bits here, so one final rounding to
float32 reproduces v_fma_f32.
"""
import numpy as np


def test_float_quantiser_is_exact():
    c = np.arange(0, 32768, dtype=np.int64)
    cf = c.astype(np.float32).astype(np.float64)
    for q in range(1, 256):
        d = q << 3
        r = np.float32(1.0) / np.float32(d)
        b = (np.float32(d >> 1) + np.float32(0.5)) * r
        thr = np.float32(d - (d >> 1))
        want = (c + (d >> 1)) // d
        nz = c.astype(np.float32) >= thr
        assert np.array_equal(nz, want != 0), q
        y = (cf * np.float64(r) + np.float64(b)).astype(np.float32)
        got = y.astype(np.int64)  # v_cvt_u32_f32 truncates; y >= 0
        assert np.array_equal(got, want), q
        assert np.array_equal(y >= np.float32(1.0), want != 0), q
        exp = np.frexp(y[nz])[1]
        bl = np.floor(np.log2(want[nz].astype(np.float64))).astype(np.int64) + 1
        assert np.array_equal(exp, bl), q
