"""Exactness of the integer forms k_fdct_color computes with v_dot2_i32_i16
(icx_kernels.hip rgb_ycc / fdct8), restated here in numpy:

* colour: jccolor.c's rgb_ycc_convert (IJG 6b, 16-bit fixed point) over the
  negated differences (g - r, g - b) as int16 pairs: the same integers for
  every one of the 2^24 inputs, because each output's weights sum to a power
  of two (19595 + 38470 + 7471 = 65536; 11059 + 21709 = 27439 + 5329 =
  32768), and every weight of the pair form fits int16 (32768 d =
  -32768 (g - b)).
* DCT: jfdctint.c's jpeg_fdct_islow rotations expanded per input (d7 =
  t4*2446 + z1*-7373 + z3*-16069 + z5 -> t4*-11363 + t5*9633 + t6*-6436 +
  t7*2260, ...) equal IJG's products for every pass, the column pass's
  doubled weights leave DESCALE(x, 15) in bits 16.. of 2x + 2^15, and every
  operand the dot2 instructions take fits int16 (checked at the extreme
  inputs: the t* are linear in the samples, so the box corners bound them).
"""
import numpy as np

CONST_BITS, PASS1_BITS = 13, 2


def test_pair_form_equals_rgb_ycc_convert():
    v = np.arange(256, dtype=np.int32)
    g, b = np.meshgrid(v, v, indexing="ij")
    g, b = g.ravel(), b.ravel()
    ky, kc = 32768 - (128 << 16), (128 << 16) + 32767
    for r in range(256):  # 64 Ki (g, b) pairs per r: small int32 arrays
        y = (19595 * r + 38470 * g + 7471 * b + 32768) >> 16
        cb = (-11059 * r - 21709 * g + 32768 * b + (128 << 16) + 32767) >> 16
        cr = (32768 * r - 27439 * g - 5329 * b + (128 << 16) + 32767) >> 16
        ne, nd = g - r, g - b  # the packed int16 pair
        y128 = g + ((-19595 * ne - 7471 * nd + ky) >> 16)
        cb2 = (11059 * ne - 32768 * nd + kc) >> 16
        cr2 = (-32768 * ne + 5329 * nd + kc) >> 16
        assert np.array_equal(y - 128, y128), r
        assert np.array_equal(cb, cb2), r
        assert np.array_equal(cr, cr2), r


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _butterfly(d):
    t0, t7, t1, t6 = d[0] + d[7], d[0] - d[7], d[1] + d[6], d[1] - d[6]
    t2, t5, t3, t4 = d[2] + d[5], d[2] - d[5], d[3] + d[4], d[3] - d[4]
    return t0 + t3, t1 + t2, t1 - t2, t0 - t3, t4, t5, t6, t7  # t10 t11 t12 t13 t4..t7


def _ijg(d, pas):
    """jpeg_fdct_islow, one pass (jfdctint.c), int64 columns of d."""
    t10, t11, t12, t13, t4, t5, t6, t7 = _butterfly(d)
    sh = CONST_BITS - PASS1_BITS if pas == 0 else CONST_BITS + PASS1_BITS
    o = [None] * 8
    if pas == 0:
        o[0], o[4] = (t10 + t11) << PASS1_BITS, (t10 - t11) << PASS1_BITS
    else:
        o[0], o[4] = _descale(t10 + t11, PASS1_BITS), _descale(t10 - t11, PASS1_BITS)
    z1 = (t12 + t13) * 4433
    o[2], o[6] = _descale(z1 + t13 * 6270, sh), _descale(z1 - t12 * 15137, sh)
    z1, z2, z3, z4 = t4 + t7, t5 + t6, t4 + t6, t5 + t7
    z5 = (z3 + z4) * 9633
    t4, t5, t6, t7 = t4 * 2446, t5 * 16819, t6 * 25172, t7 * 12299
    z1, z2, z3, z4 = z1 * -7373, z2 * -20995, z3 * -16069 + z5, z4 * -3196 + z5
    o[7], o[5] = _descale(t4 + z1 + z3, sh), _descale(t5 + z2 + z4, sh)
    o[3], o[1] = _descale(t6 + z2 + z3, sh), _descale(t7 + z1 + z4, sh)
    return o


# (output, (w12, w13)) and (output, (w4, w5, w6, w7)) of fdct8's dot2 chains
EVEN = {2: (4433, 10703), 6: (-10704, 4433)}
ODD = {7: (-11363, 9633, -6436, 2260), 5: (9633, 2261, -11362, 6437),
       3: (-6436, -11362, -2259, 9633), 1: (2260, 6437, 9633, 11363)}


def _dot2_form(d, pas, hi):
    t10, t11, t12, t13, t4, t5, t6, t7 = _butterfly(d)
    for t in (t12, t13, t4, t5, t6, t7):  # the packed operands
        assert t.min() >= -32768 and t.max() <= 32767
    sh = CONST_BITS - PASS1_BITS if pas == 0 else CONST_BITS + PASS1_BITS
    k = 2 if hi else 1
    rnd = 1 << (sh - 1 + (1 if hi else 0))
    o = [None] * 8
    if pas == 0:
        o[0], o[4] = (t10 + t11) << PASS1_BITS, (t10 - t11) << PASS1_BITS
    elif hi:
        o[0], o[4] = (t10 + t11 + 2) << 14, (t10 - t11 + 2) << 14
    else:
        o[0], o[4] = _descale(t10 + t11, PASS1_BITS), _descale(t10 - t11, PASS1_BITS)
    for n, (a, b) in EVEN.items():
        assert abs(k * a) < 32768 and abs(k * b) < 32768
        o[n] = k * a * t12 + k * b * t13 + rnd
    for n, w in ODD.items():
        assert all(abs(k * x) < 32768 for x in w)
        o[n] = k * (w[0] * t4 + w[1] * t5 + w[2] * t6 + w[3] * t7) + rnd
    for n in range(8):
        assert np.abs(o[n]).max() < 2 ** 31  # int32 accumulators
        if hi:
            o[n] = (o[n] >> 16).astype(np.int16).astype(np.int64)  # the d16_hi store
        elif n not in (0, 4):
            o[n] = o[n] >> sh
    return o


def _corners(lo, hi):
    bits = (np.arange(256)[:, None] >> np.arange(8)[None, :]) & 1
    return [np.where(bits[:, c] == 1, hi, lo).astype(np.int64) for c in range(8)]


def test_fdct_dot2_form_equals_jpeg_fdct_islow():
    rng = np.random.default_rng(5)
    rows = [np.concatenate([c, rng.integers(-128, 128, 200_000)]) for c in _corners(-128, 127)]
    out = _ijg(rows, 0)
    assert all(np.array_equal(a, b) for a, b in zip(out, _dot2_form(rows, 0, False)))
    lo = min(int(o.min()) for o in out)
    hi = max(int(o.max()) for o in out)
    assert lo >= -4096 and hi <= 4096
    cols = [np.concatenate([c, rng.integers(lo, hi + 1, 200_000)]) for c in _corners(lo, hi)]
    ref = _ijg(cols, 1)
    for h in (False, True):
        assert all(np.array_equal(a, b) for a, b in zip(ref, _dot2_form(cols, 1, h))), h
