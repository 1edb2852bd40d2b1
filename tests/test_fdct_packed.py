"""Exactness of k_fdct_color's packed column pass (icx_kernels.hip
fdct_col_pair), restated in numpy: two columns ride as the low and high
int16 halves of one dword, the butterflies and the DC/Nyquist sums are
v_pk_add_u16 / v_pk_sub_u16 (each half wraps mod 2^16 on its own) and
v_pk_ashrrev_i16, the rotations the same dot2 chains as fdct8<1, true> on
operand pairs picked from the halves by v_perm, and each output leaves as the
high half of its int32 (the d16_hi form).  Equal to jpeg_fdct_islow's column
pass for every input the row pass can produce: the row outputs lie in
[-4096, 4080] (tests/test_ycc_identity.py), so every packed partial fits
int16 and no half ever wraps; the box corners bound the linear partials.
"""
import numpy as np

from tests.test_ycc_identity import EVEN, ODD, _corners, _ijg


def _wrap16(x):
    return ((x + 32768) & 0xFFFF) - 32768  # one 16-bit half of a packed register


def _packed_columns(d):
    """fdct_col_pair on one column's values (each half is independent), with
    the int16 wrap of every packed op applied."""
    p = [_wrap16(np.asarray(v, dtype=np.int64)) for v in d]
    add = lambda a, b: _wrap16(a + b)  # noqa: E731
    sub = lambda a, b: _wrap16(a - b)  # noqa: E731
    t0, t7, t1, t6 = add(p[0], p[7]), sub(p[0], p[7]), add(p[1], p[6]), sub(p[1], p[6])
    t2, t5, t3, t4 = add(p[2], p[5]), sub(p[2], p[5]), add(p[3], p[4]), sub(p[3], p[4])
    t10, t13, t11, t12 = add(t0, t3), sub(t0, t3), add(t1, t2), sub(t1, t2)
    t10r = add(t10, 2)
    o = [None] * 8
    o[0] = add(t10r, t11) >> 2  # v_pk_ashrrev_i16 by 2
    o[4] = sub(t10r, t11) >> 2
    rnd = 1 << 15
    for n, (a, b) in EVEN.items():
        acc = 2 * a * t12 + 2 * b * t13 + rnd
        assert np.abs(acc).max() < 2 ** 31
        o[n] = _wrap16(acc >> 16)
    for n, w in ODD.items():
        acc = 2 * (w[0] * t4 + w[1] * t5 + w[2] * t6 + w[3] * t7) + rnd
        assert np.abs(acc).max() < 2 ** 31
        o[n] = _wrap16(acc >> 16)
    # no packed partial may have wrapped: the exact values fit int16
    for t in (t0, t7, t1, t6, t2, t5, t3, t4, t10, t11, t12, t13):
        assert t.min() >= -32768 and t.max() <= 32767
    return o


def test_packed_column_pair_equals_jpeg_fdct_islow_columns():
    rng = np.random.default_rng(11)
    lo, hi = -4096, 4080  # the row pass's output range
    cols = [np.concatenate([c, rng.integers(lo, hi + 1, 300_000)]) for c in _corners(lo, hi)]
    ref = _ijg(cols, 1)
    got = _packed_columns(cols)
    for n in range(8):
        assert np.array_equal(ref[n], got[n]), n


def test_packed_sums_stay_inside_int16_at_the_extremes():
    # |t10 + t11| reaches 8 * 4096 = 32768 only for an all -4096 column; the
    # rounding constant then gives -32766, and +4080 everywhere 32640 + 2
    for v in (-4096, 4080):
        col = [np.array([v], dtype=np.int64)] * 8
        assert np.array_equal(_ijg(col, 1)[0], _packed_columns(col)[0])
