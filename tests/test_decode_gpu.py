"""Parity of the device JPEG decoder (row A11, libicx.so through the C ABI)
with the oracle and the golden decodes.  Bit-exact: quantised coefficients
after DC prediction, and decoded BGR / grey pixels, with and without restart
intervals, with source subsampling, for batches mixing layouts."""
import io

import numpy as np
import pytest

from icx import _native as N
from tests.oracle_ffi import load_decode_golden, noise, smooth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dgolden():
    return load_decode_golden()


def test_decode_coefficients_match_oracle(codec, oracle, dgolden):
    meta, jpgs, _ = dgolden
    for name, data in jpgs.items():
        if meta["cases"][name].get("unsupported"):
            continue
        ref = oracle.jpeg_coefs(data)
        got = codec.debug_decode_coefs(data)
        assert got.shape == ref.shape and np.array_equal(got, ref), name


def test_decode_pixels_match_golden_batch(codec, dgolden):
    """All golden files in one batch (grey, 4:2:0, 4:2:2, 4:4:4, DRI, q1..q100,
    and progressive files, which take the host-entropy / device-pixel path)."""
    meta, jpgs, pxs = dgolden
    names = list(jpgs)
    res = codec.decode_jpg_batch([jpgs[k] for k in names], subsampling=1)
    for name, (st, img) in zip(names, res):
        if meta["cases"][name].get("unsupported") and not meta["cases"][name].get("progressive"):
            assert st == N.E_UNSUPPORTED, name
            continue
        assert st == N.OK, (name, st)
        assert img.shape == pxs[name].shape and np.array_equal(img, pxs[name]), name


def test_decode_to_device_and_subsampling(codec, oracle, dgolden):
    import torch

    import icx
    meta, jpgs, pxs = dgolden
    for s in (1, 2, 3):
        for name in ("c130x250_s2_q95", "c66x130_s1_q50", "g47x61_q90", "rst7_130x250_444", "c7x9_s2_q95"):
            img = codec.decode_jpg(jpgs[name], subsampling=s, device_out=True)
            assert isinstance(img, icx.DeviceImage)
            assert np.array_equal(img.numpy(), pxs[name][::s, ::s]), (name, s)
            # device-resident compressed input: libicx buffer and CUDA tensor
            dev_in = icx.DeviceImage.from_host(codec, jpgs[name])
            assert np.array_equal(codec.decode_jpg(dev_in, subsampling=s), pxs[name][::s, ::s]), (name, s)
            t_in = torch.from_numpy(np.frombuffer(jpgs[name], np.uint8).copy()).cuda()
            assert np.array_equal(codec.decode_jpg(t_in, subsampling=s), pxs[name][::s, ::s]), (name, s)


def test_decode_then_fit_in_hbm_matches_oracle(codec, oracle, dgolden):
    """decode -> compressJpgWithTargetSize with the frame kept in HBM
    (DeviceImage), as icx.pipeline runs it: same bytes as the oracle on the
    oracle's decode."""
    meta, jpgs, pxs = dgolden
    for name in ("c130x250_s2_q95", "c130x250_s0_q95", "g130x250_q90"):
        img = codec.decode_jpg(jpgs[name], device_out=True)
        target = len(jpgs[name]) // 3
        r = codec.fit([img], target, 0.25)[0]
        o = oracle.fit(pxs[name], target, 0.25)
        assert r["success"] == o["success"] and r.get("data") == o["data"], name


def _jpeg(rgb, **kw):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(rgb).save(b, "JPEG", **kw)
    return b.getvalue()


@pytest.mark.parametrize("kind", ["smooth", "noise"])
def test_decode_4k_q95_matches_oracle(codec, oracle, kind):
    """BASELINE sources: 4K, q95, 4:2:0 — the noise frame has almost no EOBs,
    the hardest case for self-synchronisation."""
    img = (smooth if kind == "smooth" else noise)(2160, 3840, 5)[:, :, ::-1].copy()
    data = _jpeg(img, quality=95, subsampling=2)
    rc, ref = oracle.jpeg_decode(data)
    assert rc == 0
    got = codec.decode_jpg(data)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("sub_bits", [2048, 16384, 32768, 65536])
def test_decode_subsequence_lengths(codec, oracle, monkeypatch, sub_bits):
    """The subsequence length follows the batch size (pick_sub_bits: 65536
    bits on configs[1]'s 1000-frame calls, 32768 at 200, 2048 for a lone
    small file); every length, forced on one small mixed batch (ICX_DEC_SUB_BITS),
    must decode what the oracle decodes - checkpoints, write-pass pieces and
    relaxation at that length."""
    datas = [_jpeg((smooth if i % 2 == 0 else noise)(h, w, 70 + i)[:, :, ::-1].copy(), quality=95, subsampling=2)
             for i, (h, w) in enumerate([(2160, 3840), (2160, 3840), (1080, 1920), (333, 517)])]
    monkeypatch.setenv("ICX_DEC_SUB_BITS", str(sub_bits))
    res = codec.decode_jpg_batch(datas, subsampling=1)
    for i, (data, (st, img)) in enumerate(zip(datas, res)):
        rc, ref = oracle.jpeg_decode(data)
        assert rc == 0 and st == N.OK, (i, st)
        assert np.array_equal(img, ref), (sub_bits, i)


def test_decode_batch_settling_at_different_launches(codec, oracle, dgolden):
    """One batch whose images settle their entry states at different sync
    launches (smooth frames early, uniform noise late, small files at once):
    the settled ones finish on the aux stream while the rest keep relaxing
    (icx_decode.cpp); every image must still equal the oracle."""
    meta, jpgs, _ = dgolden
    datas = [_jpeg((smooth if i % 2 == 0 else noise)(h, w, 40 + i)[:, :, ::-1].copy(), quality=95, subsampling=2)
             for i, (h, w) in enumerate([(2160, 3840), (2160, 3840), (1080, 1920), (1080, 1920), (720, 1280)])]
    datas += [jpgs["c130x250_s2_q95"], jpgs["rst7_130x250_444"]]
    res = codec.decode_jpg_batch(datas, subsampling=1)
    for i, (data, (st, img)) in enumerate(zip(datas, res)):
        rc, ref = oracle.jpeg_decode(data)
        assert rc == 0 and st == N.OK, (i, st)
        assert np.array_equal(img, ref), i


def test_decode_8k_reference_subsampling_rule(codec, oracle):
    """decodeImageWithSubsampling's rule (ImageCompression.java:140-153):
    s = 2 for an 8192-wide image, 1 below."""
    img = smooth(520, 8200, 9)[:, :, ::-1].copy()
    data = _jpeg(img, quality=80, subsampling=2)
    got = codec.decode_jpg(data)  # subsampling 0 = the reference's rule
    rc, ref = oracle.jpeg_decode(data, 2)
    assert rc == 0 and got.shape == (260, 4100, 3) and np.array_equal(got, ref)


def test_decode_of_own_encodes_round_trip(codec, oracle):
    """decode(encode(img)) on the GPU: coefficients equal the oracle decode of
    the same bytes, for smooth/noise at low and full quality, colour and grey."""
    for img, q in [(smooth(136, 200, 3), 0.25), (noise(64, 96, 4), 1.0), (smooth(50, 70, 5)[:, :, 0].copy(), 0.5)]:
        data = codec.compress_jpg_to_stream(img, q)
        assert np.array_equal(codec.debug_decode_coefs(data), oracle.jpeg_coefs(data))
        rc, ref = oracle.jpeg_decode(data)
        assert rc == 0 and np.array_equal(codec.decode_jpg(data), ref)


def test_decode_refusals_and_corrupt_input(codec, oracle, dgolden):
    """Headers the JDK reader cannot read are corrupt; a scan cut short
    decodes as that reader decodes it (IJG 6b's recovery: the oracle's
    pixels); neither spoils the batch."""
    meta, jpgs, _ = dgolden
    good = jpgs["c130x250_s2_q95"]
    cut = [good[: len(good) // 2], good[: len(good) - 3]]
    bad = [b"\xff\xd8\xff\xd9", good[:2] + b"\x00" * 100, good[:300]]
    res = codec.decode_jpg_batch(cut + bad + [good], subsampling=1)
    for d, (st, img) in zip(cut, res):
        rc, ref = oracle.jpeg_decode(d)
        assert st == N.OK and rc == 0 and np.array_equal(img, ref)
    for st, img in res[len(cut):-1]:
        assert st in (N.E_CORRUPT, N.E_UNSUPPORTED), st
    assert res[-1][0] == N.OK  # a bad file does not spoil the batch


def test_decode_fuzzed_batch(codec, oracle, dgolden):
    """400 corrupted files in one device batch (flipped entropy bytes,
    truncation, stray RSTn/EOI/fill markers, corrupted headers): every file
    ends with OK, UNSUPPORTED or CORRUPT, a bad file never spoils its
    neighbours, and whatever the device accepts decodes exactly as the oracle
    does."""
    meta, jpgs, pxs = dgolden
    rng = np.random.default_rng(99)
    names = [k for k in jpgs if not meta["cases"][k].get("unsupported")]
    datas = []
    for i in range(400):
        d = bytearray(jpgs[names[i % len(names)]])
        mode = i % 5
        if mode == 0:
            for _ in range(int(rng.integers(1, 8))):
                p = int(rng.integers(len(d) // 2, len(d)))
                d[p] = int(rng.integers(0, 256))
        elif mode == 1:
            d = d[: int(rng.integers(4, len(d)))]
        elif mode == 2:
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(len(d) // 2, len(d)))
                d[p:p] = bytes([0xFF, int(rng.choice([0xD0, 0xD3, 0xD9, 0xFF, 0xC4]))])
        elif mode == 3:
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(2, min(len(d), 700)))
                d[p] = int(rng.integers(0, 256))
        datas.append(bytes(d))  # mode 4: intact
    res = codec.decode_jpg_batch(datas, subsampling=1)
    ok = 0
    for i, (d, (st, img)) in enumerate(zip(datas, res)):
        assert st in (N.OK, N.E_UNSUPPORTED, N.E_CORRUPT, N.E_REFUSED), (i, st)
        if i % 5 == 4:
            assert st == N.OK and np.array_equal(img, pxs[names[i % len(names)]]), i
        if st == N.OK:
            rc, ref = oracle.jpeg_decode(d)
            assert rc == 0 and np.array_equal(img, ref), i
            ok += 1
    assert ok >= 240  # damaged entropy data decodes (6b recovery); header damage may not


def _with_comments(data, sizes):
    """data with COM segments of the given payload sizes inserted after SOI."""
    segs = b"".join(b"\xff\xfe" + (n + 2).to_bytes(2, "big") + bytes((i * 7) & 0x7F for i in range(n))
                    for n in sizes)
    return data[:2] + segs + data[2:]


def test_decode_device_inputs_unaligned_and_long_headers(codec, dgolden):
    """Device-resident files at every address alignment, and headers longer
    than the first 4 KiB header fetch (re-fetched at 32 KiB, then 256 KiB),
    in one batch: the k_stage header gather, and k_unstuff_* reading each
    file's scan where it lies at any byte alignment (no staging copy)."""
    import torch
    meta, jpgs, pxs = dgolden
    names = ["c130x250_s2_q95", "c66x130_s1_q50", "g47x61_q90", "rst7_130x250_444", "c7x9_s2_q95"]
    datas, want = [], []
    for k, name in enumerate(names):
        for extra in ([], [5000], [60000, 60000, 3000]):
            data = _with_comments(jpgs[name], extra)
            off = (k + len(extra)) % 4 + 4 * (len(extra) == 1)
            buf = torch.zeros(len(data) + off + 3, dtype=torch.uint8)
            buf[off:off + len(data)] = torch.from_numpy(np.frombuffer(data, np.uint8).copy())
            datas.append(buf.cuda()[off:off + len(data)])
            want.append(pxs[name])
    res = codec.decode_jpg_batch(datas, subsampling=1)
    for i, (st, img) in enumerate(res):
        assert st == N.OK, (i, st)
        assert np.array_equal(img, want[i]), i
    # the same files from pageable host memory (one DMA of each scan, 256-B aligned)
    res = codec.decode_jpg_batch([d.cpu().numpy().tobytes() for d in datas], subsampling=1)
    for i, (st, img) in enumerate(res):
        assert st == N.OK and np.array_equal(img, want[i]), i


def _sos_offsets(data):
    return [i for i in range(len(data) - 1) if data[i] == 0xFF and data[i + 1] == 0xDA]


def test_progressive_golden_subsampled_device_io(codec, dgolden):
    """Progressive golden files (libjpeg-turbo pixels) at s = 1, 2, 3, with
    host, libicx and CUDA-tensor inputs and device outputs: the device IDCT /
    colour passes over the host entropy decode."""
    import torch

    import icx
    meta, jpgs, pxs = dgolden
    names = [k for k in jpgs if meta["cases"][k].get("progressive")]
    for s in (1, 2, 3):
        for name in names:
            want = pxs[name][::s, ::s]
            img = codec.decode_jpg(jpgs[name], subsampling=s, device_out=True)
            assert isinstance(img, icx.DeviceImage) and np.array_equal(img.numpy(), want), (name, s)
            dev_in = icx.DeviceImage.from_host(codec, jpgs[name])
            assert np.array_equal(codec.decode_jpg(dev_in, subsampling=s), want), (name, s)
            t_in = torch.from_numpy(np.frombuffer(jpgs[name], np.uint8).copy()).cuda()
            assert np.array_equal(codec.decode_jpg(t_in, subsampling=s), want), (name, s)


@pytest.mark.parametrize("shape,sub", [((2160, 3840), 2), ((1080, 1920), 1), ((1081, 1917), 0), ((999, 1001), 2)])
def test_progressive_equals_baseline_twin_decode(codec, oracle, shape, sub):
    """A progressive file decodes to exactly the oracle's decode of its
    baseline twin (same pixels, same tables: same coefficients), at BASELINE
    sizes, in a batch mixed with baseline files."""
    from PIL import Image
    img = smooth(*shape, 21)
    pil = Image.fromarray(np.ascontiguousarray(img[:, :, ::-1]))
    a, b = io.BytesIO(), io.BytesIO()
    pil.save(a, "JPEG", quality=95, subsampling=sub)
    pil.save(b, "JPEG", quality=95, subsampling=sub, progressive=True)
    base, prog = a.getvalue(), b.getvalue()
    rc, ref = oracle.jpeg_decode(base)
    assert rc == 0
    res = codec.decode_jpg_batch([prog, base, prog], subsampling=1)
    for st, got in res:
        assert st == N.OK and np.array_equal(got, ref)
    assert np.array_equal(codec.debug_decode_coefs(prog), oracle.jpeg_coefs(base))


def test_progressive_refusals_in_a_batch(codec, dgolden):
    """A truncated scan script (the JDK would block-smooth it) is unsupported,
    a scan cut short is corrupt; neither spoils its batch neighbours."""
    meta, jpgs, pxs = dgolden
    good = jpgs["prog_c130x250_s2_q95"]
    sos = _sos_offsets(good)
    bad = [good[:sos[5]] + b"\xff\xd9", good[:sos[3] + 50]]
    res = codec.decode_jpg_batch(bad + [good, jpgs["c130x250_s2_q95"]], subsampling=1)
    assert res[0][0] == N.E_UNSUPPORTED and res[1][0] == N.E_CORRUPT
    assert res[2][0] == N.OK and np.array_equal(res[2][1], pxs["prog_c130x250_s2_q95"])
    assert res[3][0] == N.OK and np.array_equal(res[3][1], pxs["c130x250_s2_q95"])


def test_decode_stray_restart_markers(codec, oracle, dgolden):
    """RSTn markers where the DRI interval does not end (inserted, or one
    removed): the device walk flags the file (every interval must end after
    ri MCUs, DecWalker::invalid) and libjpeg's resynchronisation decodes it
    (icx_seqdecode.cpp) exactly as the oracle does."""
    meta, jpgs, pxs = dgolden
    good = jpgs["rst7_130x250"]
    sos = good.index(b"\xff\xda")
    body = sos + 2 + int.from_bytes(good[sos + 2:sos + 4], "big")
    rsts = [i for i in range(body, len(good) - 1) if good[i] == 0xFF and 0xD0 <= good[i + 1] <= 0xD7]
    datas = []
    for k in range(12):
        p = body + (len(good) - body) * (k + 1) // 14
        datas.append(good[:p] + bytes([0xFF, 0xD0 + k % 8]) + good[p:])
    for r in rsts[::5]:
        datas.append(good[:r] + good[r + 2:])  # one marker removed
    res = codec.decode_jpg_batch(datas + [good], subsampling=1)
    for i, (d, (st, img)) in enumerate(zip(datas, res)):
        rc, ref = oracle.jpeg_decode(d)
        assert st == N.OK and rc == 0 and np.array_equal(img, ref), (i, st)
    assert res[-1][0] == N.OK and np.array_equal(res[-1][1], pxs["rst7_130x250"])
