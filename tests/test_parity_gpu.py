"""Parity of the HIP path (libicx.so through the C ABI) with the oracle and
the golden vectors.  Bit-exact everywhere: coefficients, bitstreams, sizes,
search traces, chosen (quality, scale), resized pixels."""
import numpy as np
import pytest

import icx
from icx import _native as N
from tests.oracle_ffi import jdk_bytes, noise, smooth

pytestmark = pytest.mark.gpu


def test_fdct_coefficients_bit_exact(codec, oracle, golden):
    _, inputs, _ = golden
    for name, img in inputs.items():
        assert np.array_equal(codec.debug_fdct(img), oracle.fdct(img)), name
    rng = np.random.default_rng(7)
    for h, w in [(1, 1), (16, 16), (17, 33), (31, 129), (129, 255), (1080, 1920), (67, 1001), (256, 130)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        assert np.array_equal(codec.debug_fdct(img), oracle.fdct(img)), (h, w)
        g = img[:, :, 1].copy()
        assert np.array_equal(codec.debug_fdct(g), oracle.fdct(g)), ("grey", h, w)


def test_encode_matches_golden_bytes(codec, golden):
    meta, inputs, jpegs = golden
    n = 0
    for name, img in inputs.items():
        for q in meta["images"][name]["encodes"]:
            ref = jdk_bytes(jpegs[f"{name}@{q}"].tobytes(), meta)
            assert codec.compress_jpg_to_stream(img, float(q)) == ref, (name, q)
            n += 1
    assert n == 121


@pytest.mark.parametrize("kind", ["smooth", "noise"])
def test_encode_4k_matches_oracle(codec, oracle, kind):
    img = (smooth if kind == "smooth" else noise)(2160, 3840, 11)
    for q in (0.25, 0.125, 0.0625, 0.9, 1.0):  # 0.9/1.0 noise: most blocks outgrow the LDS slot
        assert codec.compress_jpg_to_stream(img, q) == oracle.encode(img, q), q


def test_encode_odd_sizes_match_oracle(codec, oracle):
    rng = np.random.default_rng(3)
    for _ in range(12):
        h, w = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        img = smooth(h, w, int(rng.integers(1 << 30))) if rng.random() < 0.5 else noise(h, w, 5)
        q = float(rng.uniform(0.005, 1.0))
        assert codec.compress_jpg_to_stream(img, q) == oracle.encode(img, q), (h, w, q)
        g = img[:, :, 0].copy()
        assert codec.compress_jpg_to_stream(g, q) == oracle.encode(g, q), ("grey", h, w, q)


def test_rgb_input_equals_bgr_input(codec):
    img = smooth(64, 96, 4)
    rgb = np.ascontiguousarray(img[:, :, ::-1])
    a = codec.compress_jpg_to_stream(img, 0.3)
    jobs_img = icx.core._image_struct(rgb, N.RGB24)[0]
    import ctypes
    out = np.empty(1 << 20, np.uint8)
    n = ctypes.c_size_t()
    st = N.load().icx_compress_jpg_to_stream(codec._ctx, ctypes.byref(jobs_img), 0.3, out.ctypes.data, out.size,
                                             ctypes.byref(n))
    assert st == N.OK and out[:n.value].tobytes() == a


def test_search_traces_match_golden(codec, golden):
    meta, inputs, _ = golden
    for name, img in inputs.items():
        for s in meta["images"][name]["searches"]:
            trace = []
            best = codec.find_best_quality_by_binary_search(img, s["target"], s["q0"], trace)
            assert [(np.float32(q), sz) for q, sz, _ in trace] == \
                   [(np.float32(q), sz) for q, sz, _ in s["trace"]], (name, s["target"], s["q0"])
            assert np.float32(best) == np.float32(s["best"])


def test_fit_matches_oracle_including_scale_loop_and_cache(codec, oracle, golden):
    _, inputs, _ = golden
    cases = []
    for name in ("noise_120x90", "smooth_200x136", "noise_1001x67", "grey_37x29", "smooth_64x48"):
        img = inputs[name]
        lo = len(oracle.encode(img, 0.015625))
        for target in (lo - 1, lo, lo * 2, 10 ** 7, 700, 200):
            cases.append((name, img, target))
    for name, img, target in cases:
        o = oracle.fit(img, target, 0.25)
        r = codec.fit([img], target, 0.25)[0]
        assert r["status"] == N.OK
        assert r["success"] == o["success"], (name, target)
        if o["success"]:
            assert r["data"] == o["data"], (name, target)
            assert np.float32(r["learned"].quality) == np.float32(o["quality"])
            assert r["learned"].scale == o["scale"]
            # the cached-params path reproduces the same file with one encode
            oc = oracle.fit(img, target, 0.25, cached=(o["quality"], o["scale"]))
            rc = codec.fit([img], target, 0.25, cached=[icx.LearnedParams(o["quality"], o["scale"])])[0]
            assert rc["cache_hit"] and oc["cache_hit"] and rc["data"] == oc["data"] == o["data"]
            assert rc["encodes"] == 1
        # a stale cache entry (quality too high) falls back to the full search
        rs = codec.fit([img], target, 0.25, cached=[icx.LearnedParams(1.0, 1.0)])[0]
        os_ = oracle.fit(img, target, 0.25, cached=(1.0, 1.0))
        assert rs["success"] == os_["success"] and rs["cache_hit"] == os_["cache_hit"]
        if os_["success"]:
            assert rs["data"] == os_["data"]


def test_batch_mixed_sizes_matches_oracle(codec, oracle):
    rng = np.random.default_rng(9)
    imgs = []
    for i in range(10):
        h, w = int(rng.integers(8, 400)), int(rng.integers(8, 400))
        imgs.append(smooth(h, w, i) if i % 2 else noise(h, w, i))
    for target in (3000, 20000):
        res = codec.fit(imgs, target, 0.25)
        for img, r in zip(imgs, res):
            o = oracle.fit(img, target, 0.25)
            assert r["success"] == o["success"]
            if o["success"]:
                assert r["data"] == o["data"] and r["learned"].scale == o["scale"]


def test_grouped_table_layout_matches_oracle(codec, oracle):
    """ICX_TABLES_GROUPED (one DQT, one DHT segment: 607 / 324-B headers) on
    the device equals the oracle's grouped layout byte for byte, through the
    search, the scale loop and the cached path, with sizes compared whole-file
    against -t (ImageCompressionJpg.java:176) - colour and grey."""
    rng = np.random.default_rng(41)
    imgs = []
    for i in range(8):
        h, w = int(rng.integers(8, 300)), int(rng.integers(8, 300))
        im = smooth(h, w, 500 + i) if i % 2 else noise(h, w, 500 + i)
        imgs.append(im[:, :, 1].copy() if i % 3 == 0 else im)
    imgs.append(noise(2160, 3840, 23))
    try:
        codec.set_table_layout(N.TABLES_GROUPED)
        oracle.set_table_layout(True)
        for target, cached in ((4000, None), (30000, [icx.LearnedParams(0.25, 1.0)] * len(imgs)),
                               (1 << 20, None)):
            res = codec.fit(imgs, target, 0.25, cached=cached)
            for k, (img, r) in enumerate(zip(imgs, res)):
                o = oracle.fit(img, target, 0.25, cached=(0.25, 1.0) if cached else None)
                assert r["success"] == o["success"], (k, target)
                if o["success"]:
                    assert r["data"] == o["data"], (k, target)
                    hdr = 607 if img.ndim == 3 else 324
                    assert r["data"][hdr - 14:hdr - 12] == b"\xff\xda" or r["data"][hdr - 10:hdr - 8] == b"\xff\xda"
    finally:
        codec.set_table_layout(N.TABLES_SEPARATE)
        oracle.set_table_layout(False)
    d = codec.compress_jpg_to_stream(imgs[1], 0.5)
    assert len(d) == len(oracle.encode(imgs[1], 0.5))  # back to the default layout


def test_4k_fixed_quality_cache_path(codec, oracle):
    """BASELINE config 2 semantics: cache hit (0.25, 1.0), -t 1 MiB."""
    imgs = [smooth(2160, 3840, 21), noise(2160, 3840, 22)]
    res = codec.fit(imgs, 1 << 20, 0.25, cached=[icx.LearnedParams(0.25, 1.0)] * 2)
    for img, r in zip(imgs, res):
        o = oracle.fit(img, 1 << 20, 0.25, cached=(0.25, 1.0))
        assert r["success"] == o["success"] and r["cache_hit"] == o["cache_hit"]
        assert r["data"] == o["data"]
        assert np.float32(r["learned"].quality) == np.float32(o["quality"])


def test_resize_matches_restatement(codec, oracle):
    rng = np.random.default_rng(5)
    for h, w in [(90, 120), (1, 7), (37, 29), (2160, 3840)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        s = 0.85
        while s > 0.1:
            dw, dh = oracle.scaled_dims(w, h, s)
            assert np.array_equal(codec.resize_image(img, s), oracle.resize(img, dw, dh)), (h, w, s)
            s *= 0.85
            if h * w > 10 ** 6:
                break
        g = img[:, :, 2].copy()
        dw, dh = oracle.scaled_dims(w, h, 0.5)
        assert np.array_equal(codec.resize_image(g, 0.5), oracle.resize(g, dw, dh))


@pytest.mark.parametrize("fmt", [N.XRGB32, N.ARGB32, N.ABGR32, N.RGBA32])
def test_resize_four_byte_formats_match_restatement(codec, oracle, fmt):
    """ImageTools.java:12-15 keeps the type: four-byte rasters through
    k_resize4 (premultiplied bilinear, SrcOver onto a zero image) equal the
    oracle's restatement bit for bit - transparent, opaque and partial alpha
    regions, down- and up-scaling, odd sizes, 4K."""
    rng = np.random.default_rng(fmt)
    ab = 0 if fmt == N.ABGR32 else 3
    for h, w, dw, dh in [(90, 120, 76, 51), (1, 7, 3, 1), (37, 29, 80, 61), (2160, 3840, 1920, 1080)]:
        img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
        img[: h // 3, :, ab] = 0
        img[h // 3: 2 * h // 3, :, ab] = 255
        got = codec.resize_to(img, dw, dh, fmt=fmt)
        assert np.array_equal(got, oracle.resize(img, dw, dh, fmt=fmt)), (fmt, h, w)
        if fmt == N.XRGB32:
            assert (got[:, :, 3] == 0).all()


def test_png_fit_keeps_alpha(codec, oracle, tmp_path):
    """compressPngWithTargetSize on a TYPE_4BYTE_ABGR raster: the resized PNG
    is RGBA, its pixels equal the restatement's, transparent areas stay
    transparent."""
    from PIL import Image
    rng = np.random.default_rng(4)
    abgr = rng.integers(0, 256, (600, 800, 4), dtype=np.uint8)
    abgr[:200, :, 0] = 0
    out = tmp_path / "alpha.png"
    assert codec.compress_png_with_target_size(abgr, out, icx.CompressionParams(0, 0, 100, 100, 0)) is True
    im = Image.open(out)
    assert im.mode == "RGBA" and im.size == (100, 75)
    assert np.array_equal(np.asarray(im)[:, :, ::-1], oracle.resize(abgr, 100, 75))
    assert (np.asarray(im)[:20, :, 3] == 0).all()


def test_resize_tiles_staged_and_direct_match_restatement(codec, oracle):
    """k_resize stages each 64 x 16 tile's source rectangle in LDS when it
    fits (scales down to ~0.2) and reads the taps from global memory below
    that: both paths, tile edges (widths and heights that are not multiples
    of the tile), unaligned rows (odd widths, a row stride that is not a
    multiple of 16) and upscaling equal the restatement for every pixel
    class."""
    rng = np.random.default_rng(11)
    cases = [(2160, 3840, 1920, 1080), (1081, 1921, 999, 563), (77, 131, 13, 7), (77, 131, 211, 150),
             (500, 700, 60, 40), (3, 5, 64, 17), (1, 1, 3, 2)]
    for h, w, dw, dh in cases:
        for nch in (1, 3):
            img = rng.integers(0, 256, (h, w, nch) if nch > 1 else (h, w), dtype=np.uint8)
            got = codec.resize_to(img, dw, dh)
            assert np.array_equal(got, oracle.resize(img, dw, dh)), (h, w, dw, dh, nch)
        # a padded row stride (not a multiple of 16): a view of a wider array
        wide = rng.integers(0, 256, (h, w + 3, 3), dtype=np.uint8)
        view = wide[:, :w]
        assert np.array_equal(codec.resize_to(view, dw, dh), oracle.resize(np.ascontiguousarray(view), dw, dh))


def test_resize_16bit_grey_matches_restatement(codec, oracle):
    """TYPE_USHORT_GRAY (a 16-bit grey PNG; ImageTools.java:12-15 keeps the
    type): Java2D's UshortGray loops interpolate the high byte in 8 bits and
    store 257 * v - k_resize<2> equals the oracle's restatement bit for bit,
    and the result is a uint16 raster of 257 multiples."""
    rng = np.random.default_rng(16)
    for h, w, s in [(2160, 3840, 0.5), (301, 517, 0.85), (40, 30, 0.3)]:
        img = rng.integers(0, 65536, (h, w), dtype=np.uint16)
        got = codec.resize_image(img, s)
        dw, dh = oracle.scaled_dims(w, h, s)
        assert got.dtype == np.uint16 and got.shape == (dh, dw)
        assert np.array_equal(got, oracle.resize(img, dw, dh)), (h, w, s)
        assert (got % 257 == 0).all()


def test_png_fit_batch_matches_restatement(codec, oracle):
    """icx_png_fit_batch: one launch per pixel format for a mixed group -
    sizes (same-size groups take the 2-D grid, mixed ones the slot search),
    formats, images that already fit the box (None, nothing written) - each
    result equals the one-image fit and the oracle."""
    rng = np.random.default_rng(21)
    p = icx.CompressionParams(0.25, 0, 1920, 1920, 0)
    imgs = [rng.integers(0, 256, (2160, 3840, 3), dtype=np.uint8) for _ in range(3)]
    imgs += [rng.integers(0, 256, (1500, 2500), dtype=np.uint8), rng.integers(0, 256, (2001, 1999, 4), dtype=np.uint8),
             rng.integers(0, 65536, (2400, 3000), dtype=np.uint16), rng.integers(0, 256, (800, 600, 3), dtype=np.uint8),
             rng.integers(0, 256, (1080, 4096, 3), dtype=np.uint8)]
    codec.profile(True)
    codec.profile_reset()
    res = codec.png_fit_batch(imgs, p)
    st = codec.profile_query("resize")
    codec.profile(False)
    assert st["launches"] == 4  # BGR, grey, ABGR, grey16: one launch each
    for img, r in zip(imgs, res):
        h, w = img.shape[:2]
        if w <= 1920 and h <= 1920:
            assert r is None
            continue
        dw, dh = oracle.scaled_dims(w, h, min(1920 / w, 1920 / h))
        assert r.shape[:2] == (dh, dw) and r.dtype == img.dtype
        assert np.array_equal(r, oracle.resize(img, dw, dh)), img.shape


def test_png_16bit_grey_through_the_pipeline(codec, oracle, tmp_path):
    """A 16-bit grey PNG keeps its type (ImageTools.java:12-15): read as
    TYPE_USHORT_GRAY, resized on the device and written as a 16-bit grey PNG
    whose samples equal the restatement (not clipped to 8 bits)."""
    from PIL import Image

    from icx.pipeline import process_image
    rng = np.random.default_rng(3)
    src = (rng.integers(0, 256, (300, 400), dtype=np.uint16) * 257 + rng.integers(0, 257, (300, 400))).astype(np.uint16)
    Image.fromarray(src).save(tmp_path / "g16.png")  # uint16 (H, W): mode I;16, a 16-bit grey PNG
    out = tmp_path / "out"
    out.mkdir()
    rep = process_image(tmp_path / "g16.png", out, icx.CompressionParams(0.25, 10, 100, 100, 10 ** 6), {}, codec)
    assert rep.result == icx.CompressionResult.COMPRESSED_SUCCESS
    im = Image.open(out / "g16.png")
    assert im.mode.startswith("I") and im.size == (100, 75)
    got = np.asarray(im).astype(np.uint16)
    assert np.array_equal(got, oracle.resize(src, 100, 75))
    raw = open(out / "g16.png", "rb").read()
    assert raw[24] == 16 and raw[25] == 0  # IHDR bit depth 16, colour type 0


def test_jpeg_rejects_alpha_rasters(codec):
    """The JDK JPEG writer refuses alpha rasters: the JPEG entry points return
    ICX_E_UNSUPPORTED for four-byte formats."""
    img = np.zeros((16, 16, 4), np.uint8)
    r = codec.fit([img], 10 ** 6, 0.25)[0]
    assert r["status"] == N.E_UNSUPPORTED and not r["success"]


def test_png_fit(codec, tmp_path):
    """ImageCompressionPngTest.java:38-88 restated."""
    small = np.zeros((100, 100, 3), np.uint8)
    small[:] = (0, 0, 255)
    p = icx.CompressionParams(0, 0, 100, 100, 0)
    assert codec.compress_png_with_target_size(small, tmp_path / "small.png", p) is False
    big = np.zeros((600, 800, 3), np.uint8)
    big[:] = (255, 0, 0)
    out = tmp_path / "resized.png"
    assert codec.compress_png_with_target_size(big, out, p) is True
    from PIL import Image
    im = Image.open(out)
    assert im.size == (100, 75)
    assert np.all(np.asarray(im)[:, :, 2] == 255)
    with pytest.raises(TypeError):
        codec.compress_png_with_target_size(None, out, p)
    with pytest.raises(TypeError):
        codec.compress_png_with_target_size(big, None, p)
    with pytest.raises(TypeError):
        codec.compress_png_with_target_size(big, out, None)


def test_device_resident_inputs_and_outputs(codec, oracle):
    torch = pytest.importorskip("torch")
    img = smooth(1080, 1920, 31)
    t = torch.from_numpy(img).cuda()
    out = torch.zeros(1 << 21, dtype=torch.uint8, device="cuda")
    r = codec.fit([t], 300000, 0.25, outputs=[out])[0]
    o = oracle.fit(img, 300000, 0.25)
    assert r["success"] == o["success"]
    assert out[:r["out_len"]].cpu().numpy().tobytes() == o["data"]


def test_output_buffer_too_small(codec):
    img = noise(64, 64, 1)
    import ctypes
    st_img = icx.core._image_struct(img)[0]
    out = np.empty(100, np.uint8)
    n = ctypes.c_size_t()
    st = N.load().icx_compress_jpg_to_stream(codec._ctx, ctypes.byref(st_img), 0.9, out.ctypes.data, out.size,
                                             ctypes.byref(n))
    assert st == N.E_BUFFER and n.value > 100


def test_invalid_inputs(codec):
    import ctypes
    lib = N.load()
    bad = N.Image(None, 10, 10, 30, N.BGR24)
    n = ctypes.c_size_t()
    buf = np.empty(10, np.uint8)
    assert lib.icx_compress_jpg_to_stream(codec._ctx, ctypes.byref(bad), 0.5, buf.ctypes.data, 10,
                                          ctypes.byref(n)) == N.E_NULL
    img = np.zeros((4, 4, 3), np.uint8)
    bad = N.Image(img.ctypes.data, 0, 4, 12, N.BGR24)
    assert lib.icx_compress_jpg_to_stream(codec._ctx, ctypes.byref(bad), 0.5, buf.ctypes.data, 10,
                                          ctypes.byref(n)) == N.E_INVALID


def test_candidate_lists_mixed_batch(codec, oracle):
    """One batch whose images reach different quality sets (different cached
    probes, stale and fresh, none; colour and grey; partial FDCT tiles), so
    every image gets its own candidate filter: results equal the oracle's."""
    rng = np.random.default_rng(17)
    cached_choices = [None, (0.9, 1.0), (0.05, 1.0), (1.0, 1.0), (0.3, 0.85), (0.2, 1.0)]
    imgs, cached = [], []
    for i in range(12):
        h, w = int(rng.integers(9, 360)), int(rng.integers(9, 420))
        img = smooth(h, w, 100 + i) if i % 3 else noise(h, w, 200 + i)
        if i % 4 == 3:
            img = img[:, :, 1].copy()
        imgs.append(img)
        cached.append(cached_choices[i % len(cached_choices)])
    for target, q0 in ((6000, 0.25), (25000, 0.8)):
        res = codec.fit(imgs, target, q0,
                        cached=[icx.LearnedParams(*c) if c else None for c in cached])
        for i, (img, r) in enumerate(zip(imgs, res)):
            o = oracle.fit(img, target, q0, cached=cached[i])
            assert r["status"] == N.OK
            assert (r["success"], r["cache_hit"]) == (o["success"], o["cache_hit"]), (i, target)
            if o["success"]:
                assert r["data"] == o["data"], (i, target)
                assert np.float32(r["learned"].quality) == np.float32(o["quality"])
                assert r["learned"].scale == o["scale"]


def test_same_size_batch_matches_oracle(codec, oracle):
    """Same-sized frames: the launches take the 2-D grid (image = y, no slot
    search) in every stage - the probe over all images (identity plan) and
    the search over the misses (a subset, with its id table) - and partial
    FDCT tiles (width 600 = 2 tiles + 88 px)."""
    colour = [smooth(136, 600, 300 + i) if i % 2 else noise(136, 600, 400 + i) for i in range(6)]
    grey = [im[:, :, 1].copy() for im in colour]  # grey FDCT: 2-D launch too
    cached = [icx.LearnedParams(0.25, 1.0)] * len(colour)
    for imgs, target in ((colour, 12000), (colour, 40000), (grey, 8000)):
        res = codec.fit(imgs, target, 0.25, cached=cached)
        for i, (img, r) in enumerate(zip(imgs, res)):
            o = oracle.fit(img, target, 0.25, cached=(0.25, 1.0))
            assert r["status"] == N.OK
            assert (r["success"], r["cache_hit"]) == (o["success"], o["cache_hit"]), (i, target)
            if o["success"]:
                assert r["data"] == o["data"], (i, target)
                assert np.float32(r["learned"].quality) == np.float32(o["quality"])
                assert r["learned"].scale == o["scale"]


def test_host_buffers_pipelined_over_subbatches(oracle, monkeypatch):
    """Host inputs and outputs (pageable numpy and pinned torch) through the
    pipelined host I/O of run_batch: a small workspace budget forces several
    sub-batches, so uploads of sub-batch s+1 and downloads of s-1 overlap the
    kernels of s on their own streams.  Every file equals the oracle's."""
    import torch
    monkeypatch.setenv("ICX_WORKSPACE_MB", "24")
    c = icx.Codec(0)
    try:
        imgs, targets = [], []
        for i in range(9):
            h, w = 360 + 24 * i, 520 + 40 * i
            im = (smooth if i % 2 else noise)(h, w, 40 + i)
            imgs.append(torch.from_numpy(im).pin_memory() if i % 3 == 0 else im)
            targets.append(h * w // 5)
        c.profile(True)
        c.profile_reset()
        for target in (min(targets), max(targets)):
            res = c.fit(imgs, target, 0.25)
            for i, r in enumerate(res):
                im = imgs[i].numpy() if hasattr(imgs[i], "numpy") else imgs[i]
                o = oracle.fit(im, target, 0.25)
                assert r["status"] == 0 and r["success"] == o["success"], (i, target)
                if o["success"]:
                    assert r["data"] == o["data"], (i, target)
                    assert np.float32(r["learned"].quality) == np.float32(o["quality"])
                    assert r["learned"].scale == o["scale"]
        assert c.profile_query("subbatch")["launches"] >= 6  # >= 3 sub-batches per call
        # device inputs, host outputs (the pipeline's decoded frames -> files):
        # nothing is uploaded, so the kernels of sub-batch s must still wait
        # for s-2's downloads out of the same staging arena
        dimgs = [torch.from_numpy(im.numpy() if hasattr(im, "numpy") else im).to("cuda:0") for im in imgs]
        c.profile_reset()
        for target in (min(targets), max(targets)):
            res = c.fit(dimgs, target, 0.25)
            for i, r in enumerate(res):
                o = oracle.fit(dimgs[i].cpu().numpy(), target, 0.25)
                assert r["status"] == 0 and r["success"] == o["success"], (i, target)
                if o["success"]:
                    assert r["data"] == o["data"], ("device in / host out", i, target)
        assert c.profile_query("subbatch")["launches"] >= 6
    finally:
        c.close()


def test_bench_headline_frames_match_oracle(codec, oracle):
    """The headline workload itself (bench.py: frames from make_frames, -t 1 MiB,
    cached LearnedParams(0.25, 1.0), outputs in HBM, one prepared batch run
    twice as in the timed loop): every frame's file, quality and encode count
    equal the oracle's compressJpgWithTargetSize on the same pixels."""
    import torch

    import bench
    dev = torch.device("cuda", 0)
    n = 4  # two smooth (cache hit at q = 0.25), two noise (search)
    frames = bench.make_frames(n, 1000003 * 3, dev)
    outs = torch.empty((n, bench.TARGET + 1), dtype=torch.uint8, device=dev)
    batch = codec.prepare(frames, bench.TARGET, bench.Q0, cached=[icx.LearnedParams(bench.Q0, 1.0)] * n,
                          outputs=[outs[i] for i in range(n)])
    for _ in range(2):
        batch.run()
    torch.cuda.synchronize()
    res = batch.results()
    for i in range(n):
        img = frames[i].cpu().numpy()
        ref = oracle.fit(img, bench.TARGET, bench.Q0, cached=(bench.Q0, 1.0))
        r = res[i]
        assert r["success"] and ref["success"], i
        assert outs[i, :r["out_len"]].cpu().numpy().tobytes() == ref["data"], i
        assert np.float32(r["learned"].quality) == np.float32(ref["quality"]), i
        # the oracle counts saveCompressedImage's re-encode after a search
        # (ImageCompressionJpg.java:255-260); the device stuffs the best trial instead
        trials = ref["encodes"] - (0 if ref["cache_hit"] else 1)
        assert r["learned"].scale == ref["scale"] and r["encodes"] == trials, (i, r["encodes"], ref["encodes"])
        assert r["cache_hit"] == ref["cache_hit"], i
    assert [r["cache_hit"] for r in res] == [True, False, True, False]


def test_pool_splits_batches_across_contexts(codec, oracle):
    """icx_pool over two contexts of the box's GPU (the shape of a JVM host
    driving every GPU of a node): fit, PNG fit and decode batches come back
    in the caller's order, equal to one context's results and the oracle's;
    a job with a device pointer is refused alone."""
    import torch

    pool = icx.Pool([0, 0])
    try:
        imgs = [smooth(136 + 8 * i, 200 + 16 * i, 60 + i) if i % 2 else noise(96, 120 + 8 * i, 60 + i)
                for i in range(9)]
        target = 20000
        got = pool.fit(imgs, target, 0.25)
        ref = codec.fit(imgs, target, 0.25)
        for i, (g, r) in enumerate(zip(got, ref)):
            o = oracle.fit(imgs[i], target, 0.25)
            assert g["success"] == r["success"] == o["success"], i
            assert g.get("data") == r.get("data") == o["data"], i
        big = [smooth(1080, 1920, 70 + i)[:, :, ::-1].copy() for i in range(3)]
        params = icx.CompressionParams(0.25, 1 << 20, 960, 960, 1 << 20)
        pf = pool.png_fit_batch(big + [imgs[0]], params)
        cf = codec.png_fit_batch(big + [imgs[0]], params)
        assert pf[3] is None and cf[3] is None
        for a, b in zip(pf[:3], cf[:3]):
            assert np.array_equal(a, b)
        jpgs = [oracle.encode(im, 0.9) for im in imgs]
        dec = pool.decode_jpg_batch(jpgs, subsampling=1)
        for d, (st, img) in zip(jpgs, dec):
            rc, want = oracle.jpeg_decode(d)
            assert st == N.OK and rc == 0 and np.array_equal(img, want)
        # a device-resident job is not for the pool: ICX_E_INVALID for it alone
        lib = N.load()
        dev = torch.from_numpy(np.frombuffer(jpgs[0], np.uint8).copy()).cuda()
        jobs = (N.DecodeJob * 2)()
        outs = [np.empty((136, 200, 3), np.uint8) for _ in range(2)]
        a = np.frombuffer(jpgs[1], np.uint8)
        jobs[0].data, jobs[0].len = dev.data_ptr(), dev.numel()
        jobs[1].data, jobs[1].len = a.ctypes.data, a.nbytes
        for k in range(2):
            jobs[k].subsampling = 1
            jobs[k].out, jobs[k].cap = outs[k].ctypes.data, outs[k].nbytes
        outs[1] = np.empty((imgs[1].shape[0], imgs[1].shape[1], 3), np.uint8)
        jobs[1].out, jobs[1].cap = outs[1].ctypes.data, outs[1].nbytes
        assert lib.icx_pool_decode_jpg_batch(pool._pool, jobs, 2) == N.OK
        assert jobs[0].status == N.E_INVALID and jobs[1].status == N.OK
        assert np.array_equal(outs[1], oracle.jpeg_decode(jpgs[1])[1])
        assert lib.icx_pool_size(pool._pool) == 2
    finally:
        pool.close()


def test_palette_resize_matches_restatement(codec, oracle):
    """TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY rasters (palette PNGs, 1/2/4-bit
    PNGs) through k_resize: the source's colour map to IntArgbPre, bilinear,
    SrcOver onto the new image's black, then the default map's inverse cube
    (dithered for ByteIndexed) - bit-exact against the oracle's restatement,
    single images and a batched group mixed with other formats, staged and
    direct tiles.  Parity unpinned vs Java2D (no JDK here; ImageTools.java:12-17)."""
    from icx.core import IndexedImage
    rng = np.random.default_rng(77)
    pal8 = (rng.integers(0, 1 << 24, 256) | (rng.integers(0, 256, 256) << 24)).astype(np.uint32)
    pal8[:200] |= 0xff000000  # mostly opaque, some translucent / transparent entries
    cases = []
    for (h, w) in ((300, 517), (96, 64), (1080, 1920), (37, 1501)):
        cases.append(IndexedImage(rng.integers(0, 256, (h, w)).astype(np.uint8), pal8, N.INDEXED8))
        smooth_idx = (np.add.outer(np.arange(h) // 7, np.arange(w) // 5) % 216).astype(np.uint8)
        cases.append(IndexedImage(smooth_idx, icx.default_palette(False), N.INDEXED8))
        n = 16
        pal4 = (0xff000000 | rng.integers(0, 1 << 24, n)).astype(np.uint32)
        cases.append(IndexedImage(rng.integers(0, n, (h, w)).astype(np.uint8), pal4, N.BINARY1))
        cases.append(IndexedImage(rng.integers(0, 2, (h, w)).astype(np.uint8), icx.default_palette(True),
                                  N.BINARY1))
    for im in cases:
        for scale in (0.5, 0.37, 0.13):
            got = codec.resize_image(im, scale)
            dw, dh = got.shape[1], got.shape[0]
            want = oracle.resize_indexed(im.indices, im.palette, im.fmt == N.BINARY1, dw, dh)
            assert isinstance(got, IndexedImage) and got.fmt == im.fmt
            assert np.array_equal(got.palette, icx.default_palette(im.fmt == N.BINARY1))
            assert np.array_equal(got.indices, want), (im.shape, im.fmt, scale)
    params = icx.CompressionParams(0.25, 1 << 20, 200, 150, 1 << 20)
    mixed = cases + [smooth(300, 517, 5), noise(96, 640, 6)[:, :, 1].copy()]
    res = codec.png_fit_batch(mixed, params)
    for im, r in zip(mixed, res):
        if r is None:
            continue
        if isinstance(im, IndexedImage):
            want = oracle.resize_indexed(im.indices, im.palette, im.fmt == N.BINARY1, r.shape[1], r.shape[0])
            assert np.array_equal(r.indices, want), (im.shape, im.fmt)
        else:
            assert np.array_equal(r, oracle.resize(im, r.shape[1], r.shape[0]))


def test_create_self_check_catches_a_bad_device_constant(codec, oracle):
    """the first context on a device encodes two
    known-answer frames there, every context compares the device's digest of
    the encoder's constant tables with the host's; with the Huffman constants
    overwritten on the device (debug hook) icx_create fails with
    ICX_E_DEVICE, and once they are restored it succeeds again.  The check
    costs < 1 ms per context."""
    import ctypes
    import time
    L = N.load()
    ctx = ctypes.c_void_p()
    assert L.icx_debug_corrupt_constants(0, 1) == N.OK
    try:
        assert L.icx_create(0, ctypes.byref(ctx)) == N.E_DEVICE
        # an encode on the corrupted device differs from the oracle (what the check guards against)
        img = noise(16, 16, 3)
        assert codec.compress_jpg_to_stream(img, 0.75) != oracle.encode(img, 0.75)
    finally:
        assert L.icx_debug_corrupt_constants(0, 0) == N.OK
    assert codec.compress_jpg_to_stream(img, 0.75) == oracle.encode(img, 0.75)
    times = {}
    import os
    for mode in ("0", "1", "0", "1"):
        os.environ["ICX_SELF_CHECK"] = mode
        try:
            t0 = time.perf_counter()
            for _ in range(5):
                c = ctypes.c_void_p()
                assert L.icx_create(0, ctypes.byref(c)) == N.OK
                L.icx_destroy(c)
            times[mode] = (time.perf_counter() - t0) / 5
        finally:
            del os.environ["ICX_SELF_CHECK"]
    print("icx_create ms without / with the self-check:", times["0"] * 1e3, times["1"] * 1e3)
    assert times["1"] - times["0"] < 1e-3, times


def test_upload_from_a_reader_thread_during_a_call(codec):
    """icx_upload copies host bytes to the context's device on a copy stream
    of its own, concurrently with a batch call on the same context."""
    import threading
    from icx.core import DeviceImage, PinnedBuffer
    rng = np.random.default_rng(4)
    src = [PinnedBuffer(codec, 3 << 20) for _ in range(8)]
    dst = [DeviceImage(codec, (3 << 20,)) for _ in range(8)]
    for s in src:
        s.array[:] = rng.integers(0, 256, s.size, dtype=np.uint8)
    errs = []

    def reader():
        try:
            for s, d in zip(src, dst):
                codec._check(codec._lib.icx_upload(codec._ctx, d.ptr, s.ptr, s.size), "icx_upload")
        except Exception as e:
            errs.append(e)

    t = threading.Thread(target=reader)
    img = noise(1080, 1920, 9)
    t.start()
    codec.fit([img] * 4, 1 << 18, 0.25)
    t.join()
    assert not errs
    for s, d in zip(src, dst):
        assert np.array_equal(d.numpy(), s.array)


def test_edge_tile_dead_waves_repeated(codec, oracle):
    """Widths whose right-edge FDCT tile leaves whole waves without a block
    (1920 px: 8 MCUs in the last tile, waves 2 and 3 empty; 200 px: 7 MCUs)
    encoded repeatedly in one batch: a dead wave must not store a block's list
    metadata it does not own.  The last block of every edge tile
    is checked through the bitstream, byte-exact against the oracle."""
    imgs, refs = [], []
    for i in range(8):
        for h, w in ((1080, 1920), (136, 200), (72, 968)):
            img = noise(h, w, 900 + i) if i % 2 else smooth(h, w, 900 + i)
            imgs.append(img)
    cached = [icx.LearnedParams(0.5, 1.0)] * len(imgs)
    for rep in range(3):
        res = codec.fit(imgs, 1 << 30, 0.5, cached=cached)
        for k, (img, r) in enumerate(zip(imgs, res)):
            if rep == 0:
                refs.append(oracle.encode(img, 0.5))
            assert r["status"] == N.OK and r["success"] and r["cache_hit"], (rep, k)
            assert r["data"] == refs[k], (rep, k, img.shape)
