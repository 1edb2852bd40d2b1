"""Palette rasters (ImageTools.java:12-17): a TYPE_BYTE_INDEXED
or TYPE_BYTE_BINARY PNG keeps its type through resizeImage, so the resized
image carries Java2D's DEFAULT colour map of that type and is written back as
a palette / 1-bit PNG (ImageCompressionPng.java:66-70).  Restated from the
published OpenJDK sources on both sides (oracle C, libicx C++); no JDK here,
so this is "parity unpinned" against Java2D.  CPU checks: the two
restatements of the colour-map machinery agree, and the PNG writer's palette
and 1-bit forms decode to the right pixels."""
import ctypes
import io

import numpy as np
from PIL import Image

import icx
from icx import _native as N
from icx.core import IndexedImage, default_palette
from icx.pngio import encode_png


def _oracle_cube(oracle, pal):
    cube = np.zeros(32768, np.uint8)
    p = np.ascontiguousarray(pal, np.uint32)
    oracle.L.oracle_inverse_cube(p.ctypes.data, len(p), cube.ctypes.data)
    return cube


def _icx_cube(pal):
    cube = np.zeros(32768, np.uint8)
    p = np.ascontiguousarray(pal, np.uint32)
    N.load().icx_inverse_colour_map(p.ctypes.data, len(p), cube.ctypes.data)
    return cube


def test_default_maps_and_inverse_maps_agree(oracle):
    """BufferedImage's default maps, AWT initCubemap and make_dither_arrays:
    libicx and the oracle agree (the default maps, random maps of 2..256
    entries with duplicate cells, and the dither tables)."""
    for binary in (0, 1):
        pal = default_palette(binary)
        assert np.array_equal(pal, oracle.default_palette(binary))
        assert np.array_equal(_icx_cube(pal), _oracle_cube(oracle, pal))
    pal = default_palette(False)
    assert pal[0] == 0xff000000 and pal[215] == 0xffffffff and pal[216] == 0xff121212 and pal[255] == 0xfffcfcfc
    rng = np.random.default_rng(3)
    for n in (2, 3, 16, 100, 256):
        p = (0xff000000 | rng.integers(0, 1 << 24, n)).astype(np.uint32)
        p[n // 2] = p[0]  # a duplicate cell: the first claim wins
        assert np.array_equal(_icx_cube(p), _oracle_cube(oracle, p)), n
    d = np.zeros((3, 64), np.int8)
    N.load().icx_dither_tables(d.ctypes.data)
    r, g, b = (np.zeros(64, np.int8) for _ in range(3))
    oracle.L.oracle_dither_tables(256, r.ctypes.data, g.ctypes.data, b.ctypes.data)
    assert np.array_equal(d, np.stack([r, g, b]))
    # the 8x8 Bayer order scaled to [-20, 20): red row 0 is 0, 32, 8, 40, 2, 34, 10, 42
    assert list(d[0, :8]) == [-20, 0, -15, 5, -19, 1, -14, 6]
    assert np.array_equal(d[1].reshape(8, 8), d[0].reshape(8, 8)[:, ::-1])
    assert np.array_equal(d[2].reshape(8, 8), d[0].reshape(8, 8)[::-1, :])


def test_binary_inverse_map_is_the_l1_split(oracle):
    """{black, white}: the flood fill reaches a cell from black first iff its
    5-bit L1 distance to black is the smaller (no ties: 93 is odd)."""
    c = _icx_cube(default_palette(True)).reshape(32, 32, 32)
    r, g, b = np.meshgrid(range(32), range(32), range(32), indexing="ij")
    assert np.array_equal(c == 0, r + g + b <= 46)


def test_oracle_indexed_resize_rules(oracle):
    """The restatement's own invariants: a solid primary is not dithered and
    lands on its corner cell's entry (white's cell is claimed by the grey
    ramp's 252 first: the fill seeds entries 0, 255, 1, 254, ...; which is why
    Java2D's representsPrimaries allows 5 levels of slack), a 1-bit image of
    a grey above / below the split stays white / black, transparent pixels
    compose onto black."""
    pal = np.array([0xff000000, 0xffff0000, 0xff00ff00, 0xffffffff], np.uint32)
    dp = oracle.default_palette(False)
    cube = _oracle_cube(oracle, dp)
    assert dp[cube[32767]] == 0xfffcfcfc and dp[cube[0]] == 0xff000000
    solid = np.zeros((16, 16), np.uint8)
    for k, col in enumerate(pal):
        got = oracle.resize_indexed(solid + k, pal, False, 8, 8)
        cell = (int(col) >> 9 & 0x7c00) | (int(col) >> 6 & 0x3e0) | (int(col) >> 3 & 0x1f)
        assert (got == cube[cell]).all(), hex(col)
    mid = oracle.resize_indexed(solid, np.array([0xff808080], np.uint32), False, 8, 8)
    assert len(np.unique(mid)) > 1  # a mid grey is dithered over the 8x8 pattern
    grey = np.array([0xff8a8a8a, 0xff707070, 0x00ffffff], np.uint32)
    assert (oracle.resize_indexed(np.zeros((9, 9), np.uint8), grey, True, 4, 4) == 1).all()
    assert (oracle.resize_indexed(np.ones((9, 9), np.uint8), grey, True, 4, 4) == 0).all()
    assert (oracle.resize_indexed(np.full((9, 9), 2, np.uint8), grey, True, 4, 4) == 0).all()


def test_png_writer_palette_and_one_bit():
    """PNGMetadata.initialize for an IndexColorModel: the default
    TYPE_BYTE_INDEXED map -> 8-bit palette PNG with the whole map as PLTE
    (filter 0 on every row); {black, white} -> 1-bit grey; a grey-ramp map
    -> grey; a map with alpha -> tRNS.  Decoded pixels equal the map applied."""
    rng = np.random.default_rng(5)
    idx = rng.integers(0, 256, (37, 53)).astype(np.uint8)
    im = IndexedImage(idx, default_palette(False), N.INDEXED8)
    data = encode_png(im)
    assert data[24] == 8 and data[25] == 3
    p = Image.open(io.BytesIO(data))
    assert p.mode == "P" and np.array_equal(np.asarray(p), idx)
    plte = np.frombuffer(bytes(p.getpalette()[:768]), np.uint8).reshape(-1, 3)
    want = default_palette(False)
    assert np.array_equal(plte, np.stack([want >> 16 & 255, want >> 8 & 255, want & 255], -1))
    raw = Image.open(io.BytesIO(data))
    raw.load()
    bits = rng.integers(0, 2, (19, 77)).astype(np.uint8)
    d1 = encode_png(IndexedImage(bits, default_palette(True), N.BINARY1))
    assert d1[24] == 1 and d1[25] == 0
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(d1)).convert("L")), bits * 255)
    ramp = np.arange(256, dtype=np.uint32) * 0x010101 | 0xff000000
    dg = encode_png(IndexedImage(idx, ramp, N.INDEXED8))
    assert dg[24] == 8 and dg[25] == 0 and np.array_equal(np.asarray(Image.open(io.BytesIO(dg))), idx)
    alpha = default_palette(False).copy()
    alpha[3] = 0x40ffffff & alpha[3]
    da = encode_png(IndexedImage(idx, alpha, N.INDEXED8))
    assert b"tRNS" in da and da[25] == 3
    four = IndexedImage(rng.integers(0, 4, (10, 13)).astype(np.uint8),
                        np.array([0xff000000, 0xff555555, 0xffaaaaaa, 0xffffffff], np.uint32), N.BINARY1)
    d2 = encode_png(four)
    assert d2[24] == 2 and d2[25] == 0
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(d2))) , four.indices * 85)


def test_palette_raster_shapes_through_the_abi():
    im = IndexedImage(np.zeros((5, 7), np.uint8), default_palette(False), N.INDEXED8)
    st, keep = icx.core._image_struct(im)
    assert st.fmt == N.INDEXED8 and st.palette_len == 256 and st.width == 7 and st.height == 5
    try:
        icx.core._image_struct(np.zeros((5, 7), np.uint8), N.INDEXED8)
        raise AssertionError("a bare array is not a palette raster")
    except ValueError:
        pass
    assert ctypes.sizeof(N.Image) == 40


def _palette_png(path, idx, plte, trns=None, bits=8):
    im = Image.fromarray(idx, "P")
    im.putpalette([c for rgb in plte for c in rgb])
    kw = {"bits": bits} if bits != 8 else {}
    if trns is not None:
        kw["transparency"] = bytes(trns)
    im.save(path, **kw)


def test_palette_pngs_keep_their_type_through_the_pipeline(tmp_path):
    """processImage on palette / low-bit PNGs (CPU, the oracle as codec): the
    JDK reader's raster (PNGImageReader: 8-bit palette -> TYPE_BYTE_INDEXED,
    1/2/4-bit palette or grey -> TYPE_BYTE_BINARY, map = PLTE padded with its
    last entry, tRNS alphas) resized into the type's default map and written
    as an 8-bit palette PNG (the 6x6x6 cube + grey ramp, no tRNS) or a 1-bit
    grey PNG (ImageTools.java:12-17, ImageCompressionPng.java:66-70)."""
    from icx import pipeline
    from icx.core import CompressionParams, CompressionResult
    from tests.stub_codec import OracleCodec
    rng = np.random.default_rng(11)
    plte = [tuple(int(v) for v in rng.integers(0, 256, 3)) for _ in range(200)]
    _palette_png(tmp_path / "p8.png", rng.integers(0, 200, (90, 130)).astype(np.uint8), plte,
                 trns=[255] * 10 + [0, 128])
    _palette_png(tmp_path / "p4.png", rng.integers(0, 16, (90, 130)).astype(np.uint8), plte[:16], bits=4)
    Image.fromarray((rng.integers(0, 2, (90, 130)) * 255).astype(np.uint8)).convert("1").save(tmp_path / "g1.png")
    params = CompressionParams(0.25, 10, 60, 40, 1 << 20)
    for name, want_depth, want_type in (("p8.png", 8, 3), ("p4.png", 1, 0), ("g1.png", 1, 0)):
        out = tmp_path / "out"
        out.mkdir(exist_ok=True)
        r = pipeline.process_image(tmp_path / name, out, params, {}, OracleCodec())
        assert r.result == CompressionResult.COMPRESSED_SUCCESS, (name, r)
        data = (out / name).read_bytes()
        assert (data[24], data[25]) == (want_depth, want_type), name
        assert b"tRNS" not in data
        w = int.from_bytes(data[16:20], "big")
        h = int.from_bytes(data[20:24], "big")
        assert (w, h) == (57, 40)  # min(60/130, 40/90) = 4/9 of (130, 90)
        # the expected raster: the oracle's restatement of the resize
        src = pipeline._to_array(Image.open(tmp_path / name), tmp_path / name)
        assert isinstance(src, IndexedImage)
        want = OracleCodec().png_resize(src, params)
        got = Image.open(out / name)
        if want_type == 3:
            assert np.array_equal(np.asarray(got), want.indices)
        else:
            assert np.array_equal(np.asarray(got.convert("L")) // 255, want.indices)


def test_png_reader_rasters(tmp_path):
    """_to_array's palette rasters follow PNGImageReader.getImageTypes."""
    from icx import pipeline
    rng = np.random.default_rng(2)
    idx = rng.integers(0, 5, (7, 9)).astype(np.uint8)
    _palette_png(tmp_path / "a.png", idx, [(1, 2, 3), (4, 5, 6), (7, 8, 9), (10, 11, 12), (13, 14, 15)],
                 trns=[0, 255], bits=4)
    r = pipeline._to_array(Image.open(tmp_path / "a.png"), tmp_path / "a.png")
    assert r.fmt == N.BINARY1 and len(r.palette) == 16 and np.array_equal(r.indices, idx)
    assert r.palette[0] == 0x00010203 and r.palette[1] == 0xff040506 and r.palette[4] == 0xff0d0e0f
    depth, ctype, plte, trns = pipeline.png_palette_info(tmp_path / "a.png")
    assert (depth, ctype) == (4, 3)
    for i in range(16):  # PLTE padded to 2^depth with its last entry, tRNS with 255
        assert r.palette[i] & 0xffffff == plte[min(i, len(plte) - 1)]
        assert r.palette[i] >> 24 == (trns[i] if i < len(trns) else 255)
    g = (rng.integers(0, 4, (6, 5)) * 85).astype(np.uint8)
    Image.fromarray(g).save(tmp_path / "g2.png", bits=2)
    r = pipeline._to_array(Image.open(tmp_path / "g2.png"), tmp_path / "g2.png")
    if r is not None and isinstance(r, IndexedImage):  # Pillow wrote a 2-bit grey file
        assert r.fmt == N.BINARY1 and list(r.palette) == [0xff000000, 0xff555555, 0xffaaaaaa, 0xffffffff]
        assert np.array_equal(r.indices, g // 85)


def _bayer8():
    """AWT make_uns_ordered_dither_array: the recursive 8x8 ordered-dither order."""
    oda = np.zeros((8, 8), np.int64)
    k = 1
    while k < 8:
        for i in range(k):
            for j in range(k):
                v = oda[i, j]
                oda[i, j] = v * 4
                oda[i + k, j + k] = v * 4 + 1
                oda[i, j + k] = v * 4 + 2
                oda[i + k, j] = v * 4 + 3
        k *= 2
    return oda


def test_palette_invariants_pinned_without_java2d():
    """Invariants of the (parity-unpinned) palette restatement that hold
    whatever Java2D's exact claim order is, so a refactor cannot drift
    silently: the dither matrix is a permutation of 0..63 scaled to [-20, 20)
    (make_dither_arrays), and every map entry's own 5-bit colour cell maps to
    an entry of that same cell (initCubemap seeds each entry's cell with it)."""
    bay = _bayer8()
    assert sorted(bay.ravel().tolist()) == list(range(64))
    d = np.zeros((3, 64), np.int8)
    N.load().icx_dither_tables(d.ctypes.data)
    assert np.array_equal(d[0].reshape(8, 8), bay * 40 // 64 - 20)
    rng = np.random.default_rng(17)
    maps = [default_palette(False), default_palette(True)]
    maps += [(0xff000000 | rng.integers(0, 1 << 24, n)).astype(np.uint32) for n in (2, 7, 64, 256)]
    for pal in maps:
        cube = _icx_cube(pal)
        cells = ((pal >> 9) & 0x7c00) | ((pal >> 6) & 0x3e0) | ((pal >> 3) & 0x1f)
        got = pal[cube[cells.astype(np.int64)]]
        got_cells = ((got >> 9) & 0x7c00) | ((got >> 6) & 0x3e0) | ((got >> 3) & 0x1f)
        assert np.array_equal(got_cells, cells), len(pal)


def test_png_encode_rejects_bad_colour_maps():
    """icx_png_encode validates a palette raster's map as validate() does:
    null map, no entries, more than 16 for BINARY1 or 256 for INDEXED8."""
    L = N.load()
    idx = np.zeros((4, 4), np.uint8)
    pal = np.full(300, 0xff000000, np.uint32)
    out = np.zeros(1 << 16, np.uint8)
    n = ctypes.c_size_t()
    for fmt, ptr, count in ((N.INDEXED8, None, 4), (N.INDEXED8, pal.ctypes.data, 0), (N.INDEXED8, pal.ctypes.data, 257),
                            (N.BINARY1, pal.ctypes.data, 17), (N.BINARY1, None, 2)):
        img = N.Image(idx.ctypes.data, 4, 4, 4, fmt, ptr, count)
        st = L.icx_png_encode(ctypes.byref(img), -1, out.ctypes.data, out.nbytes, ctypes.byref(n))
        assert st == N.E_INVALID, (fmt, count, st)
    for fmt, count in ((N.INDEXED8, 256), (N.BINARY1, 16), (N.BINARY1, 2)):
        img = N.Image(idx.ctypes.data, 4, 4, 4, fmt, pal.ctypes.data, count)
        assert L.icx_png_encode(ctypes.byref(img), -1, out.ctypes.data, out.nbytes, ctypes.byref(n)) == N.OK
