"""Host-side logic of processImage / CompressionBatch / cache / CLI, restating
the reference's rules (ImageCompression.java:47-183, CompressionBatch.java,
H2CacheManager.java, Execute.java).  No GPU: compression goes to an
oracle-backed test double."""
import io
import os

import numpy as np
import pytest
from PIL import Image

import icx
from icx import pipeline
from icx.cache import CacheManager, LockedDict, db_file
from icx.cli import build_parser, params_of
from icx.core import CompressionParams, CompressionResult, LearnedParams, SimilarityKey
from tests.oracle_ffi import noise, smooth
from tests.stub_codec import OracleCodec


def write_jpeg(path, bgr, quality=95):
    Image.fromarray(np.ascontiguousarray(bgr[:, :, ::-1])).save(path, "JPEG", quality=quality)


P = CompressionParams(0.25, 1000, 100, 60, 20000)


def test_not_found(tmp_path):
    r = pipeline.process_image(tmp_path / "missing.jpg", tmp_path, P, {}, None)
    assert r == icx.CompressionReport(CompressionResult.SKIPPED_NOT_FOUND, 0, 0)


def test_small_file_skipped(tmp_path):
    f = tmp_path / "a.jpg"
    write_jpeg(f, smooth(16, 16, 1))
    size = os.path.getsize(f)
    r = pipeline.process_image(f, tmp_path, CompressionParams(0.25, size, 1, 1, 10 ** 6), {}, None)
    assert r == icx.CompressionReport(CompressionResult.SKIPPED_CONDITION_NOT_MET, size, size)


def test_dims_gate_reports_unsupported_format(tmp_path):
    """Appendix A.1/A.2: w <= minW || h <= minH gives a null decode, which a
    file above -s reports as FAILED_UNSUPPORTED_FORMAT."""
    f = tmp_path / "wide.jpg"
    write_jpeg(f, noise(60, 400, 2))
    size = os.path.getsize(f)
    r = pipeline.process_image(f, tmp_path, CompressionParams(0.25, 10, 100, 60, 10 ** 6), {}, None)
    assert r == icx.CompressionReport(CompressionResult.FAILED_UNSUPPORTED_FORMAT, size, size)


def test_no_reader_is_unsupported(tmp_path):
    f = tmp_path / "text.jpg"
    f.write_bytes(b"not an image" * 500)
    r = pipeline.process_image(f, tmp_path, P, {}, None)
    assert r.result == CompressionResult.FAILED_UNSUPPORTED_FORMAT


def test_other_readable_format_fails_compression(tmp_path):
    f = tmp_path / "x.gif"
    Image.fromarray(noise(80, 120, 3)[:, :, 0]).save(f, "GIF")
    out = tmp_path / "out"
    out.mkdir()
    r = pipeline.process_image(f, out, CompressionParams(0.25, 10, 100, 60, 10 ** 6), {}, OracleCodec())
    assert r.result == CompressionResult.FAILED_COMPRESSION and r.compressed_size == 0
    assert not (out / "x.gif").exists()


def test_subsampled_decode(tmp_path):
    f = tmp_path / "big.jpg"
    img = smooth(6, 8200, 4)
    write_jpeg(f, img, 90)
    d = pipeline.decode_image_with_subsampling(str(f), CompressionParams(0.25, 0, 1, 1, 0), os.path.getsize(f))
    assert d.subsampling == 2 and d.image.shape == (3, 4100, 3) and d.format_name == "jpeg"
    full = np.asarray(Image.open(f).convert("RGB"))[:, :, ::-1]
    assert np.array_equal(d.image, full[::2, ::2])


def test_jpeg_pipeline_with_cache(tmp_path):
    f = tmp_path / "in.jpg"
    img = noise(90, 120, 5)
    write_jpeg(f, img)
    out = tmp_path / "out"
    out.mkdir()
    cache = LockedDict()
    codec = OracleCodec()
    r = pipeline.process_image(f, out, P, cache, codec)
    assert r.result == CompressionResult.COMPRESSED_SUCCESS
    data = (out / "in.jpg").read_bytes()
    assert len(data) <= P.target_max_size_bytes and r.compressed_size == len(data)
    decoded = np.asarray(Image.open(f).convert("RGB"))[:, :, ::-1]
    assert data == codec.o.fit(decoded, P.target_max_size_bytes, P.quality)["data"]
    key = SimilarityKey(1, 0, os.path.getsize(f) // 102400)
    assert key in cache
    # second run: cache hit, same bytes
    r2 = pipeline.process_image(f, out, P, cache, codec)
    assert r2.result == CompressionResult.COMPRESSED_SUCCESS and (out / "in.jpg").read_bytes() == data


def test_unreachable_target_deletes_output(tmp_path):
    f = tmp_path / "in.jpg"
    write_jpeg(f, noise(90, 120, 6))
    out = tmp_path / "out"
    out.mkdir()
    (out / "in.jpg").write_bytes(b"stale")
    r = pipeline.process_image(f, out, CompressionParams(0.25, 10, 100, 60, 300), LockedDict(), OracleCodec())
    assert r.result == CompressionResult.FAILED_COMPRESSION and not (out / "in.jpg").exists()


def test_png_pipeline(tmp_path):
    f = tmp_path / "p.png"
    Image.fromarray(smooth(300, 400, 7)[:, :, ::-1]).save(f)
    out = tmp_path / "out"
    out.mkdir()
    r = pipeline.process_image(f, out, CompressionParams(0.25, 10, 100, 60, 0), LockedDict(), OracleCodec())
    assert r.result == CompressionResult.COMPRESSED_SUCCESS
    assert Image.open(out / "p.png").size == (80, 60)  # scale = min(100/400, 60/300)


def test_cache_manager_roundtrip(tmp_path):
    path = tmp_path / "db" / "cache.mv.db"
    assert db_file(path).endswith("db/cache.icx.sqlite")
    m = CacheManager(path)
    m.init_schema()
    d = {SimilarityKey(38, 21, 9): LearnedParams(0.2421875, 1.0),
         SimilarityKey(1, 2, 3): LearnedParams(float(np.float32(0.1)), 0.85 * 0.85)}
    assert m.save_all_from_map(d) == 2
    m.save_all_from_map({SimilarityKey(1, 2, 3): LearnedParams(0.5, 1.0)})  # MERGE replaces
    back = m.load_all_to_map()
    assert back[SimilarityKey(38, 21, 9)] == LearnedParams(0.2421875, 1.0)
    assert back[SimilarityKey(1, 2, 3)] == LearnedParams(0.5, 1.0)
    m.close()


def test_batch_report_counts(tmp_path):
    files = []
    for i in range(4):
        f = tmp_path / f"n{i}.jpg"
        write_jpeg(f, noise(70 + i, 110, 10 + i))
        files.append(str(f))
    files.append(str(tmp_path / "missing.jpg"))
    small = tmp_path / "tiny.jpg"
    write_jpeg(small, smooth(8, 8, 1))
    files.append(str(small))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files) + "\n\n")
    b = pipeline.CompressionBatch(lst, tmp_path / "out", CompressionParams(0.25, 1000, 100, 60, 20000), 1,
                                  tmp_path / "cache", codecs=[OracleCodec()], group_size=3)
    rep = b.execute()
    assert rep.total == 6 and rep.success == 4
    assert rep.counts[CompressionResult.SKIPPED_NOT_FOUND] == 1
    assert rep.counts[CompressionResult.SKIPPED_CONDITION_NOT_MET] == 1
    assert rep.failed == 0 and rep.cache_size >= 1
    assert len(CacheManager(tmp_path / "cache").load_all_to_map()) == rep.cache_size


def test_cli_defaults():
    a = build_parser().parse_args(["-f", "l.txt", "-o", "o"])
    assert params_of(a) == CompressionParams(0.25, 1048576, 1920, 1920, 1048576)
    assert a.timeOut == 24 and a.cache_db == "image-compression-cache"


def test_cli_default_devices():
    """without --devices one process drives every
    visible GPU (one shared L1 cache); under torchrun a rank takes its
    LOCAL_RANK's GPU; --devices wins; no GPU visible -> device 0."""
    from icx.cli import default_devices
    assert default_devices(None, 1, 0, 8) == list(range(8))
    assert default_devices(None, 1, 0, 1) == [0]
    assert default_devices(None, 1, 0, 0) == [0]
    assert default_devices(None, 8, 5, 8) == [5]
    assert default_devices("0,0,3", 1, 0, 8) == [0, 0, 3]
    assert default_devices("2", 4, 1, 8) == [2]
    # two worker contexts per device, fixed groups of 64 (DESIGN.md §9, round 6 measurements)
    from icx.cli import build_parser
    a = build_parser().parse_args(["-f", "l.txt", "-o", "out"])
    assert a.workers_per_device == 2 and a.group == 64 and a.group_max == 0
    assert a.write_threads == 4  # JPEG outputs from a few writer threads (pipeline.CompressionBatch)


def test_shard_partition():
    lines = [f"f{i}" for i in range(11)]
    parts = [pipeline.shard(lines, r, 3) for r in range(3)]
    assert sorted(i for p in parts for i, _ in p) == list(range(11))
    assert [len(p) for p in parts] == [4, 4, 3]


def test_shard_balances_skewed_costs():
    """Cost-balanced sharding (8K and noise files cost ~2x a
    smooth 4K one): a skewed mix of file costs splits within 10 % across 8
    ranks, where the old i % world split is off by far more; every line goes
    to exactly one rank and each shard keeps list order."""
    rng = np.random.default_rng(5)
    costs = {}
    lines = []
    for i in range(400):  # 4K smooth ~2.5 MB, 4K noise ~7.7 MB, a few 8K ~30 MB, in runs
        c = [2_500_000, 7_700_000, 30_000_000][0 if i % 50 < 30 else 1 if i % 50 < 47 else 2]
        c += int(rng.integers(0, 200_000))
        lines.append(f"f{i}.jpg")
        costs[lines[-1]] = c
    world = 8
    parts = [pipeline.shard(lines, r, world, cost=costs.__getitem__) for r in range(world)]
    idx = [i for p in parts for i, _ in p]
    assert sorted(idx) == list(range(len(lines)))
    assert all([i for i, _ in p] == sorted(i for i, _ in p) for p in parts)
    loads = [sum(costs[f] for _, f in p) for p in parts]
    assert max(loads) <= 1.10 * min(loads)
    rr = [sum(costs[f] for i, f in enumerate(lines) if i % world == r) for r in range(world)]
    assert max(rr) > 1.10 * min(rr)  # the skew is real: round robin would not balance it


def test_two_codecs_share_the_work_queue(tmp_path):
    """In-process --devices: one worker thread per codec pulls device groups
    from one queue and they share one L1 cache; every output equals the
    single-codec oracle run."""
    import time

    class SlowCodec(OracleCodec):
        def fit(self, *a, **k):
            time.sleep(0.05)  # long enough that the other worker takes the next group
            return super().fit(*a, **k)

    files = []
    for i in range(8):
        f = tmp_path / f"img{i}.jpg"
        # distinct cache keys (w // 100 differs): outputs do not depend on completion order
        write_jpeg(f, (smooth if i % 2 else noise)(70 + 4 * i, 150 + 100 * i, i))
        files.append(str(f))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files))
    codecs = [SlowCodec(), SlowCodec()]
    out = tmp_path / "out"
    b = pipeline.CompressionBatch(str(lst), str(out), P, 1, str(tmp_path / "c"), codecs=codecs, group_size=1)
    rep = b.execute()
    assert rep.total == 8 and rep.success == 8
    assert all(c.calls >= 1 for c in codecs) and sum(c.calls for c in codecs) == 8
    ref_out = tmp_path / "ref"
    ref = pipeline.CompressionBatch(str(lst), str(ref_out), P, 1, str(tmp_path / "c2"), codecs=[OracleCodec()],
                                    group_size=1)
    assert ref.execute().success == 8
    for f in files:
        n = os.path.basename(f)
        assert (out / n).read_bytes() == (ref_out / n).read_bytes()


def test_four_devices_share_one_learned_cache(tmp_path, monkeypatch):
    """Single-process multi-device mode (--devices): four codecs, one L1
    cache - the reference's one ConcurrentHashMap (CompressionBatch.java:71,
    ImageCompressionJpg.java:79-85, 111).  Four files with the same
    SimilarityKey arrive one after another: the first is searched and its
    LearnedParams put; every later one, whichever device takes its group, is a
    cache hit (one encode at the learned quality), and the hits are served by
    more than one device."""
    import threading
    import time
    served = []
    lock = threading.Lock()

    class RecCodec(OracleCodec):
        def fit(self, images, target, quality, cached=None, outputs=None):
            res = super().fit(images, target, quality, cached=cached, outputs=outputs)
            with lock:
                served.extend((id(self), c is not None, r["cache_hit"]) for c, r in zip(cached or [None], res))
            return res

    img = smooth(180, 260, 7)
    files = []
    for i in range(4):  # same pixels and file size: the same (w/100, h/100, size/102400) key
        f = tmp_path / f"same{i}.jpg"
        write_jpeg(f, img)
        files.append(str(f))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files))
    orig = pipeline._prepare

    def staggered(index, *a, **k):  # file k is decoded 0.4 k s after the first
        time.sleep(0.4 * index)
        return orig(index, *a, **k)

    monkeypatch.setattr(pipeline, "_prepare", staggered)
    codecs = [RecCodec() for _ in range(4)]
    cache = {}
    b = pipeline.CompressionBatch(str(lst), str(tmp_path / "out"), P, 1, str(tmp_path / "c"), codecs=codecs,
                                  group_size=1, decode_threads=4)
    rep = b.execute(cache=cache, save_cache=False)
    assert rep.total == 4 and rep.success == 4
    assert len(served) == 4
    assert [(c, h) for _, c, h in served] == [(False, False)] + [(True, True)] * 3
    assert len({dev for dev, _, _ in served}) >= 2  # hits on devices other than the learner's
    assert rep.cache_size == 1
    outs = {(tmp_path / "out" / os.path.basename(f)).read_bytes() for f in files}
    assert len(outs) == 1  # the cached-parameter encode reproduces the searched file


def _png_idat_rows(data, h):
    """Inflated IDAT of a single-IDAT PNG, as (h, 1 + rowbytes) filtered rows."""
    import struct
    import zlib
    pos, idat = 8, b""
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        if data[pos + 4:pos + 8] == b"IDAT":
            idat += data[pos + 8:pos + 8 + n]
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8)
    return raw.reshape(h, -1)


def test_png_writer_adaptive_filters_round_trip():
    """icx_png_encode (native, libicx): every row filter the adaptive choice
    can pick decodes back to the exact pixels (PNG parity is on pixels,
    SURVEY.md §8c), and the filtered rows - filter type and residuals - equal
    the numpy reference writer's (tests/png_ref.py) for grey, BGR and ABGR."""
    import io

    from PIL import Image

    from icx.pngio import encode_png
    from tests.png_ref import filter_rows
    rng = np.random.default_rng(5)
    y = np.arange(64)[:, None]
    x = np.arange(97)[None, :]
    grad = np.stack(np.broadcast_arrays((x + y) % 256, (3 * x) % 256, (5 * y) % 256), -1).astype(np.uint8)
    alpha = np.concatenate([np.broadcast_to((x * y) % 256, (64, 97))[:, :, None].astype(np.uint8), grad], -1)
    for img in [grad, rng.integers(0, 256, (31, 17, 3), dtype=np.uint8), grad[:, :, 1].copy(),
                np.zeros((1, 1, 3), np.uint8), rng.integers(0, 256, (5, 2), dtype=np.uint8), alpha,
                rng.integers(0, 256, (9, 13, 4), dtype=np.uint8)]:
        data = encode_png(img)
        back = np.asarray(Image.open(io.BytesIO(data)))
        assert np.array_equal(back, img if img.ndim == 2 else img[:, :, ::-1])  # BGR/ABGR -> RGB/RGBA
        rows = img if img.ndim == 2 else np.ascontiguousarray(img[:, :, ::-1])
        bpp = 1 if img.ndim == 2 else img.shape[2]
        ref = filter_rows(rows.reshape(img.shape[0], -1), bpp)
        assert np.array_equal(_png_idat_rows(data, img.shape[0]), ref)
    types = set(filter_rows(grad.reshape(64, -1), 3)[:, 0].tolist())
    assert len(types) >= 2  # the smooth gradient picks predictive filters, not only "None"


def _png_chunks(data):
    import struct
    pos, out = 8, []
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        out.append((data[pos + 4:pos + 8], n))
        pos += 12 + n
    return out


def test_png_row_filter_is_the_jdk_heuristic():
    """RowFilter.filterRow (OpenJDK PNGImageWriter, restated in icx_png.cpp):
    None costs the sum of the unsigned bytes, the predictors the sum of
    |int difference| - not the residual bytes read as signed, which would
    score a row of 0xFF as 1 per byte and keep None.  Ties keep the lower
    type."""
    from icx.pngio import encode_png
    from tests.png_ref import filter_rows
    # row 0: all 255 -> None costs 255 n, Sub 255 (the first byte only): Sub;
    # row 1: the same row again -> Up costs 0: Up;
    # row 2: a ramp 0, 3, 6, ... -> Sub costs 3 per byte, Up |ramp - 255|: Sub;
    # row 3: all zero -> None costs 0, as does nothing else before it: None (tie rule)
    w = 40
    img = np.zeros((4, w), np.uint8)
    img[0] = 255
    img[1] = 255
    img[2] = (np.arange(w) * 3).astype(np.uint8)
    rows = filter_rows(img, 1)
    assert rows[:, 0].tolist() == [1, 2, 1, 0]
    assert np.array_equal(_png_idat_rows(encode_png(img), 4), rows)
    # the old signed-residual heuristic would have kept None for row 0
    assert np.abs(img[0].view(np.int8).astype(int)).sum() < 255


def test_png_idat_chunks_and_default_level():
    """IDATOutputStream cuts the zlib stream into 32768-byte IDAT chunks; the
    stream is zlib's at PNGImageWriter's default level 4 (FLEVEL 1 in the
    header: levels 2-5)."""
    from icx.pngio import encode_png
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (300, 200, 3), dtype=np.uint8)  # incompressible: ~180 KB of IDAT data
    data = encode_png(img)
    ch = _png_chunks(data)
    assert [t for t, _ in ch][0] == b"IHDR" and ch[-1] == (b"IEND", 0)
    idat = [n for t, n in ch if t == b"IDAT"]
    assert len(idat) >= 5 and all(n == 32768 for n in idat[:-1]) and 0 < idat[-1] <= 32768
    zhdr = data[8 + 25 + 8: 8 + 25 + 10]
    assert zhdr[0] == 0x78 and (zhdr[1] >> 6) == 1  # deflate, 32K window; FLEVEL 1 (zlib levels 2..5)


def test_png_16bit_grey_is_written_as_16bit():
    """TYPE_USHORT_GRAY is kept (ImageTools.java:12-15): a uint16 raster is
    written as a 16-bit grey PNG (big-endian samples, bytesPerPixel 2 for the
    row filter) that decodes to the same samples."""
    import io

    from PIL import Image

    from icx.pngio import encode_png
    from tests.png_ref import filter_rows
    rng = np.random.default_rng(8)
    img = rng.integers(0, 65536, (23, 41), dtype=np.uint16)
    img[5:] = np.arange(41, dtype=np.uint16) * 1601  # smooth rows: predictive filters
    data = encode_png(img)
    assert data[24] == 16 and data[25] == 0
    back = np.asarray(Image.open(io.BytesIO(data))).astype(np.uint16)
    assert np.array_equal(back, img)
    be = img.astype(">u2").view(np.uint8).reshape(23, -1)
    assert np.array_equal(_png_idat_rows(data, 23), filter_rows(be, 2))


def test_png_alpha_kept_through_the_pipeline(tmp_path):
    """ImageTools.java:12-15 keeps the alpha channel: an RGBA PNG is resized
    as TYPE_4BYTE_ABGR (premultiplied bilinear, icx_resize restatement) and
    written back as an RGBA PNG with its alpha; a grey+alpha PNG (TYPE_CUSTOM
    -> TYPE_INT_ARGB) comes back as RGBA too; opaque RGB stays RGB."""
    from PIL import Image

    from tests.oracle_ffi import Oracle
    rng = np.random.default_rng(9)
    h, w = 90, 160
    rgba = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    rgba[:30, :, 3] = 0      # transparent band
    rgba[30:60, :, 3] = 255  # opaque band
    Image.fromarray(rgba, "RGBA").save(tmp_path / "a.png")
    la = rng.integers(0, 256, (h, w, 2), dtype=np.uint8)
    Image.fromarray(la, "LA").save(tmp_path / "b.png")
    Image.fromarray(rgba[:, :, :3].copy(), "RGB").save(tmp_path / "c.png")
    out = tmp_path / "out"
    out.mkdir()
    params = CompressionParams(0.25, 10, 100, 60, 20000)
    o = Oracle()
    for name in ("a.png", "b.png", "c.png"):
        r = pipeline.process_image(tmp_path / name, out, params, {}, OracleCodec())
        assert r.result == CompressionResult.COMPRESSED_SUCCESS, name
    a = Image.open(out / "a.png")
    assert a.mode == "RGBA" and a.size == (100, 56)
    exp = o.resize(np.ascontiguousarray(rgba[:, :, ::-1]), 100, 56)[:, :, ::-1]  # ABGR restatement -> RGBA
    assert np.array_equal(np.asarray(a), exp)
    assert (np.asarray(a)[:15, :, 3] == 0).all() and (np.asarray(a)[:15] == 0).all()
    assert Image.open(out / "b.png").mode == "RGBA"
    assert Image.open(out / "c.png").mode == "RGB"


def test_alpha_resize_restatement_rules():
    """The oracle's four-byte resize (Java2D TransformHelper + IntArgbPre
    SrcOver blit): opaque pixels give the three-byte result, XRGB writes 0 in
    its spare byte, fully transparent output pixels are zero, and each
    channel stays within its alpha bound (C <= A when premultiplied)."""
    from tests.oracle_ffi import Oracle
    o = Oracle()
    rng = np.random.default_rng(2)
    bgr = rng.integers(0, 256, (23, 37, 3), dtype=np.uint8)
    ref = o.resize(bgr, 15, 11)
    opaque = np.concatenate([np.full((23, 37, 1), 255, np.uint8), bgr], -1)  # ABGR, A = 255
    assert np.array_equal(o.resize(opaque, 15, 11)[:, :, 1:], ref)
    xrgb = np.concatenate([bgr, rng.integers(0, 256, (23, 37, 1), dtype=np.uint8)], -1)  # B G R X
    r = o.resize(xrgb, 15, 11, fmt=3)
    assert np.array_equal(r[:, :, :3], ref) and (r[:, :, 3] == 0).all()
    clear = opaque.copy()
    clear[:, :, 0] = 0
    assert (o.resize(clear, 15, 11) == 0).all()
    mixed = np.concatenate([rng.integers(0, 256, (23, 37, 1), dtype=np.uint8), bgr], -1)
    r = o.resize(mixed, 40, 30)
    assert ((r[:, :, 0] == 0) <= (r[:, :, 1:] == 0).all(-1)).all()  # alpha 0 -> zero pixel


def _dc_symbol_16(data):
    """data with one DC Huffman table symbol set to 16: jdhuff.c
    jpeg_make_d_derived_tbl refuses the table (JERR_BAD_HUFF_TABLE), so the
    JDK reader's read() throws."""
    d = bytearray(data)
    i = d.index(b"\xff\xc4")
    assert d[i + 4] >> 4 == 0  # a DC table
    d[i + 4 + 1 + 16] = 16
    return bytes(d)


def test_truncated_jpeg_is_compressed(tmp_path):
    """A scan cut short decodes as the JDK's 6b reader decodes it (fake EOI,
    then the rest of the scan grey: jdhuff.c insufficient_data) and is
    compressed (the reference compresses such files; it was
    FAILED_IO_ERROR here)."""
    from tests.oracle_ffi import Oracle
    o = Oracle()
    good = []
    for i in range(3):
        f = tmp_path / f"g{i}.jpg"
        write_jpeg(f, noise(70 + i, 110, 20 + i))
        good.append(str(f))
    cut = tmp_path / "cut.jpg"
    data = (tmp_path / "g0.jpg").read_bytes()
    cut.write_bytes(data[: len(data) * 3 // 5])  # header intact, scan truncated
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join([good[0], str(cut), good[1], good[2]]) + "\n")
    params = CompressionParams(0.25, 1000, 60, 60, 20000)
    b = pipeline.CompressionBatch(lst, tmp_path / "out", params, 1, tmp_path / "cache", codecs=[OracleCodec()],
                                  group_size=4)
    rep = b.execute(cache=LockedDict())
    assert rep.total == 4 and rep.success == 4, rep.counts
    rc, px = o.jpeg_decode(cut.read_bytes())
    assert rc == 0 and (px[-8:] == 128).all()  # the grey tail
    ref = o.fit(px, params.target_max_size_bytes, params.quality)
    assert (tmp_path / "out" / "cut.jpg").read_bytes() == ref["data"]


def test_corrupt_jpeg_fails_alone_in_its_group(tmp_path):
    """A JPEG the JDK reader cannot read (a DC table with a symbol over 15)
    fails by itself (FAILED_IO_ERROR, as reader.read's IOException does in
    ImageCompression.java:94-96); the valid files of its device group still
    compress (one bad file used to fail the whole group).  The
    device decoder's refusal goes to the host reader, which refuses it too."""
    good = []
    for i in range(3):
        f = tmp_path / f"g{i}.jpg"
        write_jpeg(f, noise(70 + i, 110, 20 + i))
        good.append(str(f))
    bad = tmp_path / "bad.jpg"
    bad.write_bytes(_dc_symbol_16((tmp_path / "g0.jpg").read_bytes()))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join([good[0], str(bad), good[1], good[2]]) + "\n")
    b = pipeline.CompressionBatch(lst, tmp_path / "out", CompressionParams(0.25, 1000, 60, 60, 20000), 1,
                                  tmp_path / "cache", codecs=[OracleCodec()], group_size=4)
    rep = b.execute(cache=LockedDict())
    assert rep.total == 4 and rep.success == 3, rep.counts
    assert rep.counts[CompressionResult.FAILED_IO_ERROR] == 1
    for g in good:
        assert (tmp_path / "out" / os.path.basename(g)).exists()
    assert not (tmp_path / "out" / "bad.jpg").exists()


@pytest.mark.parametrize("sof", [0xC9, 0xCA, 0xCB, 0xC5, 0xCD, "p12"])
def test_refused_jpeg_flavours(tmp_path, sof):
    """Arithmetic coding (SOF9-11), hierarchical (SOF5-7, 13-15) and 12-bit
    files: the reference's reader reports their size (TwelveMonkeys parses
    the SOF) and its read() throws (the JDK's 6b: JERR_ARITH_NOTIMPL /
    JERR_SOF_UNSUPPORTED / JERR_BAD_PRECISION): FAILED_IO_ERROR past the dims
    gate, FAILED_UNSUPPORTED_FORMAT under it; never a host decode (Pillow's
    libjpeg-turbo would read an arithmetic file)."""
    f = tmp_path / "a.jpg"
    write_jpeg(f, noise(80, 120, 9))
    d = bytearray(f.read_bytes())
    i = d.index(b"\xff\xc0")
    if sof == "p12":
        d[i + 4] = 12
    else:
        d[i + 1] = sof
    f.write_bytes(bytes(d))
    size = len(d)
    out = tmp_path / "out"
    out.mkdir()
    r = pipeline.process_image(f, out, CompressionParams(0.25, 10, 100, 60, 10 ** 6), {}, OracleCodec())
    assert r == icx.CompressionReport(CompressionResult.FAILED_IO_ERROR, size, 0)
    r = pipeline.process_image(f, out, CompressionParams(0.25, 10, 100, 90, 10 ** 6), {}, OracleCodec())
    assert r == icx.CompressionReport(CompressionResult.FAILED_UNSUPPORTED_FORMAT, size, size)
    lst = tmp_path / "list.txt"
    lst.write_text(str(f) + "\n")
    rep = pipeline.CompressionBatch(lst, out, CompressionParams(0.25, 10, 100, 60, 10 ** 6), 1, tmp_path / "cache",
                                    codecs=[OracleCodec()]).execute(cache=LockedDict())
    assert rep.counts[CompressionResult.FAILED_IO_ERROR] == 1


def test_truncated_progressive_jpeg_uses_the_fake_eoi(tmp_path):
    """A file the device path leaves to the host reader (here a progressive
    file cut short) is read with the JDK source manager's fake EOI appended,
    so its damaged scan decodes instead of raising."""
    f = tmp_path / "p.jpg"
    buf = io.BytesIO()
    Image.fromarray(smooth(90, 120, 3)).save(buf, "JPEG", quality=90, progressive=True)
    data = buf.getvalue()
    f.write_bytes(data[: len(data) * 2 // 3])
    out = tmp_path / "out"
    out.mkdir()
    r = pipeline.process_image(f, out, CompressionParams(0.25, 10, 100, 60, 10 ** 6), {}, OracleCodec())
    assert r.result == CompressionResult.COMPRESSED_SUCCESS


def test_unopenable_jpeg_is_an_io_error(tmp_path):
    """FF D8 FF then garbage: the JDK's JPEG reader SPI takes the file
    (canDecodeInput) and reading fails: FAILED_IO_ERROR, not 'no reader'."""
    f = tmp_path / "g.jpg"
    f.write_bytes(b"\xff\xd8\xff\xe0" + b"\x00" * 3000)
    r = pipeline.process_image(f, tmp_path, CompressionParams(0.25, 10, 100, 60, 10 ** 6), {}, OracleCodec())
    assert r.result == CompressionResult.FAILED_IO_ERROR


def test_host_output_codec_in_the_batch(tmp_path):
    """A codec that decodes into host memory only (icx.Pool declares
    supports_device_out = False) is asked for host frames by the pipeline,
    never for device_out (every JPEG of a Pool's group failed)."""
    files = []
    for i in range(4):
        f = tmp_path / f"h{i}.jpg"
        write_jpeg(f, noise(60 + i, 100, 40 + i))
        files.append(str(f))

    class HostOnlyCodec(OracleCodec):
        supports_device_out = False

        def decode_jpg_batch(self, datas, subsampling=0, device_out=False):
            if device_out:
                raise ValueError("host output only")
            return super().decode_jpg_batch(datas, subsampling, device_out)

    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files) + "\n")
    P = CompressionParams(0.25, 1000, 50, 50, 20000)
    rep = pipeline.CompressionBatch(lst, tmp_path / "out", P, 1, tmp_path / "cache", codecs=[HostOnlyCodec()],
                                    group_size=4).execute(cache=LockedDict())
    ref = pipeline.CompressionBatch(lst, tmp_path / "ref", P, 1, tmp_path / "cache2", codecs=[OracleCodec()],
                                    group_size=4).execute(cache=LockedDict())
    assert rep.success == ref.success == 4, rep.counts
    for f in files:
        n = os.path.basename(f)
        assert (tmp_path / "out" / n).read_bytes() == (tmp_path / "ref" / n).read_bytes()


def test_cache_errors_do_not_abort(tmp_path, caplog):
    """H2CacheManager.loadAllToMap / saveAllFromMap catch SQLException, log it
    and carry on (cache/H2CacheManager.java:89-92, 148-152); the JDBC path has
    every '.mv.db' removed (:32)."""
    import sqlite3
    assert db_file(tmp_path / "a.mv.db" / "c.mv.db").endswith("a/c.icx.sqlite")
    m = CacheManager(tmp_path / "c")
    m.init_schema()
    m.save_all_from_map({SimilarityKey(1, 2, 3): LearnedParams(0.5, 1.0)})
    m.conn.execute("DROP TABLE LEARNED_PARAMS_CACHE")
    assert len(m.load_all_to_map()) == 0  # logged, empty map
    assert m.save_all_from_map({SimilarityKey(1, 2, 3): LearnedParams(0.5, 1.0)}) == 0  # rolled back
    m.close()
    # a file that is not a database: the batch logs the error and ends, no exception
    bad = tmp_path / "junk"
    (tmp_path / "junk.icx.sqlite").write_bytes(b"not a database" * 100)
    lst = tmp_path / "list.txt"
    lst.write_text("missing.jpg\n")
    rep = pipeline.CompressionBatch(lst, tmp_path / "out", P, 1, bad, codecs=[OracleCodec()]).execute()
    assert rep.total == 0


def test_worker_failure_fails_its_group_not_the_run(tmp_path):
    """an error escaping a group (here a BaseException out of the
    fit, which compress_jpeg_group does not catch) fails that group's files
    (FAILED_UNKNOWN) instead of killing the GPU worker thread, so the next
    groups still compress; and a pinned-buffer allocation failure falls back
    to host output buffers."""
    files = []
    for i in range(4):
        f = tmp_path / f"w{i}.jpg"
        write_jpeg(f, noise(60 + i, 100, 80 + i))
        files.append(str(f))

    class Boom(BaseException):
        pass

    class FlakyCodec(OracleCodec):
        def fit(self, images, *a, **k):
            if self.calls == 0:
                self.calls += 1
                raise Boom()
            return super().fit(images, *a, **k)

    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files) + "\n")
    P = CompressionParams(0.25, 1000, 50, 50, 20000)
    rep = pipeline.CompressionBatch(lst, tmp_path / "out", P, 1, tmp_path / "cache", codecs=[FlakyCodec()],
                                    group_size=2, decode_threads=1).execute(cache=LockedDict())
    assert rep.total == 4 and rep.success == 2, rep.counts
    assert rep.counts[CompressionResult.FAILED_UNKNOWN] == 2

    class NoPinned(OracleCodec):
        _ctx = object()  # looks like a libicx codec: the pipeline asks for pinned buffers

    def no_pinned(codec, size):
        raise icx.core.N.IcxError(icx.core.N.E_NOMEM, "hipHostMalloc")

    import icx.core
    orig = icx.core.PinnedBuffer.__init__
    icx.core.PinnedBuffer.__init__ = no_pinned
    try:
        it = pipeline._Item(0, files[0])
        it.decoded = pipeline.DecodedImage(np.zeros((8, 8, 3), np.uint8), "jpeg", 8, 8, 1)
        assert pipeline._pinned_outputs(NoPinned(), [it], P) is None
    finally:
        icx.core.PinnedBuffer.__init__ = orig


def test_stage_times_are_per_batch(tmp_path):
    """Two batches in one process keep their own StageTimes (a
    module-global timer let one run's end cut off the other's timing)."""
    files = []
    for i in range(3):
        f = tmp_path / f"s{i}.jpg"
        write_jpeg(f, noise(60 + i, 100, 90 + i))
        files.append(str(f))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files) + "\n")
    P = CompressionParams(0.25, 1000, 50, 50, 20000)
    import threading
    reps = {}

    def run(k):
        b = pipeline.CompressionBatch(lst, tmp_path / f"out{k}", P, 1, tmp_path / f"cache{k}",
                                      codecs=[OracleCodec()], group_size=3, stage_times=True)
        reps[k] = b.execute(cache=LockedDict())

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k in range(2):
        assert reps[k].success == 3
        assert reps[k].stages["write"]["calls"] == 3, reps[k].stages
        assert reps[k].stages["gpu_fit"]["calls"] == 1


def test_staged_items_follow_process_image_gates(tmp_path, caplog):
    """_staged_item (files staged natively by icx_stage_files) maps the staged
    facts to the results _prepare gives, in ImageCompression.java:53-76's
    order: not found, the -s size gate, an I/O error, the dims gate (a JPEG
    the device decoder took but no larger than -w/-i: FAILED_UNSUPPORTED_
    FORMAT, ImageCompression.java:69-72), other formats to the host readers,
    and a staged device JPEG with its header's facts."""
    from icx import _native as N
    P = CompressionParams(0.25, 1000, 100, 60, 20000)

    def job(**k):
        j = N.StageJob()
        j.exists, j.size, j.jpeg_status = 1, 5000, N.OK
        j.width, j.height, j.ncomp = 300, 200, 3
        for a, v in k.items():
            setattr(j, a, v)
        return j

    png = tmp_path / "x.png"
    Image.fromarray(noise(80, 120, 3)).save(png)
    reader = lambda p: open(p, "rb").read()  # noqa: E731 (host bytes: _prepare's own readers)
    R = CompressionResult
    it = pipeline._staged_item(0, "gone.jpg", job(exists=0), None, P, tmp_path, reader)
    assert it.report.result == R.SKIPPED_NOT_FOUND
    it = pipeline._staged_item(0, "small.jpg", job(size=1000), None, P, tmp_path, reader)
    assert it.report.result == R.SKIPPED_CONDITION_NOT_MET and it.report.original_size == 1000
    it = pipeline._staged_item(0, "bad.jpg", job(read_errno=5), None, P, tmp_path, reader)
    assert it.report.result == R.FAILED_IO_ERROR
    it = pipeline._staged_item(0, "tiny.jpg", job(width=100), None, P, tmp_path, reader)
    assert it.report.result == R.FAILED_UNSUPPORTED_FORMAT and it.report.compressed_size == 5000
    it = pipeline._staged_item(3, str(png), job(jpeg_status=-1, size=png.stat().st_size), None, P, tmp_path, reader)
    assert it.report is None and it.decoded.format_name == "png" and it.index == 3
    dev = object()
    it = pipeline._staged_item(4, "/in/a.jpg", job(width=9000, height=5000, ncomp=4), dev, P, tmp_path, reader)
    assert it.report is None and it.decoded.data is dev and it.decoded.subsampling == 2
    assert (it.decoded.width, it.decoded.height, it.decoded.ncomp) == (9000, 5000, 4)
    assert it.output == os.path.join(str(tmp_path), "a.jpg") and it.original_size == 5000


def test_shared_cache_log_semantics():
    """SharedCache over a key-value store (the process group's store; a dict
    stand-in here): a flush publishes the pending 28-byte records as one
    chunk under the next counter value, refresh() applies only the chunks it
    has not applied, in chunk order (later writers win), quality stays
    float32-exact, a put that changes nothing publishes nothing, and a
    refresh with nothing new reads nothing."""
    from icx.cache import SharedCache
    from icx.core import LearnedParams, SimilarityKey

    class Store:
        def __init__(self):
            self.kv = {}

        def add(self, k, n):
            self.kv[k] = int(self.kv.get(k, 0)) + n
            return self.kv[k]

        def set(self, k, b):
            self.kv[k] = b

        def multi_get(self, keys):
            return [self.kv[k] for k in keys]

    st = Store()
    a, b = SharedCache(st), SharedCache(st)
    assert a.refresh() == 0
    k1, k2 = SimilarityKey(38, 21, 7), SimilarityKey(76, 43, 12)
    a[k1] = LearnedParams(0.2421875, 1.0)
    assert a.flush() == 1
    b[k2] = LearnedParams(0.1, 0.85)
    b[k1] = LearnedParams(0.125, 0.7224999999999999)  # later writer
    assert b.flush() == 2
    assert st.kv[SharedCache.COUNT] == 2 and len(st.kv[SharedCache.CHUNK + "2"]) == 2 * 28
    assert a.refresh() == 3 and b.refresh() == 3 and a.refresh() == 0
    assert dict(a) == dict(b)
    assert a[k1] == LearnedParams(0.125, 0.7224999999999999) and a[k2].quality == float(np.float32(0.1))
    a[k2] = LearnedParams(float(np.float32(0.1)), 0.85)  # no change: nothing to publish
    assert a.flush() == 0 and b.refresh() == 0
