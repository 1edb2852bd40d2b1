"""End-to-end batch (file list -> output files) through libicx on the GPU,
compared file by file with the same pipeline driven by the oracle."""
import os

import numpy as np
import pytest
from PIL import Image

import icx
from icx import pipeline
from icx.core import CompressionParams, CompressionResult
from tests.oracle_ffi import noise, smooth
from tests.stub_codec import OracleCodec

pytestmark = pytest.mark.gpu


def _make_inputs(d):
    files = []
    rng = np.random.default_rng(0)
    for i in range(10):
        h, w = int(rng.integers(200, 700)), int(rng.integers(200, 900))
        img = smooth(h, w, i) if i % 2 else noise(h, w, i)
        f = d / f"img{i}.jpg"
        Image.fromarray(np.ascontiguousarray(img[:, :, ::-1])).save(f, "JPEG", quality=95)
        files.append(str(f))
    g = d / "grey.jpg"
    Image.fromarray(smooth(400, 500, 99)[:, :, 1]).save(g, "JPEG", quality=95)
    files.append(str(g))
    # progressive: device pixel path here, host Pillow decode on the oracle side
    pj = d / "prog.jpg"
    Image.fromarray(np.ascontiguousarray(smooth(480, 640, 98)[:, :, ::-1])).save(pj, "JPEG", quality=95,
                                                                                progressive=True)
    files.append(str(pj))
    # CMYK and its YCCK twin (Adobe transform 2): decoded on the device now
    from tests.golden.gen_cmyk_golden import cmyk_source, set_transform
    cm = d / "cmyk.jpg"
    Image.fromarray(cmyk_source(300, 410, 9), "CMYK").save(cm, "JPEG", quality=92)
    files.append(str(cm))
    (d / "ycck.jpg").write_bytes(set_transform(cm.read_bytes(), 2))
    files.append(str(d / "ycck.jpg"))
    # damaged JPEGs: the JDK's 6b reader recovers (grey tail, bad code as 0,
    # restart resync) and the reference compresses them; an arithmetic-coded
    # one it refuses (FAILED_IO_ERROR)
    src = open(files[0], "rb").read()
    (d / "cut.jpg").write_bytes(src[: len(src) * 2 // 3])
    bad = bytearray(src)
    bad[len(src) // 2:len(src) // 2 + 8] = b"\xff\x00" * 4
    (d / "badcode.jpg").write_bytes(bytes(bad))
    import io
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(smooth(360, 520, 97)[:, :, ::-1])).save(buf, "JPEG", quality=95,
                                                                                 restart_marker_blocks=3)
    r = buf.getvalue()
    k = [i for i in range(len(r) // 2, len(r) - 1) if r[i] == 0xFF and 0xD0 <= r[i + 1] <= 0xD7][0]
    (d / "rst_missing.jpg").write_bytes(r[:k] + r[k + 2:])
    arith = bytearray(src)
    arith[arith.index(b"\xff\xc0") + 1] = 0xC9
    (d / "arith.jpg").write_bytes(bytes(arith))
    files += [str(d / n) for n in ("cut.jpg", "badcode.jpg", "rst_missing.jpg", "arith.jpg")]
    p = d / "pic.png"
    Image.fromarray(smooth(500, 700, 5)[:, :, ::-1]).save(p)
    files.append(str(p))
    # palette and 1-bit PNGs: TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY kept (IndexedImage)
    pal = Image.fromarray(smooth(420, 640, 7)[:, :, ::-1]).quantize(200)
    pal.save(d / "pal.png", transparency=0)
    files.append(str(d / "pal.png"))
    Image.fromarray(noise(400, 600, 8)[:, :, 0]).convert("1").save(d / "bits.png")
    files.append(str(d / "bits.png"))
    files.append(str(d / "missing.jpg"))
    lst = d / "list.txt"
    lst.write_text("\n".join(files))
    return lst, files


def test_batch_end_to_end_matches_oracle(codec, tmp_path):
    lst, files = _make_inputs(tmp_path)
    params = CompressionParams(0.25, 1000, 150, 150, 60000)
    gpu = pipeline.CompressionBatch(lst, tmp_path / "gpu", params, 1, tmp_path / "gcache", codecs=[codec],
                                    group_size=4).execute()
    cpu = pipeline.CompressionBatch(lst, tmp_path / "cpu", params, 1, tmp_path / "ccache", codecs=[OracleCodec()],
                                    group_size=4).execute()
    assert gpu.counts == cpu.counts and gpu.total == cpu.total == len(files)
    assert gpu.counts[CompressionResult.COMPRESSED_SUCCESS] >= 13
    assert gpu.counts[CompressionResult.FAILED_IO_ERROR] == 1  # arith.jpg
    for name in ("cut.jpg", "badcode.jpg", "rst_missing.jpg"):
        assert (tmp_path / "gpu" / name).exists(), name
    for name in sorted(os.listdir(tmp_path / "cpu")):
        a = (tmp_path / "gpu" / name).read_bytes()
        b = (tmp_path / "cpu" / name).read_bytes()
        if name.endswith(".png"):  # deflate bytes may differ; pixels must not
            assert np.array_equal(np.asarray(Image.open(tmp_path / "gpu" / name)),
                                  np.asarray(Image.open(tmp_path / "cpu" / name)))
        else:
            assert a == b, name
    # a second run hits the learned cache and reproduces the files
    again = pipeline.CompressionBatch(lst, tmp_path / "gpu2", params, 1, tmp_path / "gcache", codecs=[codec],
                                      group_size=4).execute()
    assert again.counts == gpu.counts
    for name in os.listdir(tmp_path / "gpu"):
        if name.endswith(".jpg"):
            assert (tmp_path / "gpu2" / name).read_bytes() == (tmp_path / "gpu" / name).read_bytes()


def test_batch_through_a_pool_matches_one_codec(codec, tmp_path):
    """CompressionBatch driven by icx.Pool([0, 0]) (one process over a device
    list, the JVM shape of CompressionBatch.java:64-88): JPEGs decode on the
    pool's devices into host frames and fit there; the files equal one
    codec's (every JPEG of a Pool's group used to fail)."""
    lst, files = _make_inputs(tmp_path)
    params = CompressionParams(0.25, 1000, 150, 150, 60000)
    pool = icx.Pool([0, 0])
    try:
        got = pipeline.CompressionBatch(lst, tmp_path / "pool", params, 1, tmp_path / "pcache", codecs=[pool],
                                        group_size=4).execute()
    finally:
        pool.close()
    one = pipeline.CompressionBatch(lst, tmp_path / "one", params, 1, tmp_path / "ocache", codecs=[codec],
                                    group_size=4).execute()
    assert got.counts == one.counts and got.success >= 10, got.counts
    for name in sorted(os.listdir(tmp_path / "one")):
        if name.endswith(".jpg"):
            assert (tmp_path / "pool" / name).read_bytes() == (tmp_path / "one" / name).read_bytes(), name


def test_cli_main(codec, tmp_path):
    lst, files = _make_inputs(tmp_path)
    from icx.cli import main
    rc = main(["-f", str(lst), "-o", str(tmp_path / "out"), "-s", "1000", "-w", "150", "-i", "150", "-t", "60000",
               "--cache-db", str(tmp_path / "cache")])
    assert rc == 0
    outs = os.listdir(tmp_path / "out")
    assert len(outs) >= 10 and all(os.path.getsize(tmp_path / "out" / o) <= 60000 for o in outs if o.endswith(".jpg"))


def test_config_c1_single_1080p_jpeg(codec, tmp_path):
    """BASELINE configs[0]: one 1920x1080 q95 JPG file ->
    -t 524288 through CompressionBatch with -w 1000 -i 1000 -s 0 (the default
    -w/-i 1920 would reject a 1080-high image, ImageCompression.java:129-135).
    The file equals the oracle-driven pipeline's byte for byte, and the binary
    search ran (4-5 trial encodes, ImageCompressionJpg.java:158-200)."""
    src = tmp_path / "c1.jpg"
    Image.fromarray(np.ascontiguousarray(noise(1080, 1920, 1)[:, :, ::-1])).save(src, "JPEG", quality=95,
                                                                                   subsampling=2)
    assert os.path.getsize(src) > 524288  # a file above -t: the search has work to do
    lst = tmp_path / "list.txt"
    lst.write_text(str(src))
    params = CompressionParams(0.25, 0, 1000, 1000, 524288)
    calls = []

    class Counting:
        def __init__(self, c):
            self.c = c

        def __getattr__(self, k):
            return getattr(self.c, k)

        def fit(self, *a, **k):
            r = self.c.fit(*a, **k)
            calls.extend(x["encodes"] for x in r)
            return r

    gpu = pipeline.CompressionBatch(lst, tmp_path / "gpu", params, 1, tmp_path / "gc", codecs=[Counting(codec)]
                                    ).execute()
    cpu = pipeline.CompressionBatch(lst, tmp_path / "cpu", params, 1, tmp_path / "cc", codecs=[OracleCodec()]
                                    ).execute()
    assert gpu.counts[CompressionResult.COMPRESSED_SUCCESS] == cpu.counts[CompressionResult.COMPRESSED_SUCCESS] == 1
    a = (tmp_path / "gpu" / "c1.jpg").read_bytes()
    assert a == (tmp_path / "cpu" / "c1.jpg").read_bytes()
    assert len(a) <= 524288 and calls and 4 <= calls[0] <= 5
    with Image.open(tmp_path / "gpu" / "c1.jpg") as im:
        assert im.size == (1920, 1080)


def test_stage_files_facts_and_device_copies(codec, tmp_path):
    """icx_stage_files (the native reader side of the batch): per file
    exists/readable, size, header facts, the dims gate, and for a JPEG the
    device decoder takes, a device copy equal to the file's bytes; small
    files (<= -s) and non-JPEGs are not staged; a missing path is reported."""
    import ctypes
    from icx import _native as N
    from icx.core import DeviceImage
    big = tmp_path / "big.jpg"
    Image.fromarray(np.ascontiguousarray(noise(300, 420, 1)[:, :, ::-1])).save(big, "JPEG", quality=95)
    tiny = tmp_path / "tiny.jpg"
    Image.fromarray(np.ascontiguousarray(noise(50, 400, 2)[:, :, ::-1])).save(tiny, "JPEG", quality=95)
    png = tmp_path / "p.png"
    Image.fromarray(noise(300, 420, 3)).save(png)
    small = tmp_path / "small.jpg"
    Image.fromarray(smooth(300, 420, 4)).save(small, "JPEG", quality=10)
    paths = [big, tmp_path / "missing.jpg", tiny, png, small]
    min_size = small.stat().st_size  # small.jpg sits exactly at -s: not read
    jobs = (N.StageJob * len(paths))()
    keep = [str(p).encode() for p in paths]
    for j, b in zip(jobs, keep):
        j.path, j.min_size, j.min_width, j.min_height = b, min_size, 100, 100
    assert codec._lib.icx_stage_files(codec._ctx, jobs, len(paths)) == N.OK
    j = jobs[0]
    assert j.exists and j.size == big.stat().st_size and j.jpeg_status == N.OK and (j.width, j.height, j.ncomp) == (420, 300, 3)
    assert j.dev and np.array_equal(DeviceImage.adopt(codec, j.dev, (j.size,)).numpy(), np.frombuffer(big.read_bytes(), np.uint8))
    assert not jobs[1].exists and not jobs[1].dev
    assert jobs[2].exists and jobs[2].jpeg_status == N.OK and jobs[2].height == 50 and not jobs[2].dev  # dims gate
    assert jobs[3].exists and jobs[3].jpeg_status == -1 and not jobs[3].dev  # not a JPEG
    assert jobs[4].exists and jobs[4].size == min_size and jobs[4].jpeg_status == -1 and not jobs[4].dev  # at -s
