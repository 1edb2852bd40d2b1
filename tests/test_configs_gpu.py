"""BASELINE.json configs[3] at full size on the GPU, against the oracle.

configs[3]: 10,000 8K (7680x4320) JPGs, -t 1MB, binary search, sub-sampled
decode.  Per image that is ImageCompression.processImage ->
decodeImageWithSubsampling (ImageCompression.java:107-165: s = 1 for a 7680
max dimension, s = 2 from 8192 on) -> compressJpgWithTargetSize without a
cache entry (ImageCompressionJpg.java:77-122): the binary search at scale 1.0
and, for frames that never fit (uniform noise), the 0.85x
bilinear scale loop (:91-115) around it.  Everything is compared with the
oracle bit for bit: output bytes, float32 quality, double scale, encodes.
"""
import io

import numpy as np
import pytest

import icx
from icx import _native as N
from tests.oracle_ffi import noise, smooth

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _trials(o):
    """The oracle's encode count without saveCompressedImage's re-encode
    (ImageCompressionJpg.java:255-260): the device keeps the best trial's
    stream instead, so it runs exactly the search trials."""
    return o["encodes"] - (1 if o["success"] and not o["cache_hit"] else 0)


def _fit_equal(codec, oracle, imgs, target, q0):
    res = codec.fit(imgs, target, q0)
    out = []
    for i, (img, r) in enumerate(zip(imgs, res)):
        o = oracle.fit(img, target, q0)
        assert r["status"] == N.OK, (i, r["status"])
        assert r["success"] == o["success"] and r["cache_hit"] == o["cache_hit"] is False, i
        assert r["encodes"] == _trials(o), (i, r["encodes"], o["encodes"])
        if o["success"]:
            assert r["data"] == o["data"], i
            assert np.float32(r["learned"].quality) == np.float32(o["quality"]), i
            assert r["learned"].scale == o["scale"], i
        out.append(o)
    return out


def test_8k_fit_binary_search_and_scale_loop(codec, oracle):
    """7680x4320 smooth + uniform noise, -t 1 MiB, q 0.25, no cache entry (one
    device batch).  The noise frame does not fit at scale 1.0 and must come
    out of the resize loop at 0.85 or below."""
    imgs = [smooth(4320, 7680, 801), noise(4320, 7680, 802)]
    o = _fit_equal(codec, oracle, imgs, MIB, 0.25)
    assert o[0]["success"] and o[0]["scale"] == 1.0
    assert o[1]["success"] and o[1]["scale"] <= 0.85
    assert o[1]["encodes"] > 5  # more than one scale visited


def _q95_jpeg(img):
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(img[:, :, ::-1])).save(buf, "JPEG", quality=95, subsampling=2)
    return buf.getvalue()


@pytest.mark.parametrize("kind", ["smooth", "noise"])
def test_8192_source_subsampled_decode_then_fit(codec, oracle, kind):
    """An 8192x4608 q95 source (maxDim >= 8192: s = 2, ImageCompression.java:140-153)
    decoded on the device (IJG 6b decode + keep pixels (2x, 2y): 4096x2304)
    and fitted at -t 1 MiB: pixels, then bytes / q / scale equal the oracle's
    decode + compressJpgWithTargetSize."""
    src = (smooth if kind == "smooth" else noise)(4608, 8192, 803)
    data = _q95_jpeg(src)
    assert oracle.subsampling(8192, 4608) == 2
    rc, ref = oracle.jpeg_decode(data, 2)
    assert rc == 0 and ref.shape == (2304, 4096, 3)
    dec = codec.decode_jpg(data)  # subsampling 0: the reference's rule
    assert dec.shape == ref.shape and np.array_equal(dec, ref)
    # the decoded frame stays in HBM for the fit, as in the pipeline
    st_dev = codec.decode_jpg_batch([data], device_out=True)
    assert st_dev[0][0] == N.OK
    res = codec.fit([st_dev[0][1]], MIB, 0.25)[0]
    o = oracle.fit(ref, MIB, 0.25)
    assert res["status"] == N.OK and res["success"] == o["success"] and o["success"]
    assert res["data"] == o["data"] and res["encodes"] == _trials(o)
    assert np.float32(res["learned"].quality) == np.float32(o["quality"])
    assert res["learned"].scale == o["scale"]
    # the learned-cache key uses the decoded dims and the source file size (CacheTools.java:14-21)
    assert icx.core.create_key(ref, len(data)) == icx.SimilarityKey(*oracle.create_key(4096, 2304, len(data)))
