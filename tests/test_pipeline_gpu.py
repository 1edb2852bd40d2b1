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
    p = d / "pic.png"
    Image.fromarray(smooth(500, 700, 5)[:, :, ::-1]).save(p)
    files.append(str(p))
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
    assert gpu.counts[CompressionResult.COMPRESSED_SUCCESS] >= 10
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


def test_cli_main(codec, tmp_path):
    lst, files = _make_inputs(tmp_path)
    from icx.cli import main
    rc = main(["-f", str(lst), "-o", str(tmp_path / "out"), "-s", "1000", "-w", "150", "-i", "150", "-t", "60000",
               "--cache-db", str(tmp_path / "cache")])
    assert rc == 0
    outs = os.listdir(tmp_path / "out")
    assert len(outs) >= 10 and all(os.path.getsize(tmp_path / "out" / o) <= 60000 for o in outs if o.endswith(".jpg"))
