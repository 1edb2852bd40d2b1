"""world_size-2 gloo run of the sharded batch driver on CPU (no GPU): each
rank compresses its shard of the file list; counters are summed and the
learned caches merged and written by rank 0 (cli.run_distributed)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp
from PIL import Image

from tests.oracle_ffi import noise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lst, out, cache, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "image-compression_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from icx import pipeline
    from icx.cli import run_distributed
    from icx.core import CompressionParams
    from tests.stub_codec import OracleCodec
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = pipeline.CompressionBatch(lst, out, CompressionParams(0.25, 1000, 100, 60, 20000), 1, cache,
                                  codecs=[OracleCodec()], group_size=2, rank=rank, world=world)
    rep, merged = run_distributed(b, dist)
    q.put((rank, rep.total, rep.success, rep.failed, rep.original_size, len(merged)))
    dist.destroy_process_group()


def test_two_rank_sharded_batch(tmp_path):
    files = []
    for i in range(7):
        f = tmp_path / f"img{i}.jpg"
        Image.fromarray(noise(70 + 3 * i, 110 + 40 * i, i)).save(f, "JPEG", quality=95)
        files.append(str(f))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files))
    out = tmp_path / "out"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(lst), str(out), str(tmp_path / "c"), q))
          for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    # every rank reports the global (reduced) totals
    assert res[0][1:] == res[1][1:]
    _, total, success, failed, orig, ncache = res[0]
    assert total == 7 and success == 7 and failed == 0
    assert orig == sum(os.path.getsize(f) for f in files)
    assert sorted(os.listdir(out)) == sorted(os.path.basename(f) for f in files)
    from icx.cache import CacheManager
    assert len(CacheManager(tmp_path / "c").load_all_to_map()) == ncache >= 1
