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


def _worker(rank, world, port, lst, out, cache, q, report_shard=False):
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
    if report_shard:  # this rank's own shard (before the reduction): line indices and bytes
        mine = pipeline.shard(pipeline.read_file_list(lst), rank, world)
        q.put((rank, [i for i, _ in mine], sum(os.path.getsize(p) for _, p in mine), rep.total, rep.success))
    else:
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


def test_two_rank_shards_balance_skewed_sizes(tmp_path):
    """gloo world_size 2 over a skewed list (two large files among small
    ones, both large ones early in the list): each rank's shard holds within
    10 % of the bytes, every file is compressed once."""
    files = []
    for i in range(12):
        f = tmp_path / f"img{i}.jpg"
        h, w = (300, 400) if i in (0, 2) else (60 + 3 * i, 110 + 10 * i)
        Image.fromarray(noise(h, w, i)).save(f, "JPEG", quality=95)
        files.append(str(f))
    lst = tmp_path / "list.txt"
    lst.write_text("\n".join(files))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, str(lst), str(tmp_path / "out"), str(tmp_path / "c"), q,
                                            True)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    assert sorted(res[0][1] + res[1][1]) == list(range(12))
    b0, b1 = res[0][2], res[1][2]
    assert max(b0, b1) <= 1.10 * min(b0, b1), (b0, b1)
    assert res[0][3:] == res[1][3:] == (12, 12)


def _timing_worker(rank, world, port, q):
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench.rank_sync(dist)
    t0 = time.perf_counter()
    time.sleep(0.05 + 0.25 * rank)  # rank 1 is the slow one
    bench.rank_sync(dist)
    q.put((rank, time.perf_counter() - t0, bench.ranks_max(dist, 0.1 * (rank + 1))))
    dist.destroy_process_group()


def test_two_rank_leg_timing_is_max_over_ranks():
    """bench.py's host-fed legs (host_io, pool, e2e) run on every rank at
    N > 1: the timed region is bracketed by barriers (both ranks see the slow
    rank's time) and the reported time is the max over ranks (gloo)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_timing_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    for rank, wall, mx in got:
        assert wall >= 0.29, (rank, wall)  # the barrier waits for rank 1's 0.3 s
        assert abs(mx - 0.2) < 1e-9


def _shared_cache_worker(rank, world, port, a, b, out, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "image-compression_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from torch.distributed.distributed_c10d import _get_default_store
    from icx import pipeline
    from icx.cache import SharedCache
    from icx.core import CompressionParams
    from tests.stub_codec import OracleCodec

    class RecCodec(OracleCodec):
        seen = []

        def fit(self, images, target, quality, cached=None, outputs=None):
            res = super().fit(images, target, quality, cached, outputs)
            RecCodec.seen += [(c is not None, r["cache_hit"]) for c, r in zip(cached or [None] * len(res), res)]
            return res

    dist.init_process_group("gloo", rank=rank, world_size=world)
    cache = SharedCache(_get_default_store())
    P = CompressionParams(0.25, 1000, 100, 60, 40000)
    lst = os.path.join(out, f"list{rank}.txt")
    with open(lst, "w") as f:
        f.write(a if rank == 0 else b)
    batch = pipeline.CompressionBatch(lst, os.path.join(out, f"o{rank}"), P, 1, os.path.join(out, "c"),
                                      codecs=[RecCodec()], group_size=1)
    if rank == 1:
        dist.barrier()  # rank 0 has learned file a's parameters
    rep = batch.execute(cache=cache, save_cache=False)
    if rank == 0:
        dist.barrier()
    q.put((rank, rep.success, RecCodec.seen, len(cache)))
    dist.destroy_process_group()


def test_ranks_share_one_learned_cache(tmp_path):
    """under torchrun every rank had its own L1 map, so a
    key learned on rank 0 was no hit on rank 1 during the run.  With
    SharedCache (the process group's store carries new entries) rank 1's
    file, whose similarity key equals the one rank 0 learned earlier in the
    same run, is probed with the learned parameters and hits (one encode),
    as under the reference's single ConcurrentHashMap."""
    img = noise(150, 220, 5)
    a = tmp_path / "a.jpg"
    Image.fromarray(img).save(a, "JPEG", quality=95)
    b = tmp_path / "b.jpg"
    b.write_bytes(a.read_bytes())  # same dims and size bucket: the same SimilarityKey
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shared_cache_worker, args=(r, 2, port, str(a), str(b), str(tmp_path), q))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    (r0, ok0, seen0, n0), (r1, ok1, seen1, n1) = res
    assert ok0 == ok1 == 1
    assert seen0 == [(False, False)]  # rank 0: cold, full search, learns the key
    assert seen1 == [(True, True)]    # rank 1: probed with rank 0's entry, and it fits
    assert n1 == 1


def _cache_stress_worker(rank, world, port, puts, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "image-compression_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from torch.distributed.distributed_c10d import _get_default_store
    from icx.cache import SharedCache
    from icx.core import LearnedParams, SimilarityKey
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = _get_default_store()
    cache = SharedCache(store)
    rng = np.random.default_rng(rank)
    per_refresh = []
    for g in range(puts // 50):  # groups of 50 puts: refresh (probe), puts, flush - as the pipeline does
        with cache.lock:
            before = cache.records_read
            cache.refresh()
            per_refresh.append(cache.records_read - before)
            for _ in range(50):
                k = SimilarityKey(int(rng.integers(0, 40)), int(rng.integers(0, 30)), int(rng.integers(0, 20)))
                cache[k] = LearnedParams(float(np.float32(rng.uniform(0.01, 1))), float(rng.choice([1.0, 0.85])))
            cache.flush()
    dist.barrier()
    cache.refresh()
    serial = None
    if rank == 0:  # the serial last-writer-wins map: every chunk in counter order
        n = int(store.add(SharedCache.COUNT, 0))
        serial = {}
        for c in range(1, n + 1):
            for r in np.frombuffer(bytes(store.get(f"{SharedCache.CHUNK}{c}")), SharedCache._REC):
                serial[SimilarityKey(int(r["w"]), int(r["h"]), int(r["s"]))] = LearnedParams(float(r["q"]),
                                                                                                 float(r["scale"]))
        written = sum(len(np.frombuffer(bytes(store.get(f"{SharedCache.CHUNK}{c}")), SharedCache._REC))
                      for c in range(1, n + 1))
        serial = (serial, written)
    q.put((rank, dict(cache), cache.records_read, per_refresh, serial))
    dist.barrier()
    dist.destroy_process_group()


def test_shared_cache_eight_ranks_bounded_refresh():
    """8 gloo ranks, 20k puts in all (2500 each, in groups
    of 50 between refreshes).  Every rank reads each published record exactly
    once (total refresh cost = the records written: O(new entries), not the
    whole log per refresh), and every rank's final map equals the serial
    last-writer-wins map of all chunks in counter order."""
    world, puts = 8, 2500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cache_stress_worker, args=(r, world, port, puts, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda t: t[0])
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    serial, written = res[0][4]
    assert written <= world * puts
    for rank, final, read, per_refresh, _ in res:
        assert final == serial, rank
        assert read == written, (rank, read, written)  # each record read once, whatever the interleaving
        assert sum(per_refresh) <= written, rank
