"""Execute.java's picocli command (Execute.java:14-88) with the same flags and
defaults, plus GPU placement flags.

  python -m icx -f list.txt -o outdir [-q 0.25] [-s 1048576] [-w 1920] [-i 1920]
                [-t 1048576] [--timeOut 24] [--cache-db image-compression-cache]
                [--devices 0,1] [--workers-per-device 2] [--group 64] [--group-max 0]
                [--decode-threads N] [--write-threads 4]

Each device gets --workers-per-device GPU worker threads, each with its own
libicx context, so one group's host work (file bytes to the decoder, results
to the writers) overlaps another group's kernels, and one context's
latency-bound relaxation launches overlap another's bulk kernels.  Files ->
files JPEG on one MI355X, round 6 (1000 4K q95 files, medians of three runs,
interleaved configurations; profiles/r6/pipeline/): two workers with groups of
64 ran 3810-4320 files/s warm and 3825-4198 with every file searched, three
workers 3078-3148 and larger groups (--group-max 128 / 256) 3160-3670 in the
same calls; the box drifts 15-25 % over a call, so only the interleaved order
separates them.  The output files go through four writer
threads of their own (--write-threads): sixteen contended on the output
directory (warm 3597-4068 files/s against 4869-5548 with four).
Multi-GPU: by default one process drives every visible GPU (worker threads
per device sharing one L1 cache, the reference's one ConcurrentHashMap); or
one process per GPU under torchrun (RANK/WORLD_SIZE/LOCAL_RANK): the file
list is sharded by file size (longest-processing-time first,
pipeline.shard), the ranks share one L1 cache through the process group's
store while they run (cache.SharedCache), result counters are summed and
rank 0 writes the L2 cache (H2 AUTO_SERVER's multi-process role,
H2CacheManager.java:34-35).
"""
import argparse
import logging
import os
import sys

from .core import CompressionParams

log = logging.getLogger("icx")


def build_parser():
    p = argparse.ArgumentParser(prog="image-compressor", description="批次圖片壓縮工具")
    p.add_argument("-f", "--file-list", required=True, help="包含圖片路徑的文字檔案。")
    p.add_argument("-o", "--output-dir", required=True, help="壓縮後圖片的儲存目錄。")
    p.add_argument("-q", "--quality", type=float, default=0.25)
    p.add_argument("-s", "--minSize", type=int, default=1048576)
    p.add_argument("-w", "--minWidth", type=int, default=1920)
    p.add_argument("-i", "--minHeight", type=int, default=1920)
    p.add_argument("-t", "--target-max-size", type=int, default=1048576)
    p.add_argument("--timeOut", type=float, default=24)
    p.add_argument("--cache-db", default="image-compression-cache")
    p.add_argument("--devices", default=None,
                   help="GPU ordinals for this process, e.g. 0,1 (default: every visible GPU; LOCAL_RANK under torchrun)")
    p.add_argument("--workers-per-device", type=int, default=2,
                   help="GPU worker threads (libicx contexts) per device")
    p.add_argument("--group", type=int, default=64, help="JPEGs (or PNGs) per device batch")
    p.add_argument("--group-max", type=int, default=0,
                   help="files a GPU worker takes at once when more are waiting (0: --group, fixed groups; "
                        "larger calls measured no faster, DESIGN.md §9)")
    p.add_argument("--decode-threads", type=int, default=None)
    p.add_argument("--write-threads", type=int, default=4, help="threads writing the JPEG output files")
    p.add_argument("-V", "--version", action="version", version="1.0")
    return p


def default_devices(devices_arg, world: int, local_rank: int, visible: int):
    """The GPUs this process drives.  --devices wins; under torchrun (world
    > 1) each rank takes its LOCAL_RANK's GPU; otherwise ONE process drives
    every visible GPU (worker threads per device sharing one L1 learned
    cache: the reference's single ConcurrentHashMap, CompressionBatch.java:71,
    VERDICT r4 item 5), falling back to device 0."""
    if devices_arg:
        return [int(x) for x in str(devices_arg).split(",")]
    if world > 1:
        return [local_rank]
    return list(range(visible)) if visible > 0 else [0]


def params_of(a) -> CompressionParams:
    return CompressionParams(float(a.quality), int(a.minSize), int(a.minWidth), int(a.minHeight),
                             int(a.target_max_size))


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s - %(message)s")
    from .pipeline import BatchReport, CompressionBatch
    from . import Codec
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    from . import _native as N
    devices = default_devices(a.devices, world, local, N.load().icx_device_count() if not a.devices else 0)
    params = params_of(a)
    log.info("壓縮任務開始: 來源列表 %s, 輸出目錄 %s, q=%s, 最小尺寸 %dx%d, 最小大小 %d, 目標 %d, 快取 %s",
             os.path.abspath(a.file_list), os.path.abspath(a.output_dir), a.quality, a.minWidth, a.minHeight,
             a.minSize, a.target_max_size, os.path.abspath(a.cache_db))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    codecs = [Codec(d) for d in devices for _ in range(max(1, a.workers_per_device))]
    batch = CompressionBatch(a.file_list, a.output_dir, params, a.timeOut, a.cache_db, codecs=codecs,
                             group_size=a.group, decode_threads=a.decode_threads, rank=rank, world=world,
                             group_max=a.group_max, write_threads=a.write_threads)
    if dist is None:
        rep = batch.execute()
    else:
        rep, _ = run_distributed(batch, dist)
    if rank == 0:
        rep.log()
        log.info("所有任務執行完畢 (%.2f s)", rep.seconds)
    for c in codecs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


def run_distributed(batch, dist):
    """Every rank compresses its shard; the ranks share one L1 cache (loaded
    from the same L2 file, new entries exchanged through the process group's
    store, cache.SharedCache); counters are summed, the cache saved on rank 0."""
    import torch
    from .cache import CacheManager
    from .pipeline import BatchReport
    mgr = CacheManager(batch.h2_cache_path) if dist.get_rank() == 0 else None
    if mgr is not None:
        mgr.init_schema()
    dist.barrier()
    loaded = CacheManager(batch.h2_cache_path).load_all_to_map()
    # one L1 map across ranks: learned entries travel through the process
    # group's store while the ranks run (cache.SharedCache)
    from .cache import SharedCache
    from torch.distributed.distributed_c10d import _get_default_store
    cache = SharedCache(_get_default_store(), loaded)
    rep = batch.execute(cache=cache, save_cache=False)
    dist.barrier()
    cache.refresh()
    v = torch.tensor(rep.to_vector(), dtype=torch.int64)
    dist.all_reduce(v)
    total = BatchReport.from_vector(v.tolist())
    t = torch.tensor([rep.seconds], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    total.seconds = float(t.item())
    gathered = [None] * dist.get_world_size()
    dist.all_gather_object(gathered, dict(cache))
    merged = {}
    for g in gathered:  # rank order: later ranks win on equal keys (last-writer-wins, as the reference)
        merged.update(g)
    total.cache_size = len(merged)
    if mgr is not None:
        mgr.save_all_from_map(merged)
        mgr.close()
    return total, merged


if __name__ == "__main__":
    sys.exit(main())
