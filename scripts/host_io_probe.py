#!/usr/bin/env python3
"""Where the files -> files path's host time goes (GPU box): N threads read
1000 4K-q95-sized files (7.8 MB, page cache) into bytes / numpy / pinned
buffers, with and without the icx_upload to HBM, and write 1000 0.85 MB
outputs from bytes / pinned buffers.  Prints one JSON line of GB/s and
per-file milliseconds per variant."""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--size", type=int, default=7_800_000)
    ap.add_argument("--out-size", type=int, default=875_000)
    a = ap.parse_args()
    import icx
    from icx.core import DeviceImage, PinnedBuffer
    codec = icx.Codec(0)
    work = tempfile.mkdtemp(prefix="icx_io_")
    blob = np.random.default_rng(1).integers(0, 256, a.size, dtype=np.uint8).tobytes()
    paths = []
    for i in range(a.files):
        p = os.path.join(work, f"f{i:05d}.bin")
        with open(p, "wb") as f:
            f.write(blob)
        paths.append(p)
    res = {"files": a.files, "threads": a.threads, "bytes_per_file": a.size}

    def timed(name, fn, items, nbytes):
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(a.threads) as ex:
            list(ex.map(fn, items))
        dt = time.perf_counter() - t0
        res[name] = {"s": round(dt, 4), "GBps": round(nbytes / dt / 1e9, 2), "ms_per_file": round(dt / len(items) * 1e3, 3)}
        print(name, res[name], flush=True)

    def rd_bytes(p):
        with open(p, "rb") as f:
            return len(f.read())

    def rd_pinned(p):
        b = PinnedBuffer.read_file(codec, p)
        b.free()

    dev = [None] * a.files

    def rd_upload(i):
        b = PinnedBuffer.read_file(codec, paths[i])
        d = DeviceImage(codec, (b.size,))
        codec._check(codec._lib.icx_upload(codec._ctx, d.ptr, b.ptr, b.size), "icx_upload")
        b.free()
        dev[i] = d

    def rd_pread(p):
        b = PinnedBuffer(codec, a.size)
        fd = os.open(p, os.O_RDONLY)
        try:
            n = os.preadv(fd, [memoryview(b.array)], 0)
        finally:
            os.close(fd)
        b.free()
        return n

    total = a.files * a.size
    for r in range(2):  # round 2: warm pools
        timed(f"read_bytes_r{r}", rd_bytes, paths, total)
        timed(f"read_pinned_r{r}", rd_pinned, paths, total)
        timed(f"preadv_pinned_r{r}", rd_pread, paths, total)
        timed(f"read_pinned_upload_r{r}", rd_upload, list(range(a.files)), total)
        for d in dev:
            if d is not None:
                d.free()
    out = np.random.default_rng(2).integers(0, 256, a.out_size, dtype=np.uint8)
    pins = [PinnedBuffer(codec, a.out_size) for _ in range(64)]
    for p in pins:
        p.array[:] = out
    ob = out.tobytes()
    od = os.path.join(work, "out")
    os.makedirs(od)

    def wr_bytes(i):
        with open(os.path.join(od, f"b{i:05d}.jpg"), "wb") as f:
            f.write(ob)

    def wr_pinned(i):
        with open(os.path.join(od, f"p{i:05d}.jpg"), "wb") as f:
            f.write(memoryview(pins[i % 64].array))

    def wr_os(i):
        fd = os.open(os.path.join(od, f"o{i:05d}.jpg"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            os.write(fd, memoryview(pins[i % 64].array))
        finally:
            os.close(fd)

    for r in range(2):
        timed(f"write_bytes_r{r}", wr_bytes, list(range(a.files)), a.files * a.out_size)
        timed(f"write_pinned_r{r}", wr_pinned, list(range(a.files)), a.files * a.out_size)
        timed(f"write_os_pinned_r{r}", wr_os, list(range(a.files)), a.files * a.out_size)
    shutil.rmtree(work, ignore_errors=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
