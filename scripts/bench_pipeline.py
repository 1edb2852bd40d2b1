#!/usr/bin/env python3
"""End-to-end product throughput: CompressionBatch (CompressionBatch.java:41-148)
over a file list on local disk -> output files, one MI355X.  JPEG files are
read and header-parsed on host threads, decoded on the GPU straight into HBM,
compressed there (compressJpgWithTargetSize, -t 1 MiB), and written back.
Inputs: synthetic 4K q95 JPEGs (half smooth, half noise), written to a
scratch directory first (not timed).  Runs the batch twice with the same
cache DB: run 1 learns (full search), run 2 is the warm-cache run (C5's
timing rule).  Prints one JSON line."""
import argparse
import io
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=200)
    ap.add_argument("--distinct", type=int, default=8)
    ap.add_argument("--group", type=int, default=64)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    from PIL import Image

    import icx
    from icx import pipeline
    from icx.core import CompressionParams
    from tests.oracle_ffi import noise, smooth
    work = a.dir or tempfile.mkdtemp(prefix="icx_pipe_")
    src = os.path.join(work, "src")
    os.makedirs(src, exist_ok=True)
    blobs = []
    for i in range(a.distinct):
        img = (smooth if i % 2 == 0 else noise)(2160, 3840, 70 + i)
        b = io.BytesIO()
        Image.fromarray(np.ascontiguousarray(img[:, :, ::-1])).save(b, "JPEG", quality=95, subsampling=2)
        blobs.append(b.getvalue())
    paths = []
    for i in range(a.files):
        p = os.path.join(src, f"f{i:05d}.jpg")
        with open(p, "wb") as f:
            f.write(blobs[i % a.distinct])
        paths.append(p)
    lst = os.path.join(work, "list.txt")
    with open(lst, "w") as f:
        f.write("\n".join(paths))
    params = CompressionParams(0.25, 1 << 20, 1920, 1920, 1 << 20)  # Execute.java defaults
    codec = icx.Codec(0)
    runs = []
    for r in range(2):
        out = os.path.join(work, f"out{r}")
        t0 = time.perf_counter()
        rep = pipeline.CompressionBatch(lst, out, params, 1, os.path.join(work, "cache"), codecs=[codec],
                                        group_size=a.group).execute()
        dt = time.perf_counter() - t0
        runs.append({"run": "learn" if r == 0 else "warm cache", "seconds": round(dt, 3),
                     "images_per_s": round(rep.total / dt, 1), "mp_per_s": round(rep.megapixels / dt, 1),
                     "success": rep.success, "failed": rep.failed, "skipped": rep.skipped,
                     "in_bytes": rep.original_size, "out_bytes": rep.compressed_size})
    codec.close()
    print(json.dumps({"metric": "CompressionBatch end-to-end (files -> files), 4K q95 JPEG, -t 1MiB, 1 GPU",
                      "files": a.files, "group_size": a.group, "mean_src_bytes": int(np.mean([len(b) for b in blobs])),
                      "runs": runs}))
    if not a.dir:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
