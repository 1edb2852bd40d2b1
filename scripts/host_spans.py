#!/usr/bin/env python3
"""Host-side time of icx_compress_jpg_batch on the bench workload: the
library's host.* spans (sub-batch preparation up to its first launch, waits
in stage synchronisations, result collection) next to the kernel times and
the call's wall time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import icx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
dev = torch.device("cuda:0")
frames = bench.make_frames(n, 1000, dev)
codec = icx.Codec(0)
outs = [torch.empty(bench.TARGET + 1, dtype=torch.uint8, device=dev) for _ in range(n)]
cached = [icx.LearnedParams(bench.Q0, 1.0)] * n
codec.fit(frames, bench.TARGET, bench.Q0, cached=cached, outputs=outs)
torch.cuda.synchronize()
codec.profile(True)
codec.profile_reset()
t0 = time.perf_counter()
for _ in range(3):
    codec.fit(frames, bench.TARGET, bench.Q0, cached=cached, outputs=outs)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 3 * 1e3
names = ("fdct", "huff", "scan", "ffscan", "stuff", "host.prep", "host.sync", "host.results")
res = {k: codec.profile_query(k) for k in names}
kern = sum(res[k]["ms"] for k in names[:6]) / 3
print(json.dumps({"wall_ms_per_call": round(wall, 3), "kernel_ms_per_call": round(kern, 3),
                  "spans": {k: {"n": res[k]["launches"] / 3, "ms_per_call": round(res[k]["ms"] / 3, 3)}
                            for k in names[6:]}}))
