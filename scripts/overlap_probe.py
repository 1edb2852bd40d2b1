#!/usr/bin/env python3
"""Experiment: does running two sub-batches on two contexts (two HIP streams)
at once shorten the bench step?  One codec x N frames vs two codecs x N/2
frames driven from two host threads.  Timing only (outputs validated)."""
import json
import sys
import threading
import time
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import icx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda:0")
frames = bench.make_frames(n, 1000, dev)
outs = torch.empty((n, bench.TARGET + 1), dtype=torch.uint8, device=dev)
cached = [icx.LearnedParams(bench.Q0, 1.0)] * n


def timed(batches, steps=3):
    for b in batches:
        b.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        th = [threading.Thread(target=b.run) for b in batches]
        for x in th:
            x.start()
        for x in th:
            x.join()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


res = {}
c1 = icx.Codec(0)
b1 = c1.prepare(frames, bench.TARGET, bench.Q0, cached=cached, outputs=[outs[i] for i in range(n)])
res["one_ctx_ms"] = timed([b1]) * 1e3
codecs = [icx.Codec(0) for _ in range(lanes)]
per = n // lanes
bs = [codecs[k].prepare(frames[k * per:(k + 1) * per], bench.TARGET, bench.Q0, cached=cached[k * per:(k + 1) * per],
                        outputs=[outs[i] for i in range(k * per, (k + 1) * per)]) for k in range(lanes)]
res[f"{lanes}_ctx_ms"] = timed(bs) * 1e3
for b in [b1] + bs:
    r = b.results()
    assert all(x["success"] and x["status"] == 0 for x in r)
res["frames"] = n
print(json.dumps(res))
