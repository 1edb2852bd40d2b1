#!/usr/bin/env python3
"""Probe: the headline encode (1000 4K frames in HBM, -t 1 MiB, cached q 0.25)
as one call on one libicx context against the same frames split over N
contexts run at once from N host threads.  The FDCT and the Huffman trials
each sit near 0.45 of both their VALU issue and HBM roofs (latency-bound), so
two independent streams of them might fill each other's gaps.  Prints one
JSON line per configuration."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import icx  # noqa: E402


def run(frames, outs, nctx, steps):
    codecs = [icx.Codec(0) for _ in range(nctx)]
    try:
        parts = [list(range(k, len(frames), nctx)) for k in range(nctx)]
        bs = [c.prepare([frames[i] for i in p], bench.TARGET, bench.Q0, cached=[icx.LearnedParams(bench.Q0, 1.0)] * len(p),
                        outputs=[outs[i] for i in p]) for c, p in zip(codecs, parts)]
        for b in bs:
            b.run()
            assert all(r["success"] and r["status"] == 0 for r in b.results())
        torch.cuda.synchronize()
        go = threading.Barrier(nctx + 1)

        def work(b):
            go.wait()
            for _ in range(steps):
                b.run()

        ts = [threading.Thread(target=work, args=(b,)) for b in bs]
        for t in ts:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        for c in codecs:
            c.close()
    mp = len(frames) * bench.W * bench.H / 1e6
    return {"contexts": nctx, "frames": len(frames), "steps": steps, "ms_per_step": round(dt / steps * 1e3, 3),
            "MP_per_s": round(mp * steps / dt, 1)}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    frames = bench.make_frames(n, 0, dev)
    outs = torch.empty((n, bench.TARGET + 1), dtype=torch.uint8, device=dev)
    for nctx in (1, 2, 3, 1, 2, 3):
        print(json.dumps(run(frames, outs, nctx, steps)), flush=True)


if __name__ == "__main__":
    main()
