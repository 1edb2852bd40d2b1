#!/usr/bin/env python3
"""Does the device decoder overlap the encoder?  The e2e leg of bench.py (q95
4K JPEG bytes in HBM -> icx decode -> compressJpgWithTargetSize) with the
frames split over K contexts on the same GPU, one host thread each (ctypes
releases the GIL), against K = 1."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import icx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ctx", type=int, nargs="+", default=[1, 2, 4])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    import io
    import numpy as np
    from PIL import Image
    srcs = []
    for i in range(8):
        f = bench.make_frames(1, 777 + i * 2 + (i % 2), dev)[0] if i % 2 == 0 else \
            torch.randint(0, 256, (bench.H, bench.W, 3), generator=torch.Generator(device=dev).manual_seed(555 + i),
                          device=dev, dtype=torch.uint8)
        b = io.BytesIO()
        Image.fromarray(f.cpu().numpy()[:, :, ::-1].copy()).save(b, "JPEG", quality=95, subsampling=2)
        srcs.append(torch.from_numpy(np.frombuffer(b.getvalue(), np.uint8).copy()).to(dev))
    n = a.frames
    ins = [srcs[i % 8] for i in range(n)]
    px = [torch.empty((bench.H, bench.W, 3), dtype=torch.uint8, device=dev) for _ in range(n)]
    outs = torch.empty((n, bench.TARGET + 1), dtype=torch.uint8, device=dev)
    res = {}
    for k in a.ctx:
        codecs = [icx.Codec(0) for _ in range(k)]
        parts = [list(range(i, n, k)) for i in range(k)]
        preps = []
        for c, idx in zip(codecs, parts):
            dec = c.prepare_decode([ins[i] for i in idx], [px[i] for i in idx], subsampling=0)
            fit = c.prepare([px[i] for i in idx], bench.TARGET, bench.Q0,
                            cached=[icx.LearnedParams(bench.Q0, 1.0)] * len(idx), outputs=[outs[i] for i in idx])
            preps.append((dec, fit))

        def work(p):
            dec, fit = p
            for _ in range(a.steps):
                dec.run()
                fit.run()

        for p in preps:  # warm-up
            p[0].run()
            p[1].run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ths = [threading.Thread(target=work, args=(p,)) for p in preps]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        assert all(r["success"] for p in preps for r in p[1].results())
        res[k] = {"ms_per_step": round(dt * 1e3, 2), "MP/s": round(n * bench.W * bench.H / 1e6 / dt, 1)}
        print(json.dumps({"contexts": k, **res[k]}), flush=True)
        for c in codecs:
            c.close()


if __name__ == "__main__":
    main()
