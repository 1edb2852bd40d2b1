#!/usr/bin/env python3
"""Per-config throughput on one MI355X for BASELINE.json's configs (SURVEY.md
§8d), at bounded frame counts (the multi-GPU variants shard the same work per
rank with no exchange).  Inputs and outputs resident in HBM.
One JSON line per config:

  C2  4K frames, -t 1 MiB, cached q = 0.25 (bench.py's headline workload)
  C3  4K frames, -t 1 MiB, full binary search (no learned cache)
  C3e C3 from q95 JPEG bytes: device decode + search
  C4  8K (7680x4320) q95 JPEG bytes: device decode (s = 1 by the reference's
      rule) + search; noise frames do not fit at scale 1.0 and walk the 0.85x
      scale loop with the bilinear resize
  C5  PNG half: 3840x2160 -> fit into 1920x1920 (ImageCompressionPng), the
      device bilinear resize only, all frames in one icx_png_fit_batch launch
      (deflate runs on host threads)
  C5w the PNG write of those resized frames: icx_png_encode (JDK row filter
      + zlib level 4, C++) on a pool of every usable host core, one frame per
      thread
"""
import argparse
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import icx  # noqa: E402

TARGET = 1 << 20


def jpeg_sources(h, w, distinct, dev):
    from PIL import Image
    out = []
    for i in range(distinct):
        if i % 2 == 0:
            g = torch.Generator(device=dev).manual_seed(9000 + i)
            y = torch.arange(h, device=dev, dtype=torch.float32)[:, None]
            x = torch.arange(w, device=dev, dtype=torch.float32)[None, :]
            f = (127 + 100 * torch.sin(x * 0.01 + i) + 0 * y).expand(h, w)
            bgr = torch.stack([f, (127 + 100 * torch.sin(y * 0.013 + i)).expand(h, w),
                               127 + 100 * torch.sin((x + y) * 0.005)], -1)
            bgr += torch.randn(h, w, 3, generator=g, device=dev) * 16
            img = bgr.round_().clamp_(0, 255).to(torch.uint8)
        else:
            img = torch.randint(0, 256, (h, w, 3), generator=torch.Generator(device=dev).manual_seed(9000 + i),
                                device=dev, dtype=torch.uint8)
        b = io.BytesIO()
        Image.fromarray(img.cpu().numpy()[:, :, ::-1].copy()).save(b, "JPEG", quality=95, subsampling=2)
        out.append(torch.from_numpy(np.frombuffer(b.getvalue(), np.uint8).copy()).to(dev))
    return out


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def fit_line(name, codec, frames, cached, steps, desc, h, w):
    outs = torch.empty((len(frames), TARGET + 1), dtype=torch.uint8, device=frames[0].device)
    P = codec.prepare(frames, TARGET, bench.Q0, cached=cached, outputs=[outs[i] for i in range(len(frames))])
    dt = timed(P.run, steps)
    res = P.results()
    assert all(r["status"] == 0 for r in res)
    return {"config": name, "desc": desc, "frames": len(frames), "ms_per_step": round(dt * 1e3, 3),
            "value": round(len(frames) * h * w / 1e6 / dt, 1), "unit": "MP/s",
            "encodes_per_image": round(sum(r["encodes"] for r in res) / len(res), 2),
            "fit": sum(r["success"] for r in res)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--frames8k", type=int, default=48)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = icx.Codec(0)
    want = set(a.only.split(",")) if a.only else {"C2", "C3", "C3e", "C4", "C5"}
    W, H = bench.W, bench.H
    frames = bench.make_frames(a.frames, 5000, dev) if want & {"C2", "C3", "C5"} else []
    if "C2" in want:
        print(json.dumps(fit_line("C2", codec, frames, [icx.LearnedParams(bench.Q0, 1.0)] * len(frames), a.steps,
                                  "4K, -t 1MiB, cached q=0.25 (search fallback)", H, W)), flush=True)
    if "C3" in want:
        print(json.dumps(fit_line("C3", codec, frames, None, a.steps, "4K, -t 1MiB, binary search, no cache", H, W)),
              flush=True)
    for name, (h, w, n) in {"C3e": (H, W, a.frames), "C4": (4320, 7680, a.frames8k)}.items():
        if name not in want:
            continue
        srcs = jpeg_sources(h, w, 4, dev)
        ins = [srcs[i % len(srcs)] for i in range(n)]
        px = [torch.empty((h, w, 3), dtype=torch.uint8, device=dev) for _ in range(n)]
        outs = torch.empty((n, TARGET + 1), dtype=torch.uint8, device=dev)
        D = codec.prepare_decode(ins, px, subsampling=0)
        F = codec.prepare(px, TARGET, bench.Q0, cached=None, outputs=[outs[i] for i in range(n)])
        assert all(s == 0 for s in D.run())
        td = timed(D.run, a.steps)
        tf = timed(F.run, a.steps)
        res = F.results()
        print(json.dumps({"config": name, "desc": f"{w}x{h} q95 JPEG bytes in HBM -> device decode -> "
                                                  "compressJpgWithTargetSize -t 1MiB (search, scale loop)",
                          "frames": n, "ms_per_step": round((td + tf) * 1e3, 3),
                          "value": round(n * h * w / 1e6 / (td + tf), 1), "unit": "MP/s",
                          "decode_ms": round(td * 1e3, 3), "fit_ms": round(tf * 1e3, 3),
                          "encodes_per_image": round(sum(r["encodes"] for r in res) / n, 2),
                          "scales": sorted({round(r["learned"].scale, 6) for r in res if r["success"]}),
                          "fit": sum(r["success"] for r in res),
                          "mean_src_bytes": int(np.mean([s.numel() for s in srcs]))}), flush=True)
        del px, outs, D, F
    if "C5" in want:
        import ctypes
        from icx import _native as N
        nw, nh = icx.scaled_dims(W, H, min(1920 / W, 1920 / H))
        dst = torch.empty((len(frames), nh, nw, 3), dtype=torch.uint8, device=dev)
        lib, ctx = codec._lib, codec._ctx
        n = len(frames)
        jobs = (N.PngFitJob * n)()
        for i, f in enumerate(frames):
            jobs[i].src = icx.core._image_struct(f)[0]
            jobs[i].min_width = jobs[i].min_height = 1920
            jobs[i].dst, jobs[i].cap = dst[i].data_ptr(), dst[i].numel()

        def run():  # ImageCompressionPng's fit for the group: one launch (icx_png_fit_batch)
            assert lib.icx_png_fit_batch(ctx, jobs, n) == 0 and all(j.status == 0 and j.resized for j in jobs)

        run()
        codec.profile(True)
        codec.profile_reset()
        dt = timed(run, a.steps)
        k = codec.profile_query("resize")
        algo = codec.profile_query("resize.bytes")["units"]
        codec.profile(False)
        kms = k["ms"] / k["launches"]
        print(json.dumps({"config": "C5-png", "desc": f"PNG fit: {W}x{H} -> {nw}x{nh} bilinear on device, "
                                                      "icx_png_fit_batch: one launch per group (deflate on host "
                                                      "threads)",
                          "frames": n, "ms_per_step": round(dt * 1e3, 3),
                          "value": round(n * W * H / 1e6 / dt, 1), "unit": "MP/s (source pixels)",
                          "kernel_ms": round(kms, 4), "launches_per_step": k["launches"] / a.steps,
                          "algo_bytes_per_launch": int(algo / k["launches"]),
                          "algo_bytes_per_dst_px": round(algo / k["units"], 2),
                          "kernel_GBps": round(algo / k["launches"] / (kms / 1e3) / 1e9, 1),
                          "kernel_frac_of_hbm": round(algo / k["launches"] / (kms / 1e3) / 8e12, 4),
                          "frac_at_6B_per_dst_px": round(6 * k["units"] / k["launches"] / (kms / 1e3) / 8e12, 4)}),
              flush=True)
        import concurrent.futures as cf
        from icx.pngio import encode_png
        host = [d.cpu().numpy() for d in dst]
        from icx.pipeline import host_cores
        threads = host_cores()[0]
        with cf.ThreadPoolExecutor(threads) as ex:
            sizes = list(ex.map(encode_png, host[:threads]))  # warm-up
            t0 = time.perf_counter()
            sizes = [len(b) for b in ex.map(encode_png, host)]
            dt = time.perf_counter() - t0
        print(json.dumps({"config": "C5-pngwrite", "desc": f"PNG write of the {nw}x{nh} frames: icx_png_encode "
                                                           f"(JDK RowFilter + zlib level 4, 32 KiB IDATs) on {threads} host threads",
                          "frames": len(host), "threads": threads, "ms_per_step": round(dt * 1e3, 3),
                          "files_per_s": round(len(host) / dt, 1),
                          "value": round(len(host) * W * H / 1e6 / dt, 1), "unit": "MP/s (source pixels)",
                          "mean_png_bytes": int(np.mean(sizes))}), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
