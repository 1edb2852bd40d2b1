#!/usr/bin/env python3
"""Headline benchmark: megapixels/s of JPEG target-size encode on MI355X.

Workload (BASELINE.json configs[1]): synthetic 4K frames
(3840x2160, 50% "smooth", 50% "noise"), -t 1 MiB, fixed q = 0.25, i.e. the
reference's cache-hit path tryCachedParams with LearnedParams(0.25, 1.0)
(ImageCompressionJpg.java:82-89, :216-238), falling back to the full
scale-loop + binary search when the cached quality does not fit (every
noise frame does: 2.0 MB at q=0.25).  Frames and output buffers are resident
in HBM when the timed region starts.  A step = one pass over the batch.
MP counted once per image (decoded W x H).

Multi-GPU: one process per GPU (torchrun); each rank owns its own frames
(file-list sharding, no data-path collective) -> weak scaling.  The barrier
and the max-over-ranks reduction of the step time are the only collectives,
on a gloo (host) process group: no RCCL anywhere on the path.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import icx  # noqa: E402
from icx.pipeline import host_cores  # noqa: E402,F401  (the CPU baseline's thread count)

W, H = 3840, 2160
TARGET = 1 << 20
Q0 = 0.25
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s
# Algorithmic bytes of each kernel.  fdct and huff move
# content-dependent amounts (candidate lists), so the library counts them per
# launch ("<kernel>.bytes" profile entries): fdct = pixels read + lists, list
# offsets and lengths written; huff = per trial, every block's padded list +
# offset + length read, and the trial's bitstream (>= bits / 8) + per-chunk
# bit counts and 0xFF bins written.  resize: a fixed 6 B per destination pixel.
ALGO_BYTES_FIXED = {"resize": 6.0}
UNIT_NAME = {"fdct": "pixel", "huff": "scan block (per trial)", "resize": "destination pixel"}


def algo_bytes(codec, kernel, stat):
    """Algorithmic bytes of `kernel` over the profiled launches."""
    if kernel in ALGO_BYTES_FIXED:
        return ALGO_BYTES_FIXED[kernel] * stat["units"]
    return codec.profile_query(kernel + ".bytes")["units"]


def make_frames(n, seed0, device):
    """Deterministic synthetic 4K BGR frames generated on the GPU."""
    frames = []
    g = torch.Generator(device=device)
    y = torch.arange(H, device=device, dtype=torch.float32)[:, None]
    x = torch.arange(W, device=device, dtype=torch.float32)[None, :]
    for i in range(n):
        g.manual_seed(seed0 + i)
        if i % 2 == 0:  # smooth: sinusoids + gaussian sigma 16
            fx, fy, ph = (torch.rand(3, generator=g, device=device) * 0.018 + 0.002).tolist()
            r = 127 + 100 * torch.sin(x * fx * 10 + ph).expand(H, W)
            gg = 127 + 100 * torch.sin(y * fy * 10 + 2 * ph).expand(H, W)
            b = 127 + 100 * torch.sin((x + y) * fx * 5)
            bgr = torch.stack([b, gg, r], -1)
            bgr += torch.randn(H, W, 3, generator=g, device=device) * 16
            frames.append(bgr.round_().clamp_(0, 255).to(torch.uint8).contiguous())
        else:  # noise: uniform u8
            frames.append(torch.randint(0, 256, (H, W, 3), generator=g, device=device, dtype=torch.uint8))
    return frames


def pmc_traffic(kernel, units_per_launch):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_summary.json, scripts/gpu_pmc.sh): measured bytes per unit
    of work x this run's units per launch.  None when no summary exists."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        per_unit = pmc_bytes_per_unit(json.load(open(path)))[kernel]
    except (KeyError, ValueError, TypeError):
        return None
    return int(per_unit * units_per_launch)


PMC_SHORT = {"k_fdct_color": "fdct", "k_fdct_gray": "fdct", "k_huff": "huff", "k_scan": "scan",
             "k_ffscan": "ffscan", "k_stuff": "stuff", "k_resize": "resize"}


def pmc_bytes_per_unit(summary):
    """bench kernel name -> HBM bytes per unit, from scripts/pmc_summary.py's
    file form ({"bytes_per_unit": {...}}) or, should a kernel-keyed form
    ({"icx::k_huff": {"hbm_bytes_per_unit": ...}}) be committed, from that."""
    if "bytes_per_unit" in summary:
        return summary["bytes_per_unit"]
    return {PMC_SHORT[k.split("::")[-1].split("<")[0]]: v["hbm_bytes_per_unit"]
            for k, v in summary.items() if isinstance(v, dict) and "hbm_bytes_per_unit" in v
            and k.split("::")[-1].split("<")[0] in PMC_SHORT}




VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions/s: 256 CUs x 4 SIMD-32, 2 cycles each (MI355X_MICROARCH.md)
SALU_PEAK = 256 * 2.4e9          # scalar instructions/s: one scalar unit per CU


def issue_rates(kernel, units_per_launch, launch_s):
    """Instruction-issue rates of the dominant kernel from the committed SQ
    counter summary (profiles/sq_issue_summary.json, scripts/sq_issue.py):
    instructions per unit of work x this run's units per launch / launch time,
    against the chip's issue peaks.  None when no summary exists."""
    path = os.path.join(ROOT, "profiles", "sq_issue_summary.json")
    if not os.path.exists(path):
        return None
    try:
        pu = json.load(open(path))["per_unit"][kernel]
    except (KeyError, ValueError):
        return None
    valu = pu["SQ_INSTS_VALU"] * units_per_launch / launch_s
    salu = pu["SQ_INSTS_SALU"] * units_per_launch / launch_s
    return {"valu_per_s": round(valu / 1e9, 1), "valu_peak_per_s": round(VALU_PEAK / 1e9, 1),
            "valu_frac": round(valu / VALU_PEAK, 4), "salu_per_s": round(salu / 1e9, 1),
            "salu_peak_per_s": round(SALU_PEAK / 1e9, 1), "salu_frac": round(salu / SALU_PEAK, 4),
            "unit": "G wave-instructions/s"}


def cpu_baseline(frames, n_sample, threads, cores_how="", distinct=320):
    """Oracle (scalar C restatement, test infrastructure) on host cores: one
    image per pool task, as the reference's thread pool of
    availableProcessors() threads runs processImage (CompressionBatch.java:
    64-88).  At most `distinct` frames are copied to host memory (25 MB each);
    a larger sample (many cores) cycles over them."""
    from tests.oracle_ffi import Oracle
    o = Oracle()
    host = [f.cpu().numpy() for f in frames[:min(n_sample, distinct)]]
    sample = [host[i % len(host)] for i in range(n_sample)]
    t0 = time.perf_counter()
    enc, sizes, qs, scales = o.fit_batch(sample, TARGET, Q0, cached=(Q0, 1.0), threads=threads)
    dt = time.perf_counter() - t0
    mp = n_sample * W * H / 1e6
    return {"value": round(mp / dt, 3), "unit": "MP/s", "cores": threads, "kind": "port",
            "sample": f"{n_sample} of the 4K frames ({len(host)} distinct: {(len(host) + 1) // 2} smooth, "
                      f"{len(host) // 2} noise), oracle compressJpgWithTargetSize with cache (0.25, 1.0), -t 1MiB, "
                      f"{threads} threads = every host core this process may use ({cores_how}), "
                      f"{enc} full encodes, {dt:.2f} s wall"}, sizes


def ranks_max(dist, dt):
    """Max of a per-rank time over the host (gloo) group; dt itself at N = 1."""
    if not dist:
        return dt
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def rank_sync(dist):
    """Device drained, then every rank at the same point (bracket of a timed region)."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist:
        dist.barrier()


def e2e_leg(codec, dev, frames, n_frames, steps, cpu_sample=0, threads=16, small=200, dist=None, world=1):
    """Secondary measurement: the whole per-image hot loop of processImage on
    the device — q95 4:2:0 4K JPEG files resident in HBM -> decode (A11,
    decodeImageWithSubsampling) -> compressJpgWithTargetSize at -t 1 MiB with
    the cached q = 0.25 (A2-A10) -> output bytes in HBM.  Sources: n_frames
    DISTINCT files (7.8 GB for configs[1]'s 1000 frames, 1.5 GB for 200: far
    past the 256 MiB Infinity Cache, so no source is re-read from it), made
    from the headline's frames by this library's own encoder at quality 0.95 -
    JPEGQTable scaling by 0.1, the same tables, 4:2:0 sampling and Annex-K
    Huffman codes as libjpeg's q95.  The same loop over the first `small`
    sources is reported beside it (`at_small_batch`): the decoder's
    relaxation tail (the last few re-walk launches, single waves) is a fixed
    latency per call, so a smaller call runs at a lower rate."""
    line = _e2e_run(codec, dev, frames, n_frames, steps, dist, world)
    if small and small < n_frames:
        line["at_small_batch"] = {k: v for k, v in _e2e_run(codec, dev, frames, small, steps, dist, world).items()
                                  if k in ("value", "frames", "ms_per_step", "decode_ms_per_step",
                                           "encode_ms_per_step", "decode_mp_s", "decode_roofline")}
    if cpu_sample:
        srcs = _e2e_sources(codec, dev, frames, min(16, n_frames))[0]
        line["cpu_baseline"] = e2e_cpu_baseline([s.cpu().numpy().tobytes() for s in srcs], cpu_sample, threads)
    return line


def _e2e_sources(codec, dev, frames, n_frames):
    """q95 JPEG sources of the first n_frames frames, in HBM (see e2e_leg)."""
    srcs_buf = torch.empty((n_frames, 12 << 20), dtype=torch.uint8, device=dev)
    enc = codec.prepare(frames[:n_frames], 12 << 20, 0.95, cached=[icx.LearnedParams(0.95, 1.0)] * n_frames,
                        outputs=[srcs_buf[i] for i in range(n_frames)])
    enc.run()
    lens = [r["out_len"] for r in enc.results()]
    assert all(r["success"] and r["cache_hit"] for r in enc.results()), "source encode"
    srcs = [srcs_buf[i, :lens[i]] for i in range(n_frames)]
    return srcs, lens


def _e2e_run(codec, dev, frames, n_frames, steps, dist=None, world=1):
    srcs, lens = _e2e_sources(codec, dev, frames, n_frames)
    px = [torch.empty((H, W, 3), dtype=torch.uint8, device=dev) for _ in range(n_frames)]
    outs = torch.empty((n_frames, TARGET + 1), dtype=torch.uint8, device=dev)
    dec = codec.prepare_decode(srcs, px, subsampling=0)
    fit = codec.prepare(px, TARGET, Q0, cached=[icx.LearnedParams(Q0, 1.0)] * n_frames,
                        outputs=[outs[i] for i in range(n_frames)])
    assert all(s == 0 for s in dec.run())
    fit.run()
    assert all(r["success"] and r["status"] == 0 for r in fit.results())
    rank_sync(dist)
    td = tf = 0.0
    t_all = time.perf_counter()
    for _ in range(steps):
        t0 = time.perf_counter()
        dec.run()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        fit.run()
        torch.cuda.synchronize()
        td += t1 - t0
        tf += time.perf_counter() - t1
    rank_sync(dist)
    # whole job: every rank's frames over the slowest rank's time (the
    # decode / encode split below is this rank's own)
    t_all = ranks_max(dist, time.perf_counter() - t_all)
    mp = n_frames * W * H / 1e6
    line = {"metric": "megapixels/sec 4K q95 JPEG bytes in HBM -> device decode -> target-size encode (-t 1MiB, "
                      "q=0.25 cached)",
            "value": round(world * mp * steps / t_all, 1), "unit": "MP/s", "frames": n_frames, "steps": steps,
            "distinct_sources": n_frames, "n_gpus": world, "frames_per_gpu": n_frames,
            "ms_per_step": round((td + tf) / steps * 1e3, 3), "decode_ms_per_step": round(td / steps * 1e3, 3),
            "encode_ms_per_step": round(tf / steps * 1e3, 3),
            "decode_mp_s": round(mp * steps / td, 1),
            "mean_src_jpeg_bytes": int(np.mean(lens))}
    # the decode against HBM on SURVEY §8(d)'s decode bytes: the compressed
    # file read + the 3 B/px BGR frame written (the walks are latency-bound,
    # DESIGN.md §5.5, so this fraction stays small)
    dbytes = float(sum(lens)) + 3.0 * W * H * n_frames
    gbps = dbytes * steps / td / 1e9
    line["decode_roofline"] = {"bound": "hbm", "achieved": round(gbps, 1), "peak": 8000.0, "unit": "GB/s",
                               "frac": round(gbps / 8000.0, 4), "bytes_per_call": int(dbytes)}
    return line


def e2e_concurrent(local, codec, dev, frames, n_frames, steps, contexts=3, dist=None, world=1):
    """The e2e loop as the CLI runs it on one GPU: `contexts` libicx contexts
    (its --workers-per-device), each over its share of the same n_frames
    distinct sources, one host thread each, every step = decode + fit of every
    share.  One context's latency-bound relaxation launches (few waves)
    overlap another's bulk kernels.  Whole job: all frames over the wall time
    of the slowest thread (max over ranks)."""
    import threading
    srcs, lens = _e2e_sources(codec, dev, frames, n_frames)
    codecs = [icx.Codec(local) for _ in range(contexts)]
    try:
        jobs = []
        for k, c in enumerate(codecs):
            idx = list(range(k, n_frames, contexts))
            px = [torch.empty((H, W, 3), dtype=torch.uint8, device=dev) for _ in idx]
            outs = torch.empty((len(idx), TARGET + 1), dtype=torch.uint8, device=dev)
            dec = c.prepare_decode([srcs[i] for i in idx], px, subsampling=0)
            fit = c.prepare(px, TARGET, Q0, cached=[icx.LearnedParams(Q0, 1.0)] * len(idx),
                            outputs=[outs[i] for i in range(len(idx))])
            assert all(st == 0 for st in dec.run())
            fit.run()
            assert all(r["success"] and r["status"] == 0 for r in fit.results())
            jobs.append((dec, fit, px, outs))
        rank_sync(dist)
        go = threading.Barrier(contexts + 1)
        err = []

        def work(dec, fit):
            go.wait()
            try:
                for _ in range(steps):
                    dec.run()  # both calls return once their kernels are done
                    fit.run()
            except BaseException as e:  # re-raised below
                err.append(e)

        ts = [threading.Thread(target=work, args=(j[0], j[1])) for j in jobs]
        for t in ts:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in ts:
            t.join()
        if err:
            raise err[0]
        rank_sync(dist)
        dt = ranks_max(dist, time.perf_counter() - t0)
    finally:
        for c in codecs:
            c.close()
    mp = n_frames * W * H / 1e6
    return {"value": round(world * mp * steps / dt, 1), "unit": "MP/s", "contexts": contexts, "frames": n_frames,
            "steps": steps, "ms_per_step": round(dt / steps * 1e3, 3)}


def link_rates(dev, nbytes=1 << 30, reps=5):
    """PCIe link rates of this box: one pinned host buffer <-> HBM, GB/s."""
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    rates = {}
    for name, (dst, src) in (("h2d", (d, h)), ("d2h", (h, d))):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        rates[name] = nbytes * reps / (time.perf_counter() - t0) / 1e9
    return rates


def host_frames(frames, n):
    """The first n frames copied to pinned host memory (the host-fed legs)."""
    return [f.cpu().pin_memory() for f in frames[:n]]


def _timed_host_batch(b, steps, warmup, dist):
    """Warm-up, then `steps` runs of a prepared host-buffer batch bracketed by
    barriers; (per-step seconds, max over ranks), results."""
    for _ in range(max(1, warmup)):
        b.run()
    res = b.results()
    assert all(r["success"] and r["status"] == 0 for r in res), "host-fed leg: frames failed"
    rank_sync(dist)
    t0 = time.perf_counter()
    for _ in range(steps):
        b.run()
    rank_sync(dist)
    return ranks_max(dist, time.perf_counter() - t0) / steps, res


def host_io_leg(codec, frames, hf, steps, warmup, cached, dist=None, world=1):
    """SURVEY §8(d)'s headline definition, PCIe included: decoded BGR frames
    in pinned host memory -> final JPEG bytes in pinned host memory.  The
    library uploads sub-batch s+1 and downloads s-1 on their own streams while
    s computes (icx_runtime.cpp run_batch, prefetch).  At N > 1 every rank
    runs it at once (one process per GPU, each over its own link, sharing the
    host's memory), timed between barriers, max over ranks."""
    dev = frames[0].device
    n = len(hf)
    link = link_rates(dev)
    outs = torch.empty((n, TARGET + 1), dtype=torch.uint8).pin_memory()
    b = codec.prepare(hf, TARGET, Q0, cached=cached[:n] if cached else None, outputs=[outs[i] for i in range(n)])
    dt, res = _timed_host_batch(b, steps, warmup, dist)
    up = sum(f.numel() for f in hf)
    down = sum(r["out_len"] for r in res)
    h2d = up / dt / 1e9
    return {"metric": "megapixels/sec JPEG encode, pinned host BGR in -> host JPEG bytes out (PCIe included)",
            "value": round(world * n * W * H / 1e6 / dt, 1), "unit": "MP/s", "n_gpus": world, "frames_per_gpu": n,
            "steps": steps, "ms_per_step": round(dt * 1e3, 3),
            "h2d_GBps_per_gpu": round(h2d, 2), "d2h_GBps_per_gpu": round(down / dt / 1e9, 2),
            "link_h2d_GBps": round(link["h2d"], 2), "link_d2h_GBps": round(link["d2h"], 2),
            "h2d_frac_of_link": round(h2d / link["h2d"], 4)}


def pool_leg(devices, hf, steps, warmup, cached, dist=None, world=1):
    """icx_pool_compress_jpg_batch over `devices` (one process driving a
    device list from one host: the JVM shape of CompressionBatch.java:64-88,
    the only multi-GPU mode that keeps one learned cache, :71).  The same
    pinned host frames as host_io, split by the pool into per-device shares
    (LPT by pixels) run on one host thread per device.  At N > 1 each rank
    runs its own pool (over its own devices) at once."""
    n = len(hf)
    pool = icx.Pool(devices)
    try:
        outs = torch.empty((n, TARGET + 1), dtype=torch.uint8).pin_memory()
        b = pool.prepare(hf, TARGET, Q0, cached=cached[:n] if cached else None,
                         outputs=[outs[i] for i in range(n)])
        dt, res = _timed_host_batch(b, steps, warmup, dist)
    finally:
        pool.close()
    return {"metric": "megapixels/sec JPEG encode through icx_pool (pinned host BGR in -> host JPEG bytes out)",
            "value": round(world * n * W * H / 1e6 / dt, 1), "unit": "MP/s", "devices_per_process": devices,
            "contexts": len(devices), "n_gpus": world, "frames_per_process": n, "steps": steps,
            "ms_per_step": round(dt * 1e3, 3)}


def e2e_cpu_baseline(srcs, n_sample, threads):
    """The same per-image loop on host cores with the oracle (test
    infrastructure): IJG-6b decode restatement + compressJpgWithTargetSize
    restatement, one image per thread task."""
    import concurrent.futures as cf
    from tests.oracle_ffi import Oracle
    o = Oracle()

    def one(i):
        rc, img = o.jpeg_decode(srcs[i % len(srcs)])
        assert rc == 0
        return o.fit(img, TARGET, Q0, cached=(Q0, 1.0))["success"]

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        ok = sum(ex.map(one, range(n_sample)))
    dt = time.perf_counter() - t0
    assert ok == n_sample
    return {"value": round(n_sample * W * H / 1e6 / dt, 3), "unit": "MP/s", "cores": threads, "kind": "port",
            "sample": f"{n_sample} of the q95 sources ({len(srcs)} distinct, half smooth, half noise): oracle "
                      f"decode + compressJpgWithTargetSize with cache (0.25, 1.0), {threads} threads, "
                      f"{dt:.2f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--images", type=int, default=1000, help="4K frames per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="4K frames for the CPU baseline (0 = 20 per host core, at least 320: ~10 s of wall time)")
    ap.add_argument("--e2e", type=int, default=1000,
                    help="frames (distinct sources) of the decode+encode leg (0 = skip; default: configs[1]'s "
                         "1000, with the first 200 timed beside them)")
    ap.add_argument("--e2e-contexts", type=int, default=0,
                    help="also run the e2e frames over this many libicx contexts at once, one host thread each "
                         "(the CLI's --workers-per-device; <= 1 = skip; 3 contexts x 333 frames measured 76.0 k "
                         "against 81.6 k MP/s serial: at large calls the contexts only compete)")
    ap.add_argument("--host-io-frames", type=int, default=-1,
                    help="frames per GPU of the PCIe-inclusive legs (host_io, pool; pinned host in/out; 0 = skip; "
                         "default: configs[1]'s 1000 at N = 1, max(200, 2000 / N) at N > 1 to bound the pinned "
                         "host memory of a node)")
    ap.add_argument("--pool-devices", default="",
                    help="devices of the icx_pool leg, comma-separated (default: this rank's GPU twice: two "
                         "contexts, the JVM-shaped host on one GPU; 'none' = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile", type=int, default=1, help="HIP-event per-kernel timing in the timed region")
    ap.add_argument("--target", type=int, default=TARGET, help="-t bytes (default 1 MiB)")
    ap.add_argument("--no-cache", action="store_true", help="no cached LearnedParams: full binary search")
    ap.add_argument("--host-io", action="store_true",
                    help="frames and output buffers in pinned host memory (PCIe-inclusive rate; not the headline)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # host group: no device exchange on the path (no RCCL)

    frames = make_frames(args.images, 1000003 * rank, dev)
    if args.host_io:
        frames = [f.cpu().pin_memory() for f in frames]
        outs = torch.empty((args.images, min(args.target, 1 << 24) + 1), dtype=torch.uint8).pin_memory()
    else:
        outs = torch.empty((args.images, min(args.target, 1 << 24) + 1), dtype=torch.uint8, device=dev)
    codec = icx.Codec(local)
    cached = None if args.no_cache else [icx.LearnedParams(Q0, 1.0)] * args.images
    batch = codec.prepare(frames, args.target, Q0, cached=cached, outputs=[outs[i] for i in range(args.images)])
    torch.cuda.synchronize()

    def validate():
        res = batch.results()
        ok = sum(r["success"] and r["status"] == 0 for r in res)
        if ok != args.images:
            from collections import Counter
            raise SystemExit(f"{args.images - ok} frames failed: "
                             f"{Counter((r['success'], r['status']) for r in res)} err={codec.last_error()}")

    for _ in range(args.warmup):
        batch.run()
    if args.warmup:
        validate()

    codec.profile(bool(args.profile))
    codec.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    codec.profile(False)
    validate()
    if dist:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()

    mp_step = world * args.images * W * H / 1e6
    value = mp_step * args.steps / dt
    kstats = {k: codec.profile_query(k) for k in ("fdct", "count", "huff", "scan", "ffscan",
                                                  "stuff", "resize")}
    kstats = {k: v for k, v in kstats.items() if v["launches"]}
    sb = codec.profile_query("subbatch")
    roof = None
    bytes_of = {k: algo_bytes(codec, k, v) for k, v in kstats.items() if k in UNIT_NAME and v["units"]}
    if bytes_of:
        dom = max(bytes_of, key=lambda k: kstats[k]["ms"])
        ks = kstats[dom]
        achieved = bytes_of[dom] / (ks["ms"] / 1e3) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(dom, ks["units"] / ks["launches"]),
                "issue": issue_rates(dom, ks["units"] / ks["launches"], ks["ms"] / ks["launches"] / 1e3),
                "avg_launch_ms": round(ks["ms"] / ks["launches"], 4),
                "algo_bytes_per_launch": int(bytes_of[dom] / ks["launches"]),
                "frac_basis": f"{UNIT_NAME[dom]}: the bytes the kernel must move (DESIGN.md §4)"}
        # SURVEY.md §8(d)'s per-unit bytes, beside the kernel's own: 128 B per
        # block-trial (64 int16 coefficients read) for k_huff, 6 B/px for k_fdct
        s8d = {"huff": 128.0, "fdct": 6.0}.get(dom)
        if s8d is not None:
            roof["frac_s8d"] = round(s8d * ks["units"] / (ks["ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
            roof["frac_s8d_basis"] = ("SURVEY.md 8(d): 128 B per scan block per trial (its coefficients read)"
                                      if dom == "huff" else "SURVEY.md 8(d): 6 B/px (BGR read + int16 coefficients)")
    # every kernel with an algorithmic-bytes model, against the HBM roofline
    # (the north star's >= 60 % target is for the DCT stage, k_fdct)
    stages = {k: {"achieved_GBps": round(b / (kstats[k]["ms"] / 1e3) / 1e9, 1),
                  "frac": round(b / (kstats[k]["ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                  "avg_launch_ms": round(kstats[k]["ms"] / kstats[k]["launches"], 4),
                  "algo_bytes_per_unit": round(b / kstats[k]["units"], 2), "unit": UNIT_NAME[k]}
              for k, b in bytes_of.items()}
    if "fdct" in stages:  # launch-size independent forms (sub-batch sizes follow the HBM budget)
        px, ms = kstats["fdct"]["units"], kstats["fdct"]["ms"]
        stages["fdct"]["ms_per_333_frames"] = round(ms / px * 333.3 * W * H, 4)
        stages["fdct"]["frac_at_6B_per_px"] = round(6 * px / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    res = batch.results()
    line = {
        "metric": ("megapixels/sec JPEG encode (4K, -t 1MiB, q=0.25 cached), frames in HBM -> JPEG bytes in HBM"
                   if not args.host_io else
                   "megapixels/sec JPEG encode (4K, -t 1MiB, q=0.25 cached), pinned host BGR -> host JPEG bytes"),
        "definition": ("value: decoded 4K BGR frames already resident in HBM when the timed region starts, every "
                       "trial and the final bytes on the device (the task's bench contract); BASELINE.md's "
                       "'encode path' (host BGR in -> host JPEG bytes out, PCIe included) is the host_io leg"
                       if not args.host_io else
                       "value: BASELINE.md's 'encode path', pinned host BGR in -> host JPEG bytes out, PCIe included"),
        "value": round(value, 2), "unit": "MP/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8/int16",
        "data": ("synthetic (seeded smooth+noise 4K frames), pinned host memory in and out: PCIe-inclusive"
                 if args.host_io else "synthetic (seeded smooth+noise 4K frames generated on device)"),
        "config": {"workload": "BASELINE configs[1]: 4K (3840x2160) JPG, -t 1MB, fixed q=0.25 "
                               "(cache-hit path, search fallback)",
                   "images_per_gpu": args.images, "global_images": world * args.images,
                   "target_bytes": TARGET, "quality": Q0, "parallelism": f"file-list shard x{world}",
                   "encodes_per_image": round(sum(r["encodes"] for r in res) / len(res), 3),
                   "mean_out_bytes": int(np.mean([r["out_len"] for r in res])),
                   "subbatches_per_step": round(sb["launches"] / args.steps, 2),
                   "workspace_mb_per_subbatch": int(sb["units"] / max(1, sb["launches"]))},
        "roofline": roof,
        "stages": stages,
        "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3), "units": v["units"],
                        **({"algo_bytes": int(bytes_of[k])} if k in bytes_of else {})}
                    for k, v in kstats.items()},
    }
    # the host-fed legs and e2e run on every rank (each over its own link and
    # GPU, together), timed between barriers, max over ranks
    n_host = args.host_io_frames if args.host_io_frames >= 0 else (1000 if world == 1 else max(200, 2000 // world))
    n_host = min(n_host, args.images)
    if n_host and not args.host_io:
        batch = None
        hf = host_frames(frames, n_host)
        line["host_io"] = host_io_leg(codec, frames, hf, args.steps, args.warmup, cached, dist, world)
        if args.pool_devices != "none":
            devs = [int(d) for d in args.pool_devices.split(",")] if args.pool_devices else [local, local]
            line["pool"] = pool_leg(devs, hf, args.steps, args.warmup, cached, dist, world)
            line["pool"]["vs_host_io"] = round(line["pool"]["value"] / line["host_io"]["value"], 3)
        hf = None
    cores, cores_how = host_cores()
    if args.e2e and not args.host_io:
        batch = None
        line["e2e"] = e2e_leg(codec, dev, frames, min(args.e2e, args.images), args.steps,
                              cpu_sample=0 if (args.no_cpu_baseline or rank) else max(64, 4 * cores), threads=cores,
                              dist=dist, world=world)
        if args.e2e_contexts > 1:
            line["e2e"]["concurrent"] = e2e_concurrent(local, codec, dev, frames, min(args.e2e, args.images),
                                                       args.steps, args.e2e_contexts, dist, world)
    if rank == 0 and not args.no_cpu_baseline:
        # rank 0 only, after the timed region (the other ranks wait at the
        # final barrier); at N > 1 the line still carries it
        cb, _ = cpu_baseline(frames, args.cpu_sample or max(320, 20 * cores), cores, cores_how)
        line["cpu_baseline"] = cb
        line["speedup_vs_cpu"] = round(value / cb["value"], 1)
    if rank == 0:
        print(json.dumps(line), flush=True)
    codec.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
