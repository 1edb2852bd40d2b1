#!/usr/bin/env python3
"""Timing-only driver: per-kernel HIP-event times of codec.fit on the bench
workload, no output validation (for the ICX_HUFF_EXP builds, whose output is
deliberately incomplete).  ICX_LIB selects the library build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import icx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
target = int(sys.argv[2]) if len(sys.argv) > 2 else bench.TARGET  # a huge target: one probe trial per frame
dev = torch.device("cuda:0")
kind = sys.argv[3] if len(sys.argv) > 3 else "mixed"  # mixed | smooth | noise
frames = bench.make_frames(n if kind == "mixed" else 2 * n, 1000, dev)
if kind != "mixed":
    frames = frames[0 if kind == "smooth" else 1::2]
codec = icx.Codec(0)
outs = [torch.empty(min(target, 1 << 25) + 1, dtype=torch.uint8, device=dev) for _ in range(n)]
cached = [icx.LearnedParams(bench.Q0, 1.0)] * n
codec.fit(frames, target, bench.Q0, cached=cached, outputs=outs)
torch.cuda.synchronize()
codec.profile(True)
codec.profile_reset()
for _ in range(2):
    codec.fit(frames, target, bench.Q0, cached=cached, outputs=outs)
torch.cuda.synchronize()
res = {k: codec.profile_query(k) for k in ("fdct", "huff", "scan", "ffscan", "stuff")}
stats = None
if os.environ.get("ICX_STATS"):  # ICX_HUFF_EXP=7 build: list statistics over all trials
    import ctypes
    lib = ctypes.CDLL(os.environ["ICX_LIB"])
    buf = (ctypes.c_ulonglong * 6)()
    lib.icx_debug_huff_stats(buf)
    ent, wave_slots, nz, blocks, srt, split = list(buf)
    stats = {"entries_per_block": ent / blocks, "wave_max_per_block": wave_slots / blocks,
             "lane_efficiency": ent / wave_slots, "coded_ac_per_block": nz / blocks, "block_trials": blocks,
             "lane_eff_sorted": ent / srt, "lane_eff_luma_chroma_split": ent / split}
print(json.dumps({"stats": stats, "lib": os.path.basename(os.environ.get("ICX_LIB", "libicx.so")), "images": n, "kind": kind,
                  "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3)} for k, v in res.items()}}))
