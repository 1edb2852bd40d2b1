#!/usr/bin/env python3
"""How many findBestQualityByBinarySearch / tryCachedParams decisions the JPEG
table marker layout can flip (SURVEY.md §7 hard part 2).

The reference compares the WHOLE file size with -t (`bos.size()`,
ImageCompressionJpg.java:176 and :228).  libjpeg writes one DQT / DHT segment
per table (623-B colour header); if the JDK grouped its tables into one DQT and
one DHT segment the header would be 607 B, every trial 16 B smaller, and a
decision flips exactly when a trial's size lands in (target, target + 16] under
the per-table layout.  After the first flip the two searches diverge, so the
outcome (best q, scale, bytes) differs for exactly the images with one.

  --cpu : the oracle over the golden searches (tests/golden, whose targets sit
          next to trial sizes on purpose) and configs[0] (C1: a 1920x1080
          smooth frame decoded from its q95 JPEG, -t 512 KiB, q 0.25)
  --gpu : libicx on the device, both layouts, over the headline frames
          (bench.py make_frames: configs[1], cached q 0.25, -t 1 MiB) and the
          configs[2] search (C3: no cache, full binary search); per-trial sizes
          from icx_find_best_quality, outcomes from whole-batch fits in both
          layouts (the two counts must agree)
Writes one JSON object per part to stdout.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-compression_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

DELTA = 16  # 623 - 607


def classify(trials, target):
    """(flipped, min margin) of one trace [(q, size_separate), ...]."""
    flipped = any(target < s <= target + DELTA for _, s in trials)
    margin = min((abs(s - target) for _, s in trials), default=None)
    return flipped, margin


def cpu_part():
    from tests.oracle_ffi import Oracle, load_golden, smooth
    o = Oracle()
    meta, inputs, _ = load_golden()
    n = flips = out_diff = trials_total = 0
    for name, img in inputs.items():
        for s in meta["images"][name]["searches"]:
            o.set_table_layout(False)
            best_a, tr_a = o.find_best_quality(img, s["target"], s["q0"])
            o.set_table_layout(True)
            best_b, tr_b = o.find_best_quality(img, s["target"], s["q0"])
            o.set_table_layout(False)
            delta = DELTA if img.ndim == 3 else 4
            f = any(s["target"] < sz <= s["target"] + delta for _, sz in tr_a)
            n += 1
            trials_total += len(tr_a)
            flips += f
            out_diff += best_a != best_b
            assert f == (best_a != best_b or [q for q, _ in tr_a] != [q for q, _ in tr_b]), name
    golden = {"searches": n, "trials": trials_total, "searches_with_a_flipped_decision": flips,
              "searches_whose_best_quality_differs": out_diff}
    # C1: a 1080p smooth frame read back from its q95 JPEG, -t 512 KiB, q 0.25
    img = smooth(1080, 1920, 7)
    rc, dec = o.jpeg_decode(o.encode(img, 0.95))
    assert rc == 0
    res = {}
    for grouped in (False, True):
        o.set_table_layout(grouped)
        best, tr = o.find_best_quality(dec, 524288, 0.25)
        res[grouped] = (best, tr)
    o.set_table_layout(False)
    fl, mg = classify(res[False][1], 524288)
    c1 = {"trials": [[q, s] for q, s in res[False][1]], "flipped": fl, "min_margin_bytes": mg,
          "best_separate": res[False][0], "best_grouped": res[True][0]}
    return {"part": "cpu (oracle)", "golden": golden, "c1": c1}


def gpu_part(n_head, n_c3):
    import torch

    import icx
    from icx import _native as N
    from bench import make_frames
    dev = torch.device("cuda", 0)
    codec = icx.Codec(0)
    out = {"part": "gpu (libicx)"}
    T = 1 << 20
    for label, n, cached in (("headline_configs1_cached_q0.25", n_head, True), ("c3_search_no_cache", n_c3, False)):
        frames = make_frames(n, 0 if cached else 777, dev)
        flips, margins, probe_flips = 0, [], 0
        for f in frames:
            trials = []
            if cached:  # tryCachedParams: one encode at the cached q, kept if it fits
                s0 = len(codec.compress_jpg_to_stream(f, 0.25))
                trials.append((0.25, s0))
                if s0 <= T:
                    fl, mg = classify(trials, T)
                    flips += fl
                    probe_flips += fl
                    margins.append(mg)
                    continue
            tr = []
            codec.find_best_quality_by_binary_search(f, T, 0.25, trace=tr)
            trials += [(q, s) for q, s, _ in tr]
            fl, mg = classify(trials, T)
            flips += fl
            margins.append(mg)
        outcomes = {}
        for layout in (N.TABLES_SEPARATE, N.TABLES_GROUPED):
            codec.set_table_layout(layout)
            res = codec.fit(frames, T, 0.25, cached=[icx.LearnedParams(0.25, 1.0)] * n if cached else None)
            outcomes[layout] = [(r["success"], np.float32(r["learned"].quality) if r["success"] else None,
                                 r["learned"].scale if r["success"] else None, r["encodes"], r["out_len"]) for r in res]
        codec.set_table_layout(N.TABLES_SEPARATE)
        diff_q = sum(a[1] != b[1] or a[2] != b[2] or a[3] != b[3]
                     for a, b in zip(outcomes[N.TABLES_SEPARATE], outcomes[N.TABLES_GROUPED]))
        size_ok = all(a[4] - b[4] == DELTA for a, b in zip(outcomes[N.TABLES_SEPARATE], outcomes[N.TABLES_GROUPED])
                      if a[1] == b[1] and a[2] == b[2])
        m = np.array(margins)
        out[label] = {"frames": n, "decisions_flipped_images": int(flips), "cache_probe_flips": int(probe_flips),
                      "outcome_differs_images": int(diff_q), "same_outcome_files_differ_by_16B": bool(size_ok),
                      "min_margin_bytes": int(m.min()), "margin_p1_bytes": int(np.percentile(m, 1)),
                      "median_margin_bytes": int(np.median(m))}
    codec.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--c3-frames", type=int, default=200)
    a = ap.parse_args()
    if a.cpu:
        print(json.dumps(cpu_part()), flush=True)
    if a.gpu:
        print(json.dumps(gpu_part(a.frames, a.c3_frames)), flush=True)


if __name__ == "__main__":
    main()
