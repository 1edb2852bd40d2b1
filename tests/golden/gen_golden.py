#!/usr/bin/env python3
"""Generate the committed golden fixtures for the JPEG encode path.

Test infrastructure only.  Run once in the build container; the outputs in this
directory are committed and the GPU box never runs this script.

Independent encoder used as the pin: libjpeg-turbo 3.1.4 (bundled in Pillow
12.2).  The reference (PolloChang/image-compression) encodes through the JDK's
javax.imageio JPEG writer, i.e. IJG libjpeg 6b (ImageCompressionJpg.java:136-147).
No JDK exists here, so the arithmetic is pinned on a libjpeg of
the same 6b lineage driven with the exact parameters the JDK writer uses:

  * quantisation tables from JPEG.convertToLinearQuality(q) and
    JPEGQTable.K1Luminance/K2Chrominance.getScaledInstance(lin, true)
    (reached from ImageCompressionJpg.java:140-143; restated below in float32),
  * 4:2:0 (Y 2x2, Cb/Cr 1x1), JDCT_ISLOW, standard Annex-K Huffman tables,
    no restart interval, baseline SOF0, JFIF APP0.

The only byte the JDK writes differently is the JFIF minor version (JDK 1.02,
libjpeg 1.01, file offset 12); every length is identical, so sizes and the
entropy-coded segment are pinned bit for bit.

Outputs (all small):
  inputs.npz          u8 BGR images (H, W, 3) and one grey image
  jpeg_golden.npz     Pillow/turbo JPEG bytes per (image, quality)
  golden.json         sizes, sha256, quality tables, binary-search traces
"""
import hashlib
import io
import json
import os

import numpy as np
from PIL import Image, features

HERE = os.path.dirname(os.path.abspath(__file__))

# Annex K.1 / K.2 base tables, natural order (JPEGQTable.K1Luminance/K2Chrominance).
K1 = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
      14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
      18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
      49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99]
K2 = [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
      24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32

F32 = np.float32


def linear_quality(q):
    """JPEG.convertToLinearQuality, float32 semantics."""
    q = F32(q)
    if q <= F32(0.0):
        q = F32(0.01)
    if q > F32(1.0):
        q = F32(1.0)
    if q < F32(0.5):
        return F32(F32(0.5) / q)
    return F32(F32(2.0) - F32(q * F32(2.0)))


def scaled_table(base, lin):
    """JPEGQTable.getScaledInstance(lin, forceBaseline=true)."""
    out = []
    for v in base:
        sv = int(F32(F32(F32(v) * lin) + F32(0.5)))
        out.append(min(255, max(1, sv)))
    return out


def jdk_tables(q):
    lin = linear_quality(q)
    return scaled_table(K1, lin), scaled_table(K2, lin)


def encode(img_bgr, q):
    """One encode at quality q with JDK tables via libjpeg-turbo."""
    lum, chrom = jdk_tables(q)
    buf = io.BytesIO()
    if img_bgr.ndim == 2:
        Image.fromarray(img_bgr, "L").save(buf, "JPEG", qtables=[lum], optimize=False)
    else:
        rgb = np.ascontiguousarray(img_bgr[:, :, ::-1])
        Image.fromarray(rgb, "RGB").save(buf, "JPEG", qtables=[lum, chrom],
                                         subsampling=2, optimize=False)
    return buf.getvalue()


def find_best_quality_trace(img, target, q0):
    """ImageCompressionJpg.findBestQualityByBinarySearch (:158-200), float32."""
    lo, hi, best = F32(0.0), F32(q0), F32(-1.0)
    trace = []
    for _ in range(8):
        mid = F32(F32(lo + hi) / F32(2.0))
        if mid < F32(0.01):
            break
        size = len(encode(img, float(mid)))
        fits = size <= target
        trace.append([float(mid), size, fits])
        if fits:
            best, lo = mid, mid
        else:
            hi = mid
        if F32(hi - lo) < F32(0.01):
            break
    return float(best), trace


def smooth(h, w, seed):
    rng = np.random.default_rng(seed)
    fx, fy, ph = rng.uniform(0.002, 0.02, 3)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    r = 127 + 100 * np.sin(x * fx * 10 + ph)
    g = 127 + 100 * np.sin(y * fy * 10 + 2 * ph)
    b = 127 + 100 * np.sin((x + y) * fx * 5)
    rgb = np.stack([r, g, b], -1) + rng.normal(0, 16, (h, w, 3))
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)[:, :, ::-1].copy()


def noise(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def main():
    assert features.check("libjpeg_turbo"), "Pillow must be built on libjpeg-turbo"
    imgs = {
        "smooth_64x48": smooth(48, 64, 1),
        "noise_16x16": noise(16, 16, 2),
        "smooth_200x136": smooth(136, 200, 3),   # Y dummy column + dummy block row
        "noise_1001x67": noise(67, 1001, 4),     # odd width/height, bottom dummy row
        "smooth_17x17": smooth(17, 17, 5),       # W%16==1, H%16==1
        "noise_7x9": noise(9, 7, 6),             # smaller than one MCU
        "smooth_1x1": smooth(1, 1, 7),
        "smooth_24x40": smooth(40, 24, 8),       # H even, not a multiple of 16
        "noise_120x90": noise(90, 120, 9),       # H%16 = 10: chroma row replication
        "solid_48x32": np.full((32, 48, 3), (30, 60, 200), np.uint8),
        "grey_37x29": smooth(29, 37, 10)[:, :, 1].copy(),
    }
    qualities = [0.01, 0.03125, 0.0625, 0.125, 0.1875, 0.25, 0.3, 0.5, 0.75, 0.95, 1.0]
    jpegs, meta = {}, {"encoder": "libjpeg-turbo " + features.version("libjpeg_turbo"),
                       "jfif_version_offset": 12, "images": {}, "tables": {}}
    for q in qualities:
        lum, chrom = jdk_tables(q)
        meta["tables"][repr(q)] = {"lum": lum, "chrom": chrom}
    for name, img in imgs.items():
        entry = {"shape": list(img.shape), "encodes": {}, "searches": []}
        for q in qualities:
            data = encode(img, q)
            key = f"{name}@{q!r}"
            jpegs[key] = np.frombuffer(data, np.uint8)
            entry["encodes"][repr(q)] = {"size": len(data),
                                         "sha256": hashlib.sha256(data).hexdigest()}
        # binary-search traces at targets that straddle the encoded sizes
        sizes = sorted(v["size"] for v in entry["encodes"].values())
        for target in sorted({sizes[0] - 1, sizes[1], sizes[len(sizes) // 2], sizes[-2] + 3}):
            for q0 in (0.25, 1.0, 0.3):
                best, trace = find_best_quality_trace(img, target, q0)
                entry["searches"].append({"target": int(target), "q0": q0,
                                          "best": best, "trace": trace})
        meta["images"][name] = entry
    np.savez_compressed(os.path.join(HERE, "inputs.npz"), **imgs)
    np.savez_compressed(os.path.join(HERE, "jpeg_golden.npz"), **jpegs)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
