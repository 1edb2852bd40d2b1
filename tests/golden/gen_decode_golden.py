#!/usr/bin/env python3
"""Generate the committed golden fixtures for the JPEG decode row (A11).

Test infrastructure only.  Run once in the build container; the output
(decode_golden.npz, decode_golden.json) is committed and the GPU box never
runs this script.

The reference decodes through javax.imageio's JPEGImageReader, i.e. the JDK's
bundled IJG libjpeg 6b (ImageCompression.java:113-155): ISLOW IDCT, fancy
(triangle) upsampling, ycc_rgb_convert, then keeps pixels (x*s, y*s).  No JDK
exists here; the independent pin is libjpeg-turbo 3.1.4 (6b API
level, bundled in Pillow 12.2), whose decoder is of the same lineage
 for every sampling layout covered here.  4:4:0 (h1v2) is left
out on purpose: libjpeg-turbo upsamples it with a triangle filter where 6b
replicates rows, so it cannot pin the JDK there.

Inputs are synthetic (seeded), encoded by Pillow at several qualities,
chroma layouts and restart intervals, plus progressive (SOF2) files: the
oracle restates the baseline decoder only and refuses them ("unsupported"),
the device decoder reads them ("progressive": host entropy decode of every
scan, device IDCT and colour).  libjpeg-turbo applies no block smoothing to
these (every scan script Pillow writes refines AC 1..5 fully), so it pins the
JDK's final output pass for them as for baseline files.
"""
import io
import json
import os

import numpy as np
from PIL import Image, features

HERE = os.path.dirname(os.path.abspath(__file__))


def smooth(h, w, seed):
    rng = np.random.default_rng(seed)
    fx, fy, ph = rng.uniform(0.02, 0.2, 3)
    y = np.arange(h, dtype=np.float32)[:, None]
    x = np.arange(w, dtype=np.float32)[None, :]
    r = 127 + 100 * np.sin(x * fx + ph) + 0 * y
    g = 127 + 100 * np.sin(y * fy + 2 * ph) + 0 * x
    b = 127 + 100 * np.sin((x + y) * fx / 2)
    rgb = np.stack([r, g, b], -1) + rng.normal(0, 12, (h, w, 3)).astype(np.float32)
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)


def noise(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def encode(rgb, **kw):
    buf = io.BytesIO()
    mode = "L" if rgb.ndim == 2 else "RGB"
    Image.fromarray(rgb, mode).save(buf, "JPEG", **kw)
    return buf.getvalue()


def segments(data):
    """(marker, bytes) of the segments before the first SOS, then ('scan', rest)."""
    out, i = [], 2
    while True:
        m = data[i + 1]
        n = int.from_bytes(data[i + 2:i + 4], "big")
        out.append((m, data[i:i + 2 + n]))
        i += 2 + n
        if m == 0xDA:
            out.append(("scan", data[i:]))
            return out


def rewrite(data, app, ids):
    """data with its APP0/APP14 segments replaced by `app` (None: dropped) and
    the component ids of SOF and SOS set to `ids` (None: kept)."""
    parts = [b"\xff\xd8"] + ([app] if app else [])
    for m, seg in segments(data):
        if m in (0xE0, 0xEE):
            continue
        if ids is not None and m in (0xC0, 0xC2):
            seg = bytearray(seg)
            for c in range(seg[9]):
                seg[10 + 3 * c] = ids[c]
            seg = bytes(seg)
        if ids is not None and m == 0xDA:
            seg = bytearray(seg)
            for c in range(seg[4]):
                seg[5 + 2 * c] = ids[c]
            seg = bytes(seg)
        parts.append(seg)
    return b"".join(parts)


def adobe_app14(transform):
    body = b"Adobe" + bytes([0, 100, 0, 0, 0, 0, transform])
    return b"\xff\xee" + (len(body) + 2).to_bytes(2, "big") + body


JFIF_APP0 = b"\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
XMP_APP1 = b"\xff\xe1\x00\x23http://ns.adobe.com/xap/1.0/\x00<x/>"
COM = b"\xff\xfe\x00\x06note"


def decode_bgr(data):
    im = Image.open(io.BytesIO(data))
    im.load()
    a = np.asarray(im)
    if a.ndim == 3:
        a = a[:, :, ::-1]  # TYPE_3BYTE_BGR
    return np.ascontiguousarray(a)


def main():
    cases = []
    sizes = [(1, 1), (2, 2), (3, 5), (5, 3), (4, 6), (7, 9), (16, 16), (17, 33), (33, 17), (48, 64),
             (47, 61), (66, 130), (130, 250)]
    seed = 0
    for (h, w) in sizes:
        for sub in (2, 1, 0):
            for q in (50, 95):
                seed += 1
                img = smooth(h, w, seed) if seed % 3 else noise(h, w, seed)
                cases.append((f"c{h}x{w}_s{sub}_q{q}", img, dict(quality=q, subsampling=sub)))
        seed += 1
        g = smooth(h, w, seed)[:, :, 1]
        cases.append((f"g{h}x{w}_q90", g, dict(quality=90)))
    # restart intervals (DRI), including one MCU per interval
    for (h, w), rb in [((48, 64), 1), ((66, 130), 3), ((130, 250), 7), ((17, 33), 2)]:
        seed += 1
        cases.append((f"rst{rb}_{h}x{w}", smooth(h, w, seed), dict(quality=85, subsampling=2,
                                                                    restart_marker_blocks=rb)))
        seed += 1
        cases.append((f"rst{rb}_{h}x{w}_444", noise(h, w, seed), dict(quality=75, subsampling=0,
                                                                       restart_marker_blocks=rb)))
    seed += 1
    cases.append(("rstrows_130x250", smooth(130, 250, seed), dict(quality=90, subsampling=2,
                                                                   restart_marker_rows=1)))
    seed += 1
    cases.append(("grey_rst_66x130", smooth(66, 130, seed)[:, :, 0], dict(quality=70,
                                                                        restart_marker_blocks=5)))
    # extreme qualities: q=100 (all-ones tables, long AC codes), q=1
    seed += 1
    cases.append(("q100_noise_40x72", noise(40, 72, seed), dict(quality=100, subsampling=2)))
    seed += 1
    cases.append(("q1_smooth_40x72", smooth(40, 72, seed), dict(quality=1, subsampling=2)))

    jpegs, expect, meta = {}, {}, {"libjpeg_turbo": features.version("libjpeg_turbo"),
                                    "pillow": Image.__version__, "cases": {}}
    for name, img, kw in cases:
        data = encode(img, **kw)
        out = decode_bgr(data)
        jpegs[name] = np.frombuffer(data, np.uint8)
        expect[name] = out
        meta["cases"][name] = {"w": int(out.shape[1]), "h": int(out.shape[0]),
                               "ncomp": 1 if out.ndim == 2 else 3, "params": kw, "bytes": len(data)}
    # progressive: refused by the baseline oracle (status 5), decoded by the device path
    seed += 1
    prog = encode(smooth(32, 48, seed), quality=80, progressive=True)
    jpegs["progressive_32x48"] = np.frombuffer(prog, np.uint8)
    expect["progressive_32x48"] = decode_bgr(prog)
    meta["cases"]["progressive_32x48"] = {"w": 48, "h": 32, "ncomp": 3, "unsupported": True, "progressive": True,
                                          "params": {"progressive": True}, "bytes": len(prog)}
    pcases = [("prog_c130x250_s2_q95", smooth(130, 250, 501), dict(quality=95, subsampling=2)),
              ("prog_c66x130_s1_q50", noise(66, 130, 502), dict(quality=50, subsampling=1)),
              ("prog_c47x61_s0_q90", smooth(47, 61, 503), dict(quality=90, subsampling=0)),
              ("prog_g66x130_q85", smooth(66, 130, 504)[:, :, 1], dict(quality=85)),
              ("prog_rst3_130x250", smooth(130, 250, 505), dict(quality=85, subsampling=2, restart_marker_blocks=3)),
              ("prog_rstrows_g47x61", smooth(47, 61, 506)[:, :, 2], dict(quality=75, restart_marker_rows=1)),
              ("prog_c7x9_s2_q95", noise(7, 9, 507), dict(quality=95, subsampling=2)),
              ("prog_c1x1_s2_q75", smooth(1, 1, 508), dict(quality=75, subsampling=2)),
              ("prog_q100_noise_40x72", noise(40, 72, 509), dict(quality=100, subsampling=2))]
    for name, img, kw in pcases:
        data = encode(img, progressive=True, **kw)
        out = decode_bgr(data)
        jpegs[name] = np.frombuffer(data, np.uint8)
        expect[name] = out
        meta["cases"][name] = {"w": int(out.shape[1]), "h": int(out.shape[0]), "ncomp": 1 if out.ndim == 2 else 3,
                               "unsupported": True, "progressive": True, "params": dict(kw, progressive=True),
                               "bytes": len(data)}
    # colour space as the JDK reader settles it (oracle/icx_oracle_decode.c
    # colour_space): Adobe transform 0 -> RGB (Pillow keep_rgb writes it, and
    # libjpeg-turbo reads it the same way), and files derived from it or from a
    # YCbCr file by rewriting markers and component ids only (same tables and
    # entropy data, so the expected pixels are those of the file they come from):
    #   ids 'R','G','B', no marker          -> RGB   (libjpeg's guess)
    #   ids 0,1,2, no marker, equal sampling -> RGB   (OpenJDK imageioJPEG.c override;
    #                                                  libjpeg-turbo would say YCbCr)
    #   ids 0,1,2 with an EXIF APP1          -> YCbCr (the override needs no EXIF)
    #   Adobe transform 1, ids 'R','G','B'   -> YCbCr (the Adobe marker wins)
    #   Adobe transform 2                    -> unknown: refused ("unsupported")
    seed += 1
    rgb_img = smooth(66, 130, seed)
    adobe = encode(rgb_img, quality=90, subsampling=0, keep_rgb=True)
    ycc = encode(rgb_img, quality=90, subsampling=0)
    rgb_px, ycc_px = decode_bgr(adobe), decode_bgr(ycc)
    derived = [("rgb_adobe0_66x130", adobe, rgb_px, False),
               ("rgb_ids_nomarker_66x130", rewrite(adobe, app=None, ids=b"RGB"), rgb_px, False),
               ("rgb_ids012_nomarker_66x130", rewrite(adobe, app=None, ids=bytes([0, 1, 2])), rgb_px, False),
               ("ycc_ids012_exif_66x130", rewrite(ycc, app=b"\xff\xe1\x00\x08Exif\x00\x00", ids=bytes([0, 1, 2])),
                ycc_px, False),
               ("ycc_adobe1_rgbids_66x130", rewrite(ycc, app=adobe_app14(1), ids=b"RGB"), ycc_px, False),
               ("unknown_adobe2_66x130", rewrite(ycc, app=adobe_app14(2), ids=None), None, True),
               # (round 4) the override also reaches a JFIF file with an Adobe
               # marker: transform 0 -> unknown, 1 -> YCbCr; IS_EXIF only asks
               # whether the first saved COM/APPn marker is an APP1
               ("unknown_jfif_adobe0_66x130", rewrite(ycc, app=JFIF_APP0 + adobe_app14(0), ids=None), None, True),
               ("ycc_jfif_adobe1_66x130", rewrite(ycc, app=JFIF_APP0 + adobe_app14(1), ids=None), ycc_px, False),
               ("ycc_ids012_xmp_first_66x130", rewrite(ycc, app=XMP_APP1, ids=bytes([0, 1, 2])), ycc_px, False),
               ("rgb_ids012_com_exif_66x130", rewrite(adobe, app=COM + b"\xff\xe1\x00\x08Exif\x00\x00",
                                                      ids=bytes([0, 1, 2])), rgb_px, False)]
    for name, data, px, refused in derived:
        jpegs[name] = np.frombuffer(data, np.uint8)
        meta["cases"][name] = {"w": 130, "h": 66, "ncomp": 3, "bytes": len(data), "colour": True,
                               "params": {"derived": True}}
        if refused:
            meta["cases"][name]["unsupported"] = True
        else:
            expect[name] = px
    prog_rgb = encode(smooth(47, 61, seed + 1), quality=85, subsampling=0, keep_rgb=True, progressive=True)
    jpegs["prog_rgb_adobe0_47x61"] = np.frombuffer(prog_rgb, np.uint8)
    expect["prog_rgb_adobe0_47x61"] = decode_bgr(prog_rgb)
    meta["cases"]["prog_rgb_adobe0_47x61"] = {"w": 61, "h": 47, "ncomp": 3, "unsupported": True, "progressive": True,
                                              "colour": True, "params": {"progressive": True, "keep_rgb": True},
                                              "bytes": len(prog_rgb)}
    np.savez_compressed(os.path.join(HERE, "decode_golden.npz"),
                        **{f"jpg:{k}": v for k, v in jpegs.items()},
                        **{f"px:{k}": v for k, v in expect.items()})
    with open(os.path.join(HERE, "decode_golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(len(jpegs), "cases")


if __name__ == "__main__":
    main()
