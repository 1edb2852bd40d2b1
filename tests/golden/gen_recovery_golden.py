#!/usr/bin/env python3
"""Generate the committed fixtures for the decoder's recovery semantics (A11).

Test infrastructure only.  Run once in the build container
(`JSIMD_FORCENONE=1` is set below, before Pillow loads libjpeg-turbo: its C
code paths are IJG 6b's arithmetic, its x86 SIMD ISLOW IDCT dequantises in 16
bits, which corrupt coefficients can overflow); the output
(recovery_golden.npz / .json) is committed and the GPU box never runs this.

The reference reads JPEGs through the JDK's JPEGImageReader (IJG libjpeg 6b,
ImageCompression.java:113-155), whose recovery from damaged entropy data the
reference inherits (an IOException would map to FAILED_IO_ERROR, :94-96, but
libjpeg only warns here, so the file is decoded and compressed):
  * end of file inside the scan: the JDK's source manager inserts a fake EOI
    (imageioJPEG.c imageio_fill_input_buffer); jdhuff.c then pads the bit
    buffer with zeros and sets insufficient_data: the MCU being decoded ends on
    zero bits and every later MCU of the segment stays zero (grey 128);
  * a bad Huffman code decodes as symbol 0 after 17 bits (JWRN_HUFF_BAD_CODE);
  * a missing, stray or misnumbered RSTn: jdmarker.c read_restart_marker /
    jpeg_resync_to_restart decide where decoding resumes.
libjpeg-turbo 3.1.4 keeps jdhuff.c's and jdmarker.c's logic, and Pillow's
LOAD_TRUNCATED_IMAGES appends the same fake EOI (JpegImagePlugin.load_read),
so its decodes pin these semantics for the sampling layouts both libraries
upsample alike (4:2:0, 4:2:2, 4:4:4, grey).  4:4:0 (h1v2) and 4:1:1 files are
added with the luma plane only pinned (Pillow's draft('L') decodes Y alone):
libjpeg-turbo upsamples h1v2 with a triangle filter where 6b replicates rows
(jdsample.c int_upsample), so their colour output is "parity unpinned".

Inputs are synthetic (seeded) files written by Pillow, then damaged: cut at
several points of the scan (also right after a 0xFF, and around an RSTn),
EOI removed, a run of 0xFF-data bytes planted (bad codes), an RSTn removed,
duplicated, renumbered or preceded by garbage bytes.
"""
import io
import json
import os
import sys

os.environ["JSIMD_FORCENONE"] = "1"

import numpy as np  # noqa: E402
from PIL import Image, ImageFile, features  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_decode_golden import encode, noise, smooth  # noqa: E402

ImageFile.LOAD_TRUNCATED_IMAGES = False


def scan_start(data):
    i = 2
    while True:
        m = data[i + 1]
        n = int.from_bytes(data[i + 2:i + 4], "big")
        i += 2 + n
        if m == 0xDA:
            return i


def rst_positions(data, s0):
    """Offsets of the RSTn markers (their 0xFF) in the scan."""
    out, i = [], s0
    while i + 1 < len(data):
        if data[i] == 0xFF and 0xD0 <= data[i + 1] <= 0xD7:
            out.append(i)
            i += 2
        else:
            i += 1
    return out


def decode(data, luma_only=False):
    """BGR / grey pixels of the file read with a fake EOI appended (the JDK's
    source manager inserts one at end of stream; this is what Pillow's
    LOAD_TRUNCATED_IMAGES does too, but with the flag off an error after the
    scan - jpeg_finish_decompress walks the markers up to EOI - still raises);
    None when libjpeg-turbo raises (the JDK reader throws: FAILED_IO_ERROR)."""
    im = Image.open(io.BytesIO(data + b"\xff\xd9"))
    if luma_only:
        im.draft("L", im.size)
    try:
        im.load()
    except OSError:
        return None
    a = np.asarray(im)
    if a.ndim == 3:
        a = a[:, :, ::-1]  # TYPE_3BYTE_BGR
    return np.ascontiguousarray(a)


def damaged(name, data):
    """(case name, bytes) of every damaged variant of one file."""
    s0 = scan_start(data)
    end = len(data) - 2  # the EOI
    n = end - s0
    out = []
    for f in (0.03, 0.3, 0.6, 0.9, 0.999):
        out.append((f"{name}_cut{int(f * 1000):03d}", data[:s0 + max(1, int(n * f))]))
    ff = [i for i in range(s0 + n // 3, end - 1) if data[i] == 0xFF and data[i + 1] == 0x00]
    if ff:
        out.append((f"{name}_cut_after_ff", data[:ff[0] + 1]))
        out.append((f"{name}_cut_after_ff00", data[:ff[0] + 2]))
    out.append((f"{name}_no_eoi", data[:end]))
    out.append((f"{name}_cut_scan_end", data[:end - 1]))
    mid = s0 + n // 2
    bad = bytearray(data)
    bad[mid:mid + 8] = b"\xff\x00" * 4  # 32 one bits: a bad code wherever the decoder meets them
    out.append((f"{name}_badcode", bytes(bad)))
    rst = rst_positions(data, s0)
    if rst:
        k = rst[len(rst) // 2]
        out.append((f"{name}_rst_missing", data[:k] + data[k + 2:]))
        out.append((f"{name}_rst_dup", data[:k + 2] + data[k:]))
        wrong = bytearray(data)
        wrong[k + 1] = 0xD0 + ((data[k + 1] - 0xD0 + 3) & 7)
        out.append((f"{name}_rst_wrong", bytes(wrong)))
        nxt = bytearray(data)
        nxt[k + 1] = 0xD0 + ((data[k + 1] - 0xD0 + 1) & 7)
        out.append((f"{name}_rst_skip1", bytes(nxt)))
        out.append((f"{name}_rst_garbage", data[:k] + b"\x12\x34\x56" + data[k:]))
        out.append((f"{name}_cut_before_rst", data[:k]))
        out.append((f"{name}_cut_in_rst", data[:k + 1]))
        out.append((f"{name}_cut_after_rst", data[:k + 2]))
        if len(rst) > 2:
            out.append((f"{name}_rst_missing_first", data[:rst[0]] + data[rst[0] + 2:]))
            bad2 = bytearray(data)
            a = rst[0] + 2 + (rst[1] - rst[0]) // 2
            bad2[a:a + 6] = b"\xff\x00" * 3
            out.append((f"{name}_badcode_interval", bytes(bad2)))
    return out


def trailers(name, data):
    """Markers after the scan, before EOI: jpeg_finish_decompress reads them
    (jdmarker.c read_markers) and throws on a duplicate SOI / SOF, a second
    SOS in a one-scan file, an unknown marker or a malformed table segment;
    COM / APPn / DHT / DQT / DRI / RSTn and garbage bytes are fine."""
    body, eoi = data[:-2], data[-2:]
    sos = data.index(b"\xff\xda")
    sof = data.index(b"\xff\xc0")
    dht = data.index(b"\xff\xc4")
    dht_seg = data[dht:dht + 2 + int.from_bytes(data[dht + 2:dht + 4], "big")]
    t = {"com": b"\xff\xfe\x00\x06note", "app1": b"\xff\xe1\x00\x04ab", "dht_ok": dht_seg,
         "dqt_ok": b"\xff\xdb\x00\x43\x01" + bytes(range(1, 65)), "dri_ok": b"\xff\xdd\x00\x04\x00\x05",
         "rst_extra": b"\xff\xd3", "garbage": b"\x12\x34\xff\x00\x56", "tem": b"\xff\x01",
         "dup_sos": data[sos:sos + 2 + int.from_bytes(data[sos + 2:sos + 4], "big")], "unknown": b"\xff\x02",
         "jpgn": b"\xff\xf3\x00\x02", "bad_dht": b"\xff\xc4\x00\x05\x00\x01\x02",
         "bad_dqt": b"\xff\xdb\x00\x43\x05" + bytes(64), "bad_dri": b"\xff\xdd\x00\x05\x00\x05\x00",
         "dup_soi": b"\xff\xd8", "dup_sof": data[sof:sof + 19], "sof9": b"\xff\xc9" + data[sof + 2:sof + 19]}
    return [(f"{name}_trailer_{k}", body + v + eoi) for k, v in t.items()]


def main():
    files = [
        ("c420_200x136", encode(smooth(136, 200, 7001), quality=95, subsampling=2)),
        ("c420_noise_72x96", encode(noise(72, 96, 7002), quality=80, subsampling=2)),
        ("c444_noise_80x96", encode(noise(80, 96, 7003), quality=75, subsampling=0)),
        ("c422_66x130", encode(smooth(66, 130, 7004), quality=90, subsampling=1)),
        ("grey_88x120", encode(smooth(88, 120, 7005)[:, :, 1], quality=85)),
        ("rst_c420_136x200", encode(smooth(136, 200, 7006), quality=95, subsampling=2, restart_marker_blocks=3)),
        ("rst_c444_80x96", encode(noise(80, 96, 7007), quality=75, subsampling=0, restart_marker_blocks=5)),
        ("rstrows_c422_66x130", encode(smooth(66, 130, 7008), quality=90, subsampling=1, restart_marker_rows=1)),
        ("rst_grey_88x120", encode(smooth(88, 120, 7009)[:, :, 0], quality=70, restart_marker_blocks=4)),
        ("rst1_c420_48x64", encode(smooth(48, 64, 7010), quality=85, subsampling=2, restart_marker_blocks=1)),
    ]
    jpegs, expect, meta = {}, {}, {"libjpeg_turbo": features.version("libjpeg_turbo"),
                                    "pillow": Image.__version__, "jsimd": "forcenone", "cases": {}}
    for k, (name, data) in enumerate(files):
        extra = trailers(name, data) if k in (0, 4, 5) else []
        for cname, d in [(name + "_intact", data)] + damaged(name, data) + extra:
            out = decode(d)
            jpegs[cname] = np.frombuffer(d, np.uint8)
            if out is None:  # the reader throws
                meta["cases"][cname] = {"bytes": len(d), "pinned": "error"}
                continue
            expect[cname] = out
            meta["cases"][cname] = {"w": int(out.shape[1]), "h": int(out.shape[0]),
                                    "ncomp": 1 if out.ndim == 2 else 3, "bytes": len(d), "pinned": "pixels"}
    # 4:4:0 and 4:1:1: the JDK replicates chroma (int_upsample); only Y is pinned
    for name, sub_y, img, kw in [("c440_66x130", (1, 2), smooth(66, 130, 7101), dict(quality=90)),
                                 ("c440_noise_47x61", (1, 2), noise(47, 61, 7102), dict(quality=80)),
                                 ("c411_66x130", (4, 1), smooth(66, 130, 7103), dict(quality=90)),
                                 ("rst_c440_66x130", (1, 2), smooth(66, 130, 7104),
                                  dict(quality=85, restart_marker_blocks=2))]:
            data = sampled(img, sub_y, **kw)
            variants = [(name + "_intact", data)] + [v for v in damaged(name, data)
                                                   if v[0].endswith(("cut300", "cut600", "badcode", "rst_missing"))]
            for cname, d in variants:
                y = decode(d, luma_only=True)
                assert y is not None, cname
                jpegs[cname] = np.frombuffer(d, np.uint8)
                expect[cname] = y
                meta["cases"][cname] = {"w": int(y.shape[1]), "h": int(y.shape[0]), "ncomp": 3,
                                        "bytes": len(d), "pinned": "luma", "sampling": list(sub_y)}
    np.savez_compressed(os.path.join(HERE, "recovery_golden.npz"),
                        **{f"jpg:{k}": v for k, v in jpegs.items()},
                        **{f"px:{k}": v for k, v in expect.items()})
    with open(os.path.join(HERE, "recovery_golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(len(jpegs), "cases")


def sampled(img, sub_y, quality, restart_marker_blocks=0):
    """A 3-component JPEG with luma sampled (h, v) = sub_y and 1x1 chroma,
    written by IJG libjpeg 9's encoder through mk_sampled_jpeg.c (Pillow's
    writer has no 4:4:0 / 4:1:1).  Only the file matters: its decode is what
    the fixtures pin."""
    import subprocess
    import tempfile
    tool = os.path.join(tempfile.gettempdir(), "mk_sampled_jpeg")
    subprocess.run(["gcc", "-O1", "-I/opt/conda/include", "-o", tool, os.path.join(HERE, "mk_sampled_jpeg.c"),
                    "-L/opt/conda/lib", "-ljpeg", "-Wl,-rpath,/opt/conda/lib"], check=True)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.rgb"), os.path.join(d, "out.jpg")
        np.ascontiguousarray(img).tofile(src)
        h, w = img.shape[:2]
        subprocess.run([tool, str(w), str(h), str(quality), str(sub_y[0]), str(sub_y[1]),
                        str(restart_marker_blocks), src, dst], check=True)
        with open(dst, "rb") as f:
            return f.read()


if __name__ == "__main__":
    main()
