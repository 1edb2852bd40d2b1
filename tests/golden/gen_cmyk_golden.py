#!/usr/bin/env python3
"""Golden vectors for 4-component (CMYK / YCCK) JPEG decode.

The reference reads such files through TwelveMonkeys (ImageCompression.java
:32-35, 113-157), which delegates the baseline decode to the JDK's IJG 6b
and converts CMYK to RGB with an ICC profile.  The decode part is pinned
here by libjpeg-turbo 3.1.4 (Pillow 12.2's bundled libjpeg, 6b-lineage
jdcolor.c): its CMYK samples of
  * cmyk*:   Pillow-written CMYK files (Adobe APP14, transform 0: no colour
             transform), one with restart intervals;
  * ycck*:   the same files with only the Adobe transform byte set to 2
             (YCCK: the decoder runs jdcolor.c ycck_cmyk_convert on the
             same entropy data);
  * noadobe: the APP14 marker removed (4 components, no marker -> CMYK);
and the RGB step the build uses (Pillow: samples read as Adobe-inverted
CMYK, then cmyk2rgb) - TwelveMonkeys' ICC conversion is not restatable
without its profile (parity unpinned for that step).  Pillow inverts CMYK
JPEG samples on read ("CMYK;I"), so libjpeg's own samples are 255 - Pillow's.
Writes cmyk_golden.npz (files + expected CMYK samples + expected BGR)."""
import io
import os

import numpy as np
from PIL import Image, features

HERE = os.path.dirname(os.path.abspath(__file__))


def cmyk_source(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    ch = [127 + 100 * np.sin(x * rng.uniform(0.02, 0.2) + y * rng.uniform(0.01, 0.1) + k) for k in range(4)]
    a = np.stack(ch, -1) + rng.normal(0, 12, (h, w, 4))
    return np.clip(a, 0, 255).astype(np.uint8)


def set_transform(data, t):
    i = data.find(b"Adobe")
    assert i > 0
    b = bytearray(data)
    b[i + 11] = t  # APP14: "Adobe", version(2), flags0(2), flags1(2), transform(1)
    return bytes(b)


def drop_adobe(data):
    i = data.find(b"\xff\xee")
    n = (data[i + 2] << 8) | data[i + 3]
    return data[:i] + data[i + 2 + n:]


def main():
    assert features.check("libjpeg_turbo")
    files = {}
    for name, (h, w, seed, q, rst) in {"cmyk_64x48": (48, 64, 1, 90, 0), "cmyk_37x23": (23, 37, 2, 95, 0),
                                       "cmyk_130x66_rst": (66, 130, 3, 85, 1), "cmyk_201x9": (9, 201, 4, 75, 0)}.items():
        b = io.BytesIO()
        kw = {"restart_marker_rows": 1} if rst else {}
        Image.fromarray(cmyk_source(h, w, seed), "CMYK").save(b, "JPEG", quality=q, **kw)
        files[name] = b.getvalue()
    for name in list(files):
        files[name.replace("cmyk", "ycck")] = set_transform(files[name], 2)
    files["noadobe_64x48"] = drop_adobe(files["cmyk_64x48"])
    out = {}
    for name, data in files.items():
        im = Image.open(io.BytesIO(data))
        assert im.mode == "CMYK", name
        pil = np.asarray(im)
        out[f"{name}.jpg"] = np.frombuffer(data, np.uint8)
        out[f"{name}.cmyk"] = 255 - pil                      # libjpeg's samples
        out[f"{name}.bgr"] = np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])
    np.savez_compressed(os.path.join(HERE, "cmyk_golden.npz"), **out)
    print({k: v.shape for k, v in out.items() if k.endswith(".jpg")})


if __name__ == "__main__":
    main()
