"""Test double for icx.Codec backed by the CPU oracle.  Test infrastructure
only: lets the host-side batch/cache/sharding logic run in CPU-only CI; the
product package never uses it."""
import numpy as np

from icx import _native as N
from icx.core import IndexedImage, LearnedParams, default_palette, image_dims
from tests.oracle_ffi import Oracle


class OracleCodec:
    def __init__(self):
        self.o = Oracle()
        self.calls = 0

    def fit(self, images, target, quality, cached=None, outputs=None):
        self.calls += 1
        res = []
        for i, im in enumerate(images):
            c = cached[i] if cached else None
            r = self.o.fit(im, target, quality, cached=(c.quality, c.scale) if c else None)
            res.append({"status": 0, "success": r["success"], "cache_hit": r["cache_hit"],
                        "out_len": len(r["data"]) if r["success"] else 0, "encodes": r["encodes"],
                        "learned": LearnedParams(r["quality"], r["scale"]) if r["success"] else None,
                        "data": r["data"]})
        return res

    def decode_jpg_batch(self, datas, subsampling=0, device_out=False):
        """The oracle's IJG 6b decode (+ the reference's subsampling rule)."""
        out = []
        for d in datas:
            rc, w, h, _ = self.o.jpeg_info(d)
            if rc:
                out.append((rc, None))
                continue
            s = subsampling if subsampling > 0 else self.o.subsampling(w, h)
            out.append(self.o.jpeg_decode(d, s))
        return out

    def png_resize(self, img, params):
        w, h = image_dims(img)
        if w <= params.min_width and h <= params.min_height:
            return None
        s = min(params.min_width / w, params.min_height / h)
        dw, dh = self.o.scaled_dims(w, h, s)
        if isinstance(img, IndexedImage):  # the type kept, with its default colour map
            binary = img.fmt == N.BINARY1
            return IndexedImage(self.o.resize_indexed(img.indices, img.palette, binary, dw, dh),
                                default_palette(binary), img.fmt)
        return self.o.resize(img, dw, dh)  # (H, W, 4) = ABGR, as icx.core._fmt_of

    def png_fit_batch(self, images, params):
        return [self.png_resize(im, params) for im in images]

    def compress_png_with_target_size(self, img, output_file, params):
        r = self.png_resize(img, params)
        if r is None:
            return False
        from icx.pngio import write_png
        write_png(output_file, r)
        return True
