"""ctypes access to oracle/liboracle.so — the CPU restatement used as the
checker (test infrastructure only; never imported by the product package)."""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")
FMT = {"bgr": 0, "rgb": 1, "gray": 2}


def build_oracle():
    lib = os.path.join(ORACLE_DIR, "liboracle.so")
    srcs = [os.path.join(ORACLE_DIR, f) for f in ("icx_oracle.c", "icx_oracle_decode.c", "icx_oracle.h")]
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return lib


def fmt_of(img):
    return 2 if img.ndim == 2 else 0


class Oracle:
    def __init__(self):
        L = ctypes.CDLL(build_oracle())
        c, P = ctypes, ctypes.POINTER
        L.oracle_encode.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.c_float, c.c_void_p,
                                    c.c_size_t, P(c.c_size_t)]
        L.oracle_num_blocks.restype = c.c_long
        L.oracle_num_blocks.argtypes = [c.c_int, c.c_int, c.c_int]
        L.oracle_fdct.restype = c.c_long
        L.oracle_fdct.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.c_void_p]
        L.oracle_qtables.argtypes = [c.c_float, P(c.c_uint16), P(c.c_uint16)]
        L.oracle_find_best_quality.restype = c.c_float
        L.oracle_find_best_quality.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int64,
                                               c.c_float, P(c.c_float), P(c.c_int64), P(c.c_int)]
        L.oracle_resize.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_int,
                                    c.c_int, c.c_int]
        L.oracle_scaled_dims.argtypes = [c.c_int, c.c_int, c.c_double, P(c.c_int), P(c.c_int)]
        L.oracle_compress_jpg_with_target_size.argtypes = [
            c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.c_int64, c.c_float, c.c_int, c.c_float,
            c.c_double, c.c_void_p, c.c_size_t, P(c.c_size_t), P(c.c_float), P(c.c_double), P(c.c_int),
            P(c.c_int)]
        L.oracle_subsampling.argtypes = [c.c_int, c.c_int]
        L.oracle_create_key.argtypes = [c.c_int, c.c_int, c.c_int64, P(c.c_int), P(c.c_int), P(c.c_int64)]
        L.oracle_fit_batch.restype = c.c_long
        L.oracle_fit_batch.argtypes = [c.c_int, P(c.c_void_p), P(c.c_int), P(c.c_int), P(c.c_int), c.c_int,
                                       c.c_int64, c.c_float, c.c_int, c.c_float, c.c_double, c.c_int,
                                       P(c.c_int64), P(c.c_float), P(c.c_double)]
        L.oracle_jpeg_info.argtypes = [c.c_void_p, c.c_size_t, P(c.c_int), P(c.c_int), P(c.c_int)]
        L.oracle_jpeg_num_blocks.restype = c.c_long
        L.oracle_jpeg_num_blocks.argtypes = [c.c_void_p, c.c_size_t]
        L.oracle_jpeg_coefs.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t]
        L.oracle_jpeg_decode.argtypes = [c.c_void_p, c.c_size_t, c.c_int, c.c_void_p, c.c_size_t, P(c.c_int),
                                         P(c.c_int), P(c.c_int)]
        L.oracle_jpeg_decode_cmyk.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, P(c.c_int), P(c.c_int)]
        L.oracle_jpeg_decode_luma.argtypes = [c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, P(c.c_int), P(c.c_int)]
        L.oracle_set_table_layout.argtypes = [c.c_int]
        L.oracle_resize_indexed.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_void_p,
                                            c.c_int, c.c_int, c.c_int]
        L.oracle_default_palette.argtypes = [c.c_int, c.c_void_p, P(c.c_int)]
        L.oracle_inverse_cube.argtypes = [c.c_void_p, c.c_int, c.c_void_p]
        L.oracle_dither_tables.argtypes = [c.c_int, c.c_void_p, c.c_void_p, c.c_void_p]
        self.L = L

    def set_table_layout(self, grouped):
        """Process-wide table marker layout (0: one DQT/DHT per table, the
        default; 1: grouped).  Tests that change it restore 0."""
        self.L.oracle_set_table_layout(1 if grouped else 0)

    def encode(self, img, q):
        img = np.ascontiguousarray(img)
        h, w = img.shape[:2]
        cap = w * h * 4 + 8192
        out = np.empty(cap, np.uint8)
        n = ctypes.c_size_t()
        rc = self.L.oracle_encode(img.ctypes.data, w, h, img.strides[0], fmt_of(img), float(np.float32(q)),
                                  out.ctypes.data, cap, ctypes.byref(n))
        assert rc == 0, rc
        return out[:n.value].tobytes()

    def fdct(self, img):
        img = np.ascontiguousarray(img)
        h, w = img.shape[:2]
        nb = self.L.oracle_num_blocks(w, h, fmt_of(img))
        out = np.empty((nb, 64), np.int16)
        self.L.oracle_fdct(img.ctypes.data, w, h, img.strides[0], fmt_of(img), out.ctypes.data)
        return out

    def qtables(self, q):
        a = (ctypes.c_uint16 * 64)()
        b = (ctypes.c_uint16 * 64)()
        self.L.oracle_qtables(float(np.float32(q)), a, b)
        return list(a), list(b)

    def find_best_quality(self, img, target, q0):
        img = np.ascontiguousarray(img)
        h, w = img.shape[:2]
        tq = (ctypes.c_float * 8)()
        ts = (ctypes.c_int64 * 8)()
        nt = ctypes.c_int()
        best = self.L.oracle_find_best_quality(img.ctypes.data, w, h, img.strides[0], fmt_of(img), int(target),
                                               float(np.float32(q0)), tq, ts, ctypes.byref(nt))
        return best, [(tq[i], ts[i]) for i in range(nt.value)]

    def scaled_dims(self, w, h, s):
        a, b = ctypes.c_int(), ctypes.c_int()
        self.L.oracle_scaled_dims(w, h, float(s), ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def resize(self, img, dw, dh, fmt=None):
        """fmt: icx_fmt numbering; default grey / BGR24 / ABGR32 by channels,
        GRAY16 (7) for a uint16 (H, W) array."""
        img = np.ascontiguousarray(img)
        h, w = img.shape[:2]
        nch = 1 if img.ndim == 2 else img.shape[2]
        if fmt is None:
            fmt = 7 if img.dtype == np.uint16 else 2 if nch == 1 else 0 if nch == 3 else 5
        out = np.empty((dh, dw, nch) if nch > 1 else (dh, dw), img.dtype)
        self.L.oracle_resize(img.ctypes.data, w, h, img.strides[0], fmt, out.ctypes.data, dw, dh,
                             dw * nch * img.itemsize)
        return out

    def default_palette(self, binary):
        pal = np.zeros(256, np.uint32)
        n = ctypes.c_int()
        self.L.oracle_default_palette(1 if binary else 0, pal.ctypes.data, ctypes.byref(n))
        return pal[:n.value].copy()

    def resize_indexed(self, indices, palette, binary, dw, dh):
        """TYPE_BYTE_INDEXED (binary 0) / TYPE_BYTE_BINARY (1) resize: source
        indices + colour map -> indices into the type's default map."""
        src = np.ascontiguousarray(indices, np.uint8)
        pal = np.full(256, 0xff000000, np.uint32)
        p = np.asarray(palette, np.uint32)
        pal[:len(p)] = p
        out = np.empty((dh, dw), np.uint8)
        h, w = src.shape
        rc = self.L.oracle_resize_indexed(src.ctypes.data, w, h, src.strides[0], pal.ctypes.data, 1 if binary else 0,
                                          out.ctypes.data, dw, dh, dw)
        assert rc == 0, rc
        return out

    def fit(self, img, target, q0, cached=None):
        img = np.ascontiguousarray(img)
        h, w = img.shape[:2]
        cap = w * h * 4 + 8192
        out = np.empty(cap, np.uint8)
        n = ctypes.c_size_t()
        bq, bs = ctypes.c_float(), ctypes.c_double()
        enc, hit = ctypes.c_int(), ctypes.c_int()
        has = cached is not None
        cq, cs = (cached if has else (0.0, 1.0))
        rc = self.L.oracle_compress_jpg_with_target_size(
            img.ctypes.data, w, h, img.strides[0], fmt_of(img), int(target), float(np.float32(q0)), int(has),
            float(np.float32(cq)), float(cs), out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(bq),
            ctypes.byref(bs), ctypes.byref(enc), ctypes.byref(hit))
        assert rc >= 0
        return {"success": rc == 1, "data": out[:n.value].tobytes() if rc == 1 else None,
                "quality": bq.value if rc == 1 else None, "scale": bs.value if rc == 1 else None,
                "encodes": enc.value, "cache_hit": bool(hit.value)}

    def jpeg_info(self, data):
        data = np.frombuffer(bytes(data), np.uint8)
        w, h, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = self.L.oracle_jpeg_info(data.ctypes.data, data.size, ctypes.byref(w), ctypes.byref(h),
                                     ctypes.byref(n))
        return rc, w.value, h.value, n.value

    def jpeg_coefs(self, data):
        """Quantised coefficients (natural order) per scan block; None if refused."""
        data = np.frombuffer(bytes(data), np.uint8)
        nb = self.L.oracle_jpeg_num_blocks(data.ctypes.data, data.size)
        if nb < 0:
            return None
        out = np.empty((nb, 64), np.int16)
        rc = self.L.oracle_jpeg_coefs(data.ctypes.data, data.size, out.ctypes.data, nb)
        return out if rc == 0 else None

    def jpeg_decode(self, data, s=1):
        """(status, pixels): BGR (H, W, 3) or grey (H, W) after source subsampling s."""
        data = np.frombuffer(bytes(data), np.uint8)
        rc, w, h, n = self.jpeg_info(data)
        if rc:
            return rc, None
        dw, dh = -(-w // s), -(-h // s)
        out = np.empty(dw * dh * n, np.uint8)
        ow, oh, of = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = self.L.oracle_jpeg_decode(data.ctypes.data, data.size, s, out.ctypes.data, out.size,
                                       ctypes.byref(ow), ctypes.byref(oh), ctypes.byref(of))
        if rc:
            return rc, None
        return 0, out[:dw * dh * min(n, 3)].reshape((oh.value, ow.value, 3) if n >= 3 else (oh.value, ow.value))

    def jpeg_decode_luma(self, data):
        """(status, samples): a 3-component file's luma samples alone (H, W)."""
        data = np.frombuffer(bytes(data), np.uint8)
        rc, w, h, n = self.jpeg_info(data)
        if rc:
            return rc, None
        out = np.empty(w * h, np.uint8)
        ow, oh = ctypes.c_int(), ctypes.c_int()
        rc = self.L.oracle_jpeg_decode_luma(data.ctypes.data, data.size, out.ctypes.data, out.size, ctypes.byref(ow),
                                            ctypes.byref(oh))
        return (rc, None) if rc else (0, out.reshape(h, w))

    def jpeg_decode_cmyk(self, data):
        """(status, samples): a 4-component file's CMYK samples (H, W, 4) as libjpeg outputs them."""
        data = np.frombuffer(bytes(data), np.uint8)
        rc, w, h, n = self.jpeg_info(data)
        if rc:
            return rc, None
        out = np.empty(w * h * 4, np.uint8)
        ow, oh = ctypes.c_int(), ctypes.c_int()
        rc = self.L.oracle_jpeg_decode_cmyk(data.ctypes.data, data.size, out.ctypes.data, out.size, ctypes.byref(ow),
                                            ctypes.byref(oh))
        return (rc, None) if rc else (0, out.reshape(h, w, 4))

    def subsampling(self, w, h):
        return self.L.oracle_subsampling(w, h)

    def create_key(self, w, h, size):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        self.L.oracle_create_key(w, h, size, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def fit_batch(self, imgs, target, q0, cached=None, threads=1):
        n = len(imgs)
        imgs = [np.ascontiguousarray(i) for i in imgs]
        ptrs = (ctypes.c_void_p * n)(*[i.ctypes.data for i in imgs])
        ws = (ctypes.c_int * n)(*[i.shape[1] for i in imgs])
        hs = (ctypes.c_int * n)(*[i.shape[0] for i in imgs])
        ss = (ctypes.c_int * n)(*[i.strides[0] for i in imgs])
        sizes = (ctypes.c_int64 * n)()
        qs = (ctypes.c_float * n)()
        sc = (ctypes.c_double * n)()
        has = cached is not None
        cq, cs = cached if has else (0.0, 1.0)
        enc = self.L.oracle_fit_batch(n, ptrs, ws, hs, ss, fmt_of(imgs[0]), int(target), float(np.float32(q0)),
                                      int(has), float(np.float32(cq)), float(cs), threads, sizes, qs, sc)
        return enc, list(sizes), list(qs), list(sc)


def load_golden():
    meta = json.load(open(os.path.join(GOLDEN_DIR, "golden.json")))
    inputs = dict(np.load(os.path.join(GOLDEN_DIR, "inputs.npz")))
    jpegs = dict(np.load(os.path.join(GOLDEN_DIR, "jpeg_golden.npz")))
    return meta, inputs, jpegs


def load_decode_golden():
    meta = json.load(open(os.path.join(GOLDEN_DIR, "decode_golden.json")))
    z = np.load(os.path.join(GOLDEN_DIR, "decode_golden.npz"))
    jpgs = {k[4:]: z[k].tobytes() for k in z.files if k.startswith("jpg:")}
    pxs = {k[3:]: z[k] for k in z.files if k.startswith("px:")}
    return meta, jpgs, pxs


def jdk_bytes(turbo_bytes, meta):
    """The golden file with the JFIF minor version the JDK writes (1.02)."""
    b = bytearray(turbo_bytes)
    b[meta["jfif_version_offset"]] = 2
    return bytes(b)


def smooth(h, w, seed):
    rng = np.random.default_rng(seed)
    fx, fy, ph = rng.uniform(0.002, 0.02, 3)
    y = np.arange(h, dtype=np.float32)[:, None]
    x = np.arange(w, dtype=np.float32)[None, :]
    r = 127 + 100 * np.sin(x * fx * 10 + ph) + 0 * y
    g = 127 + 100 * np.sin(y * fy * 10 + 2 * ph) + 0 * x
    b = 127 + 100 * np.sin((x + y) * fx * 5)
    rgb = np.stack([r, g, b], -1) + rng.normal(0, 16, (h, w, 3)).astype(np.float32)
    return np.clip(np.rint(rgb), 0, 255).astype(np.uint8)[:, :, ::-1].copy()


def noise(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
