"""Host-side mirror of the reference's hot-path interface, backed by libicx.

Reference (PolloChang/image-compression @ 2025-07-25) -> here:

  report/CompressionParams.java:3        CompressionParams
  report/CompressionReport.java:5        CompressionReport
  core/CompressionResult.java:3-11       CompressionResult
  learn/LearnedParams.java:8             LearnedParams
  learn/jpg/SimilarityKey.java:9         SimilarityKey
  tools/CacheTools.java:14-21            create_key
  tools/ImageTools.java:7-26             Codec.resize_image
  core/ImageCompressionJpg.java:136-147  Codec.compress_jpg_to_stream
  core/ImageCompressionJpg.java:158-200  Codec.find_best_quality_by_binary_search
  core/ImageCompressionJpg.java:77-122   Codec.compress_jpg_with_target_size
  core/ImageCompressionPng.java:37-75    Codec.compress_png_with_target_size

Images are numpy arrays (H, W, 3) uint8 in BGR order (BufferedImage
TYPE_3BYTE_BGR) or (H, W) uint8 grey (TYPE_BYTE_GRAY), or CUDA tensors of the
same shape (then no host<->device copy of the pixels happens).
"""
import ctypes
import enum
import logging
import threading
from dataclasses import dataclass
from typing import Dict, MutableMapping, Optional

import numpy as np

from . import _native as N

log = logging.getLogger("icx")


class CompressionResult(enum.Enum):
    COMPRESSED_SUCCESS = "成功壓縮"
    SKIPPED_CONDITION_NOT_MET = "不符條件跳過"
    SKIPPED_NOT_FOUND = "來源檔案不存在"
    FAILED_COMPRESSION = "壓縮失敗(無法達標)"
    FAILED_UNSUPPORTED_FORMAT = "格式不支援"
    FAILED_IO_ERROR = "IO錯誤"
    FAILED_OUT_OF_MEMORY = "記憶體溢位"
    FAILED_UNKNOWN = "未知錯誤"

    @property
    def description(self):
        return self.value


@dataclass(frozen=True)
class CompressionParams:
    quality: float
    min_size_bytes: int
    min_width: int
    min_height: int
    target_max_size_bytes: int


@dataclass(frozen=True)
class CompressionReport:
    result: CompressionResult
    original_size: int
    compressed_size: int


@dataclass(frozen=True)
class LearnedParams:
    quality: float  # Java float: always a float32-representable value here
    scale: float


@dataclass(frozen=True)
class SimilarityKey:
    width_bucket: int
    height_bucket: int
    size_bucket: int


def _f32(x):
    return float(np.float32(x))


def image_dims(img):
    shape = tuple(img.shape)
    return shape[1], shape[0]


def create_key(image, file_size) -> SimilarityKey:
    """CacheTools.createKey: (w/100, h/100, fileSize/102400), decoded dims."""
    w, h = image_dims(image)
    return SimilarityKey(w // 100, h // 100, int(file_size) // 102400)


class IndexedImage:
    """A TYPE_BYTE_INDEXED (fmt INDEXED8) or TYPE_BYTE_BINARY (BINARY1) raster:
    one colour-map index per byte (`indices`, (H, W) uint8; a 1/2/4-bit raster
    unpacked) and its IndexColorModel (`palette`, 0xAARRGGBB uint32).  How the
    JDK's PNG reader returns palette PNGs and 1/2/4-bit grey PNGs; the resize
    keeps the type with the type's DEFAULT map (ImageTools.java:12-17)."""

    def __init__(self, indices, palette, fmt):
        self.indices = np.ascontiguousarray(indices, dtype=np.uint8)
        self.palette = np.ascontiguousarray(palette, dtype=np.uint32)
        if fmt not in (N.INDEXED8, N.BINARY1) or self.indices.ndim != 2:
            raise ValueError("IndexedImage: (H, W) indices, fmt INDEXED8 or BINARY1")
        if not 1 <= len(self.palette) <= (16 if fmt == N.BINARY1 else 256):
            raise ValueError("IndexedImage: palette size")
        self.fmt = fmt

    @property
    def shape(self):
        return self.indices.shape

    @property
    def ndim(self):
        return 2

    @property
    def dtype(self):
        return self.indices.dtype

    def colours(self) -> np.ndarray:
        """(H, W, 4) bytes A, R, G, B per pixel (the map applied)."""
        p = self.palette[np.minimum(self.indices, len(self.palette) - 1)]
        return np.stack([(p >> s & 255).astype(np.uint8) for s in (24, 16, 8, 0)], -1)

    @classmethod
    def default(cls, fmt, height, width):
        """An all-zero raster of `new BufferedImage(width, height, type)`."""
        return cls(np.zeros((height, width), np.uint8), default_palette(fmt == N.BINARY1), fmt)


def default_palette(binary: bool) -> np.ndarray:
    """The colour map of a new TYPE_BYTE_INDEXED (256 entries: 6x6x6 cube +
    grey ramp) or TYPE_BYTE_BINARY (black, white) BufferedImage."""
    pal = (ctypes.c_uint32 * 256)()
    n = N.load().icx_default_palette(1 if binary else 0, pal)
    return np.array(pal[:n], dtype=np.uint32)


def _fmt_of(img):
    """The BufferedImage type of an array: (H, W) grey = TYPE_BYTE_GRAY,
    (H, W, 3) = TYPE_3BYTE_BGR, (H, W, 4) = TYPE_4BYTE_ABGR (bytes A, B, G, R:
    how ImageIO reads an RGBA PNG).  Other layouts: pass fmt explicitly."""
    if isinstance(img, IndexedImage):
        return img.fmt
    if img.ndim == 2 and str(getattr(img, "dtype", "")) in ("uint16", "torch.uint16", "torch.int16"):
        return N.GRAY16  # TYPE_USHORT_GRAY
    if img.ndim == 2 or (img.ndim == 3 and img.shape[2] == 1):
        return N.GRAY8
    if img.ndim == 3 and img.shape[2] == 3:
        return N.BGR24
    if img.ndim == 3 and img.shape[2] == 4:
        return N.ABGR32
    raise ValueError(f"unsupported image shape {tuple(img.shape)}")


def _out_shape(h, w, fmt):
    nch = N.CHANNELS[fmt]
    return (h, w) if nch == 1 else (h, w, nch)


def _out_dtype(fmt):
    return np.uint16 if fmt == N.GRAY16 else np.uint8


def _new_raster(h, w, fmt):
    """The destination of a resize: an array of the source's type, or for a
    palette type a new raster with that type's default colour map."""
    if fmt in (N.INDEXED8, N.BINARY1):
        return IndexedImage(np.empty((h, w), np.uint8), default_palette(fmt == N.BINARY1), fmt)
    return np.empty(_out_shape(h, w, fmt), _out_dtype(fmt))


def _pixels(raster):
    return raster.indices if isinstance(raster, IndexedImage) else raster


class DeviceImage:
    """A frame (or byte string) in the codec GPU's HBM, allocated through the
    C ABI (icx_device_alloc): (H, W, 3) BGR or (H, W) grey uint8, contiguous.
    Decoded frames stay here between icx_decode_jpg_batch and
    icx_compress_jpg_batch; the product path needs no PyTorch."""
    icx_device = True

    def __init__(self, codec, shape):
        self.codec = codec
        self.shape = tuple(int(x) for x in shape)
        self.nbytes = int(np.prod(self.shape))
        p = ctypes.c_void_p()
        codec._check(codec._lib.icx_device_alloc(codec._ctx, self.nbytes, ctypes.byref(p)), "icx_device_alloc")
        self.ptr = p.value

    @property
    def ndim(self):
        return len(self.shape)

    def data_ptr(self):
        return self.ptr

    def numel(self):
        return self.nbytes

    def numpy(self, nbytes=None) -> np.ndarray:
        """Copy to host (the first nbytes as a flat array when given)."""
        n = self.nbytes if nbytes is None else min(int(nbytes), self.nbytes)
        out = np.empty(self.shape if nbytes is None else (n,), np.uint8)
        self.codec._check(self.codec._lib.icx_memcpy(self.codec._ctx, out.ctypes.data, self.ptr, n), "icx_memcpy")
        return out

    @classmethod
    def adopt(cls, codec, ptr, shape) -> "DeviceImage":
        """Take ownership of a buffer this codec's context allocated
        (icx_device_alloc, e.g. a file icx_stage_files staged)."""
        d = cls.__new__(cls)
        d.codec = codec
        d.shape = tuple(int(x) for x in shape)
        d.nbytes = int(np.prod(d.shape))
        d.ptr = ptr
        return d

    @classmethod
    def from_host(cls, codec, arr) -> "DeviceImage":
        a = np.ascontiguousarray(np.frombuffer(arr, np.uint8) if isinstance(arr, (bytes, bytearray)) else arr)
        d = cls(codec, a.shape)
        codec._check(codec._lib.icx_memcpy(codec._ctx, d.ptr, a.ctypes.data, d.nbytes), "icx_memcpy")
        return d

    def free(self):
        if self.ptr and self.codec._ctx:
            self.codec._lib.icx_device_free(self.codec._ctx, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedBuffer:
    """Page-locked host bytes from the codec's pool (icx_host_alloc): a file
    read into one is uploaded by DMA with no staging copy.  `array` is a
    numpy view of the first `size` bytes."""

    def __init__(self, codec, size):
        self.codec = codec
        self.size = int(size)
        p = ctypes.c_void_p()
        codec._check(codec._lib.icx_host_alloc(codec._ctx, max(1, self.size), ctypes.byref(p)), "icx_host_alloc")
        self.ptr = p.value
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, self.size)).from_address(self.ptr))[:self.size]

    @classmethod
    def read_file(cls, codec, path) -> "PinnedBuffer":
        import os
        size = os.path.getsize(path)
        b = cls(codec, size)
        with open(path, "rb", buffering=0) as f:
            n = f.readinto(memoryview(b.array))
        b.size = n
        b.array = b.array[:n]
        return b

    @property
    def nbytes(self):
        return self.size

    def __getitem__(self, k):
        return self.array[k]

    def __len__(self):
        return self.size

    def free(self):
        if self.ptr and self.codec._ctx:
            self.array = None
            self.codec._lib.icx_host_free(self.codec._ctx, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _image_struct(img, fmt=None):
    """Describe a numpy array, DeviceImage or CUDA tensor as an icx_image (no copy)."""
    if img is None:
        raise TypeError("image must not be null")
    if fmt is None:
        fmt = _fmt_of(img)
    h, w = int(img.shape[0]), int(img.shape[1])
    bpp = N.BYTES_PER_PX[fmt]
    if isinstance(img, IndexedImage):
        if fmt != img.fmt:
            raise ValueError("an IndexedImage keeps its own format")
        return N.Image(img.indices.ctypes.data, w, h, img.indices.strides[0], fmt, img.palette.ctypes.data,
                       len(img.palette)), img
    if fmt in (N.INDEXED8, N.BINARY1):
        raise ValueError("palette formats need an IndexedImage (indices + colour map)")
    if getattr(img, "icx_device", False):
        return N.Image(img.data_ptr(), w, h, w * bpp, fmt), img
    if isinstance(img, np.ndarray):
        want = np.uint16 if fmt == N.GRAY16 else np.uint8
        if img.dtype != want:
            raise ValueError(f"image must be {np.dtype(want).name}")
        nch = N.CHANNELS[fmt]
        if not (img.flags["C_CONTIGUOUS"] or (img.strides[-1] == img.itemsize
                                              and (img.ndim == 2 or img.strides[1] == nch)
                                              and (bpp != 4 or img.strides[0] % 4 == 0))):
            img = np.ascontiguousarray(img)
        ptr, stride = img.ctypes.data, img.strides[0]
    else:  # torch tensor (CUDA or CPU)
        if str(img.dtype) not in ("torch.uint8",) + (("torch.uint16", "torch.int16") if fmt == N.GRAY16 else ()):
            raise ValueError("image must be uint8 (uint16 / int16 bits for GRAY16)")
        if not img.is_contiguous():
            raise ValueError("tensor image must be contiguous")
        ptr, stride = img.data_ptr(), img.stride(0) * img.element_size()
    return N.Image(ptr, w, h, stride, fmt), img


class Codec:
    """One libicx context (one GPU).  Thread-safe."""

    supports_device_out = True  # decode_jpg_batch(device_out=True) leaves frames in this GPU's HBM

    def __init__(self, device: int = 0):
        self._lib = N.load()
        self._ctx = ctypes.c_void_p()
        st = self._lib.icx_create(device, ctypes.byref(self._ctx))
        if st != N.OK:
            raise N.IcxError(st, f"icx_create(device={device}) failed: "
                                 f"{self._lib.icx_status_string(st).decode()}")
        self.device = device
        self._lock = threading.Lock()

    def close(self):
        if self._ctx:
            self._lib.icx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        return self._lib.icx_last_error(self._ctx).decode()

    def _batch_call(self, what, jobs, n):
        return getattr(self._lib, f"icx_{what}_batch")(self._ctx, jobs, n)

    def _check(self, st, what):
        if st != N.OK:
            raise N.IcxError(st, f"{what}: {self._lib.icx_status_string(st).decode()} "
                                 f"({self._lib.icx_last_error(self._ctx).decode()})")

    # -------------------------------------------------------------- A12
    def resize_image(self, original_image, scale: float, fmt=None) -> np.ndarray:
        """ImageTools.resizeImage(BufferedImage, double): Java2D bilinear; the
        result keeps the source type (ImageTools.java:12-15)."""
        img, keep = _image_struct(original_image, fmt)
        w = ctypes.c_int32()
        h = ctypes.c_int32()
        self._lib.icx_scaled_dims(img.width, img.height, float(scale), ctypes.byref(w), ctypes.byref(h))
        res = _new_raster(h.value, w.value, img.fmt)
        out = _pixels(res)
        st = self._lib.icx_resize_image(self._ctx, ctypes.byref(img), float(scale), out.ctypes.data, out.nbytes,
                                        ctypes.byref(w), ctypes.byref(h))
        self._check(st, "icx_resize_image")
        return res

    def resize_to(self, original_image, width: int, height: int, fmt=None) -> np.ndarray:
        img, keep = _image_struct(original_image, fmt)
        res = _new_raster(height, width, img.fmt)
        out = _pixels(res)
        st = self._lib.icx_resize_bilinear(self._ctx, ctypes.byref(img), out.ctypes.data, width, height,
                                           width * N.BYTES_PER_PX[img.fmt])
        self._check(st, "icx_resize_bilinear")
        return res

    # -------------------------------------------------------------- A4
    def compress_jpg_to_stream(self, image, quality: float) -> bytes:
        """compressJpgToStream: one JPEG encode at `quality` (float32)."""
        img, keep = _image_struct(image)
        cap = max(1 << 16, img.width * img.height * 3 + 4096)
        for _ in range(2):
            out = np.empty(cap, np.uint8)
            n = ctypes.c_size_t()
            st = self._lib.icx_compress_jpg_to_stream(self._ctx, ctypes.byref(img), _f32(quality),
                                                      out.ctypes.data, cap, ctypes.byref(n))
            if st == N.E_BUFFER:
                cap = n.value
                continue
            self._check(st, "icx_compress_jpg_to_stream")
            return out[:n.value].tobytes()
        raise N.IcxError(N.E_BUFFER, "output buffer")

    # -------------------------------------------------------------- A3
    def find_best_quality_by_binary_search(self, image, target_max_size_bytes: int, initial_quality: float,
                                           trace: Optional[list] = None) -> float:
        img, keep = _image_struct(image)
        best = ctypes.c_float()
        tq = (ctypes.c_float * 8)()
        ts = (ctypes.c_int64 * 8)()
        nt = ctypes.c_int32()
        st = self._lib.icx_find_best_quality(self._ctx, ctypes.byref(img), int(target_max_size_bytes),
                                             _f32(initial_quality), ctypes.byref(best), tq, ts, ctypes.byref(nt))
        self._check(st, "icx_find_best_quality")
        if trace is not None:
            trace.extend((tq[i], ts[i], ts[i] <= target_max_size_bytes) for i in range(nt.value))
        return best.value

    # -------------------------------------------------------------- A2
    def fit(self, images, target_max_size_bytes, quality, cached=None, outputs=None):
        """Batched compressJpgWithTargetSize core: returns one dict per image.
        cached: list of LearnedParams|None; outputs: optional preallocated buffers."""
        n = len(images)
        jobs = (N.FitJob * n)()
        keep, bufs = [], []
        for i, im in enumerate(images):
            img, k = _image_struct(im)
            keep.append(k)
            j = jobs[i]
            j.img = img
            j.target_max_size = int(target_max_size_bytes)
            j.quality = _f32(quality)
            c = cached[i] if cached else None
            if c is not None:
                j.has_cached = 1
                j.cached = N.LearnedParams(_f32(c.quality), float(c.scale))
            if outputs is not None:
                buf = outputs[i]
                j.out = buf.data_ptr() if hasattr(buf, "data_ptr") else buf.ctypes.data
                j.cap = buf.numel() if hasattr(buf, "numel") else buf.nbytes
            else:
                buf = np.empty(int(target_max_size_bytes) + 1, np.uint8)
                j.out = buf.ctypes.data
                j.cap = buf.nbytes
            bufs.append(buf)
        with self._lock:
            st = self._batch_call("compress_jpg", jobs, n)
        self._check(st, "icx_compress_jpg_batch")
        res = []
        for i in range(n):
            j = jobs[i]
            r = {"status": j.status, "success": bool(j.success), "cache_hit": bool(j.cache_hit),
                 "out_len": j.out_len, "encodes": j.encodes,
                 "learned": LearnedParams(j.learned.quality, j.learned.scale) if j.success else None}
            if outputs is None and j.success and j.status == N.OK:
                r["data"] = bufs[i][:j.out_len].tobytes()
            res.append(r)
        return res

    def prepare(self, images, target_max_size_bytes, quality, cached=None, outputs=None):
        """A reusable job array over device- or host-resident images (bench)."""
        return PreparedBatch(self, images, target_max_size_bytes, quality, cached, outputs)

    def compress_jpg_with_target_size(self, original_image, original_size: int, output_file,
                                      params: CompressionParams,
                                      cache: MutableMapping[SimilarityKey, LearnedParams]) -> bool:
        """ImageCompressionJpg.compressJpgWithTargetSize (cache probe, scale loop,
        binary search, save, learn)."""
        key = create_key(original_image, original_size)
        cached = cache.get(key)
        r = self.fit([original_image], params.target_max_size_bytes, params.quality, cached=[cached])[0]
        if r["status"] == N.E_NOMEM:
            raise MemoryError("device out of memory")
        if r["status"] != N.OK:
            raise OSError(f"icx encode failed with status {r['status']}")
        if cached is not None and r["cache_hit"]:
            log.info("快取成功: %s 使用學習參數直接達成目標。", output_file)
        elif cached is not None:
            log.warning("快取失效: %s 使用學習參數後檔案仍超標，退回標準流程。", output_file)
        if not r["success"]:
            log.warning("無法在目標大小限制下完成壓縮: %s", output_file)
            return False
        with open(output_file, "wb") as f:
            f.write(r["data"])
        if not r["cache_hit"]:
            cache[key] = r["learned"]
        return True

    # -------------------------------------------------------------- PNG
    def compress_png_with_target_size(self, original_image, output_file, params: CompressionParams) -> bool:
        """ImageCompressionPng.compressPngWithTargetSize: fit into the
        (minWidth x minHeight) box with the bilinear scaler, write PNG."""
        if original_image is None:
            raise TypeError("originalImage must not be null")
        if output_file is None:
            raise TypeError("outputFile must not be null")
        if params is None:
            raise TypeError("params must not be null")
        resized = self.png_resize(original_image, params)
        if resized is None:
            return False
        from .pngio import write_png
        write_png(output_file, resized)
        return True

    def png_resize(self, original_image, params: CompressionParams):
        """The device part of compressPngWithTargetSize (ImageCompressionPng.java:
        45-67): None when the image already fits the (minWidth x minHeight) box,
        else the bilinear resize by min(minWidth/w, minHeight/h)."""
        if original_image is None:
            raise TypeError("originalImage must not be null")
        w, h = image_dims(original_image)
        if w <= params.min_width and h <= params.min_height:
            log.info("PNG 圖片尺寸 %dx%d 未超過目標 %dx%d，不處理。", w, h, params.min_width, params.min_height)
            return None
        scale = min(params.min_width / w, params.min_height / h)
        return self.resize_image(original_image, scale)

    def png_fit_batch(self, images, params: CompressionParams, fmts=None):
        """The device part of compressPngWithTargetSize for a group of images
        in one launch (icx_png_fit_batch): per image None when it already
        fits the (minWidth x minHeight) box (ImageCompressionPng.java:49-53),
        else the bilinear resize by min(minWidth/w, minHeight/h) (:57-66),
        keeping the raster type (ImageTools.java:12-15)."""
        n = len(images)
        jobs = (N.PngFitJob * n)()
        keep, outs = [], [None] * n
        for i, im in enumerate(images):
            img, k = _image_struct(im, fmts[i] if fmts else None)
            keep.append(k)
            j = jobs[i]
            j.src = img
            j.min_width, j.min_height = int(params.min_width), int(params.min_height)
            if img.width <= params.min_width and img.height <= params.min_height:
                continue
            dw, dh = scaled_dims(img.width, img.height,
                                 min(params.min_width / img.width, params.min_height / img.height))
            outs[i] = _new_raster(dh, dw, img.fmt)
            j.dst, j.cap = _pixels(outs[i]).ctypes.data, _pixels(outs[i]).nbytes
        with self._lock:
            st = self._batch_call("png_fit", jobs, n)
        self._check(st, "icx_png_fit_batch")
        res = []
        for i in range(n):
            self._check(jobs[i].status, "icx_png_fit_batch job")
            res.append(outs[i] if jobs[i].resized else None)
        return res

    # -------------------------------------------------------------- A11 decode
    def decode_jpg_batch(self, datas, subsampling: int = 0, device_out: bool = False, infos=None):
        """Decode JPEG files (bytes / uint8 arrays / DeviceImage / CUDA uint8
        tensors) on the GPU: decodeImageWithSubsampling's read
        (ImageCompression.java:113-155).  subsampling 0 = the reference's
        rule.  Returns one (status, image) per file; image is (H, W, 3) BGR or
        (H, W) grey, a DeviceImage when device_out (it stays in HBM for the
        encoder), else numpy.  infos: the files' icx_jpeg_info results when the
        caller has them (the batch driver parsed every header already)."""
        n = len(datas)
        jobs = (N.DecodeJob * n)()
        keep, outs = [], [None] * n
        for i, d in enumerate(datas):
            if d is None:
                raise TypeError("data must not be null")
            if isinstance(d, PinnedBuffer):
                keep.append(d)
                jobs[i].data, jobs[i].len = d.ptr, d.size
            elif hasattr(d, "data_ptr"):
                keep.append(d)
                jobs[i].data, jobs[i].len = d.data_ptr(), d.numel()
            else:
                a = np.frombuffer(d, np.uint8) if isinstance(d, (bytes, bytearray, memoryview)) else d
                keep.append(a)
                jobs[i].data, jobs[i].len = a.ctypes.data, a.nbytes
            jobs[i].subsampling = int(subsampling)
            info = infos[i] if infos is not None else jpeg_info(_host_header(d))
            if info[0] == N.OK:
                _, w, h, nc = info
                s = subsampling if subsampling > 0 else subsampling_factor(w, h)
                # (CMYK / YCCK files decode to BGR too: k_dec_color)
                shape = (-(-h // s), -(-w // s), 3) if nc >= 3 else (-(-h // s), -(-w // s))
                if device_out:
                    out = DeviceImage(self, shape)
                    jobs[i].out, jobs[i].cap = out.data_ptr(), out.numel()
                else:
                    out = np.empty(shape, np.uint8)
                    jobs[i].out, jobs[i].cap = out.ctypes.data, out.nbytes
                outs[i] = out
            else:
                jobs[i].out, jobs[i].cap = None, 0
        with self._lock:
            st = self._batch_call("decode_jpg", jobs, n)
        self._check(st, "icx_decode_jpg_batch")
        return [(jobs[i].status, outs[i] if jobs[i].status == N.OK else None) for i in range(n)]

    def prepare_decode(self, datas, outputs, subsampling: int = 0):
        """A reusable decode job array over preallocated inputs/outputs
        (numpy arrays or CUDA tensors), for repeated timed runs (bench)."""
        return PreparedDecode(self, datas, outputs, subsampling)

    def decode_jpg(self, data, subsampling: int = 0, device_out: bool = False):
        st, img = self.decode_jpg_batch([data], subsampling, device_out)[0]
        self._check(st, "icx_decode_jpg")
        return img

    def debug_decode_cmyk(self, data) -> np.ndarray:
        """A 4-component JPEG's CMYK samples (H, W, 4) as libjpeg outputs them
        (icx_debug_decode_cmyk: YCCK through ycck_cmyk_convert)."""
        a = np.frombuffer(bytes(data), np.uint8)
        st, w, h, nc = jpeg_info(a)
        self._check(st, "icx_jpeg_info")
        out = np.empty((h, w, 4), np.uint8)
        self._check(self._lib.icx_debug_decode_cmyk(self._ctx, a.ctypes.data, a.nbytes, out.ctypes.data, out.nbytes),
                    "icx_debug_decode_cmyk")
        return out

    def debug_decode_coefs(self, data) -> np.ndarray:
        a = np.frombuffer(bytes(data), np.uint8)
        st, w, h, nc = jpeg_info(a)
        self._check(st, "icx_jpeg_info")
        nb = _scan_blocks(a)
        out = np.zeros((nb, 64), np.int16)
        st = self._lib.icx_debug_decode_coefs(self._ctx, a.ctypes.data, a.nbytes,
                                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), out.size)
        self._check(st, "icx_debug_decode_coefs")
        return out

    # -------------------------------------------------------------- parity / metrics
    def debug_fdct(self, image) -> np.ndarray:
        img, keep = _image_struct(image)
        nb = self._lib.icx_num_blocks(img.width, img.height, img.fmt)
        out = np.empty((nb, 64), np.int16)
        st = self._lib.icx_debug_fdct(self._ctx, ctypes.byref(img),
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), out.size)
        self._check(st, "icx_debug_fdct")
        return out

    def profile(self, on=True):
        self._check(self._lib.icx_profile_enable(self._ctx, 1 if on else 0), "icx_profile_enable")

    def set_table_layout(self, layout: int):
        """JPEG table marker layout of later encodes (icx_set_table_layout):
        N.TABLES_SEPARATE (default, 623-B header) or N.TABLES_GROUPED (607 B)."""
        self._check(self._lib.icx_set_table_layout(self._ctx, int(layout)), "icx_set_table_layout")

    def profile_reset(self):
        self._check(self._lib.icx_profile_reset(self._ctx), "icx_profile_reset")

    def profile_query(self, kernel: str) -> Dict[str, float]:
        n = ctypes.c_int64()
        ms = ctypes.c_double()
        u = ctypes.c_int64()
        self._check(self._lib.icx_profile_query(self._ctx, kernel.encode(), ctypes.byref(n), ctypes.byref(ms),
                                                ctypes.byref(u)), "icx_profile_query")
        return {"launches": n.value, "ms": ms.value, "units": u.value}


class Pool(Codec):
    """Several GPUs behind one libicx handle (icx_pool_*, include/icx.h): the
    batched calls - fit, png_fit_batch, decode_jpg_batch - split the images
    into per-device shares balanced by pixels, run them concurrently and
    return the results in the caller's order, as one Codec would.  Host
    buffers only (device_out / CUDA tensors belong with one device's Codec);
    single-image helpers run on the first device's context.  The shape of a
    JVM host that drives every GPU of the node from one process
    (CompressionBatch.java:64-88)."""

    supports_device_out = False  # decode_jpg_batch returns host frames (the pipeline asks for those)

    def __init__(self, devices):
        self._lib = N.load()
        self._pool = ctypes.c_void_p()
        arr = (ctypes.c_int32 * len(devices))(*devices)
        st = self._lib.icx_pool_create(arr, len(devices), ctypes.byref(self._pool))
        if st != N.OK:
            raise N.IcxError(st, f"icx_pool_create({list(devices)}) failed: "
                                 f"{self._lib.icx_status_string(st).decode()}")
        self.devices = list(devices)
        self.device = self.devices[0]
        self._ctx = ctypes.c_void_p(self._lib.icx_pool_context(self._pool, 0))
        self._lock = threading.Lock()

    def close(self):
        if self._pool:
            self._lib.icx_pool_destroy(self._pool)
            self._pool = ctypes.c_void_p()
            self._ctx = ctypes.c_void_p()

    def _batch_call(self, what, jobs, n):
        return getattr(self._lib, f"icx_pool_{what}_batch")(self._pool, jobs, n)

    def set_table_layout(self, layout: int):
        for i in range(self._lib.icx_pool_size(self._pool)):
            st = self._lib.icx_set_table_layout(self._lib.icx_pool_context(self._pool, i), int(layout))
            self._check(st, "icx_set_table_layout")

    def decode_jpg_batch(self, datas, subsampling: int = 0, device_out: bool = False, infos=None):
        if device_out:
            raise ValueError("a Pool decodes into host memory; use one device's Codec for device_out")
        return super().decode_jpg_batch(datas, subsampling, False, infos)


def jpeg_info(data):
    """(status, width, height, ncomp) from the JPEG header (host bytes)."""
    lib = N.load()
    a = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else data
    w, h, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    st = lib.icx_jpeg_info(a.ctypes.data, a.nbytes, ctypes.byref(w), ctypes.byref(h), ctypes.byref(n))
    return st, w.value, h.value, n.value


def _host_header(d):
    """Host bytes holding at least the JPEG header of d (a CUDA tensor is
    copied up to its SOS, in growing pieces)."""
    if isinstance(d, PinnedBuffer):
        return d.array
    if not hasattr(d, "data_ptr"):
        return np.frombuffer(d, np.uint8) if isinstance(d, (bytes, bytearray, memoryview)) else d
    n = min(d.numel(), 1 << 16)
    while True:
        a = d.numpy(n) if getattr(d, "icx_device", False) else d[:n].cpu().numpy()
        if n == d.numel() or jpeg_info(a)[0] != N.E_CORRUPT:
            return a
        n = min(d.numel(), n * 4)


def _scan_blocks(a):
    """Blocks in the scan of a supported JPEG (MCU order incl. dummy blocks)."""
    i = 2
    while i + 4 <= len(a):
        if a[i] != 0xFF:
            i += 1
            continue
        m = int(a[i + 1])
        if m in (0xC0, 0xC1, 0xC2):
            h = int(a[i + 5]) << 8 | int(a[i + 6])
            w = int(a[i + 7]) << 8 | int(a[i + 8])
            nc = int(a[i + 9])
            if nc == 1:
                return -(-w // 8) * -(-h // 8)
            if nc == 4:  # CMYK / YCCK, every component 1x1
                return -(-w // 8) * -(-h // 8) * 4
            hs, vs = int(a[i + 11]) >> 4, int(a[i + 11]) & 15
            return -(-w // (8 * hs)) * -(-h // (8 * vs)) * (hs * vs + 2)
        if m == 0xFF or m == 0xD8:
            i += 1
            continue
        i += 2 + (int(a[i + 2]) << 8 | int(a[i + 3]))
    raise ValueError("no SOF0/SOF1/SOF2 marker")


def progressive_coefs(data) -> np.ndarray:
    """Coefficients of a progressive JPEG from the host entropy decode the
    device decoder's progressive path uses (icx_debug_progressive_coefs)."""
    lib = N.load()
    a = np.frombuffer(bytes(data), np.uint8)
    out = np.zeros((_scan_blocks(a), 64), np.int16)
    st = lib.icx_debug_progressive_coefs(a.ctypes.data, a.nbytes, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                         out.size)
    if st != N.OK:
        raise N.IcxError(st, "icx_debug_progressive_coefs")
    return out


def recovery_coefs(data) -> np.ndarray:
    """Coefficients of a sequential JPEG from the host entropy decode with
    IJG 6b's recovery that the device decoder runs for the files its own
    decode flags (icx_debug_recovery_coefs)."""
    lib = N.load()
    a = np.frombuffer(bytes(data), np.uint8)
    out = np.zeros((_scan_blocks(a), 64), np.int16)
    st = lib.icx_debug_recovery_coefs(a.ctypes.data, a.nbytes, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                      out.size)
    if st != N.OK:
        raise N.IcxError(st, "icx_debug_recovery_coefs")
    return out


def quality_tables(quality: float):
    lib = N.load()
    lum = (ctypes.c_uint16 * 64)()
    chrom = (ctypes.c_uint16 * 64)()
    lib.icx_quality_tables(_f32(quality), lum, chrom)
    return list(lum), list(chrom)


def subsampling_factor(width: int, height: int) -> int:
    return N.load().icx_subsampling_factor(width, height)


def scaled_dims(width: int, height: int, scale: float):
    w = ctypes.c_int32()
    h = ctypes.c_int32()
    N.load().icx_scaled_dims(width, height, float(scale), ctypes.byref(w), ctypes.byref(h))
    return w.value, h.value


class PreparedBatch:
    """icx_fit_job array built once and re-run (outputs overwritten each run)."""

    def __init__(self, codec, images, target, quality, cached=None, outputs=None):
        self.codec = codec
        self.n = len(images)
        self.jobs = (N.FitJob * self.n)()
        self._keep = []
        for i, im in enumerate(images):
            img, k = _image_struct(im)
            self._keep.append(k)
            j = self.jobs[i]
            j.img = img
            j.target_max_size = int(target)
            j.quality = _f32(quality)
            c = cached[i] if cached else None
            if c is not None:
                j.has_cached = 1
                j.cached = N.LearnedParams(_f32(c.quality), float(c.scale))
            buf = outputs[i] if outputs is not None else np.empty(int(target) + 1, np.uint8)
            self._keep.append(buf)
            j.out = buf.data_ptr() if hasattr(buf, "data_ptr") else buf.ctypes.data
            j.cap = buf.numel() if hasattr(buf, "numel") else buf.nbytes

    def run(self):
        # icx_compress_jpg_batch, or icx_pool_compress_jpg_batch for a Pool
        st = self.codec._batch_call("compress_jpg", self.jobs, self.n)
        self.codec._check(st, "icx_compress_jpg_batch")
        return self

    def results(self):
        return [{"status": j.status, "success": bool(j.success), "cache_hit": bool(j.cache_hit),
                 "out_len": j.out_len, "encodes": j.encodes,
                 "learned": LearnedParams(j.learned.quality, j.learned.scale)} for j in self.jobs]


class PreparedDecode:
    """icx_decode_jpg_batch over fixed buffers: run() decodes all files again."""

    def __init__(self, codec, datas, outputs, subsampling=0):
        self.codec = codec
        n = len(datas)
        self.n = n
        self.jobs = (N.DecodeJob * n)()
        self.keep = list(datas) + list(outputs)
        for i, (d, o) in enumerate(zip(datas, outputs)):
            j = self.jobs[i]
            if hasattr(d, "data_ptr"):
                j.data, j.len = d.data_ptr(), d.numel()
            else:
                j.data, j.len = d.ctypes.data, d.nbytes
            if hasattr(o, "data_ptr"):
                j.out, j.cap = o.data_ptr(), o.numel()
            else:
                j.out, j.cap = o.ctypes.data, o.nbytes
            j.subsampling = int(subsampling)

    def run(self):
        with self.codec._lock:
            st = self.codec._batch_call("decode_jpg", self.jobs, self.n)
        self.codec._check(st, "icx_decode_jpg_batch")
        return [self.jobs[i].status for i in range(self.n)]
