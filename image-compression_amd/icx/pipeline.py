"""Per-image pipeline and batch driver around the GPU hot path.

Mirrors (reference = src/main/java/work/pollochang/compression/image/):
  core/ImageCompression.java:47-105    process_image          (gates, dispatch, result mapping)
  core/ImageCompression.java:107-165   decode_image_with_subsampling
  core/ImageCompression.java:167-183   compress_image_iteratively (format switch)
  CompressionBatch.java:41-148         CompressionBatch.execute

Differences that are design, not semantics:
  * the reference runs processImage on N CPU threads; here decoding runs on
    host threads while JPEG images are grouped into device batches (one
    icx_compress_jpg_batch launch sequence per group), one worker per GPU;
  * the learned-cache lookup for an image happens when its group is formed
    (the reference's lookups also race with other tasks' puts: results of
    both depend on completion order).
JPEG files the device decoder supports (baseline/extended Huffman, one
interleaved scan or grey, any restart interval; progressive Huffman files with
the same layouts — icx_jpeg_info) are only read and header-parsed on the host
threads; each device group decodes them on the GPU (icx_decode_jpg_batch: the
JDK reader's IJG 6b arithmetic plus source subsampling; a progressive file's
scans are entropy-decoded by libicx on host threads, its IDCT and colour run
on the device) straight into HBM tensors that the encoder then reads, so no
decoded pixel crosses PCIe (CMYK / YCCK JPEGs too, to BGR on the device).
Damaged sequential JPEGs (truncated scans, bad Huffman codes, restart markers
out of sequence) are decoded by libicx as the JDK's 6b reader decodes them
(its recovery, icx_seqdecode.cpp), so they compress as in the reference.
JPEGs that reader refuses (arithmetic coding, hierarchical, not 8-bit:
ICX_E_REFUSED) fail with FAILED_IO_ERROR after the dims gate, as its read()
throws.  Other files (lossless or progressive-CMYK JPEG, PNG, GIF, BMP, ...)
and JPEGs the device decoder rejects (an invalid table, a damaged progressive
file, a scan script the JDK would block-smooth) are decoded on the host with
libjpeg-turbo / Pillow (6b-lineage ISLOW IDCT + h2v2 fancy upsampling for
JPEG), a JPEG with the JDK source manager's fake EOI appended.
"""
import concurrent.futures as cf
import logging
import os
import queue
import sqlite3
import threading
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _native as N
from .core import (CompressionParams, CompressionReport, CompressionResult, create_key,
                   subsampling_factor)

log = logging.getLogger("icx.pipeline")


class StageTimes:
    """Seconds spent per stage of a CompressionBatch run, summed over the
    threads doing it (thread-seconds): where the host time of the files ->
    files path goes.  Stages: stat, read (file bytes into
    pinned memory), parse (JPEG header), host_decode (Pillow: PNG and files
    the device decoder refuses), queue_wait (a GPU worker idle for work),
    gpu_decode / gpu_fit / gpu_png (the batched device calls, wall time of
    the calling worker), write (JPEG file writes), png_write (filter + deflate
    + write)."""

    def __init__(self):
        self._lock = threading.Lock()
        self.seconds = {}
        self.calls = {}

    def add(self, name, dt):
        with self._lock:
            self.seconds[name] = self.seconds.get(name, 0.0) + dt
            self.calls[name] = self.calls.get(name, 0) + 1

    def as_dict(self):
        with self._lock:
            return {k: {"seconds": round(v, 4), "calls": self.calls[k]} for k, v in sorted(self.seconds.items())}


# The StageTimes of the CompressionBatch whose task this thread runs (per
# thread: two batches in one process time their own stages, and a batch's
# end does not cut off another's timing).
_tls = threading.local()


def _in_batch(stages, fn, *args, **kw):
    """Run fn(*args, **kw) on this thread with `stages` as its StageTimes."""
    prev = getattr(_tls, "stages", None)
    _tls.stages = stages
    try:
        return fn(*args, **kw)
    finally:
        _tls.stages = prev


class _StagedPool:
    """A thread pool whose tasks record into one batch's StageTimes."""

    def __init__(self, threads, stages):
        self.pool = cf.ThreadPoolExecutor(threads)
        self.stages = stages

    def submit(self, fn, *args, **kw):
        return self.pool.submit(_in_batch, self.stages, fn, *args, **kw)

    def shutdown(self, wait=True):
        self.pool.shutdown(wait=wait)


class _span:
    __slots__ = ("name", "t0", "st")

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.st = getattr(_tls, "stages", None)
        self.t0 = time.perf_counter() if self.st is not None else 0.0

    def __exit__(self, *exc):
        if self.st is not None:
            self.st.add(self.name, time.perf_counter() - self.t0)
        return False

# Pillow format -> javax.imageio reader SPI getFormatNames()[0].toLowerCase()
# (formats the JDK can read; anything else has no reader: readers.hasNext() == false)
IMAGEIO_FORMATS = {"JPEG": "jpeg", "PNG": "png", "GIF": "gif", "BMP": "bmp", "TIFF": "tif", "WBMP": "wbmp"}


@dataclass
class DecodedImage:
    """core/DecodedImage.java:7-16: pixels + the reader's format name.

    For a JPEG left to the device decoder, image is None until its group is
    decoded and `data` holds the file bytes."""
    image: Optional[np.ndarray]
    format_name: str
    width: int
    height: int
    subsampling: int
    data: Optional[bytes] = None
    ncomp: int = 3  # components of a JPEG left to the device decoder (its header, parsed once)

    @property
    def decoded_dims(self):
        """Dimensions after source subsampling (what reader.read(0, param) returns)."""
        s = self.subsampling
        return -(-self.width // s), -(-self.height // s)


def format_file_size(size: int) -> str:
    """FileTools.formatFileSize: 1024-based, '#,##0.#'."""
    if size <= 0:
        return "0"
    units = ["B", "KB", "MB", "GB", "TB"]
    import math
    g = min(int(math.log10(size) / math.log10(1024)), len(units) - 1)
    return f"{size / 1024 ** g:,.1f}".rstrip("0").rstrip(".") + " " + units[g]


def png_palette_info(path):
    """(bit depth, colour type, PLTE entries as 0xRRGGBB, tRNS bytes or None)
    of a PNG file, from its chunks before the first IDAT; None if not a PNG."""
    import struct
    with open(path, "rb") as f:
        if f.read(8) != b"\x89PNG\r\n\x1a\n":
            return None
        depth = ctype = None
        plte, trns = [], None
        while True:
            head = f.read(8)
            if len(head) < 8:
                break
            n, tag = struct.unpack(">I4s", head)
            if tag == b"IDAT" or tag == b"IEND":
                break
            body = f.read(n)
            f.read(4)
            if tag == b"IHDR":
                depth, ctype = body[8], body[9]
            elif tag == b"PLTE":
                plte = [(body[3 * i] << 16) | (body[3 * i + 1] << 8) | body[3 * i + 2] for i in range(n // 3)]
            elif tag == b"tRNS":
                trns = body
    return depth, ctype, plte, trns


def _indexed_raster(im, path):
    """The JDK PNG reader's raster for a palette PNG (colour type 3) or a
    1/2/4-bit grey PNG, else None (PNGImageReader.getImageTypes):
      - palette, 8 bits -> TYPE_BYTE_INDEXED; 1/2/4 bits -> TYPE_BYTE_BINARY;
        the IndexColorModel is PLTE padded to 2^depth entries with its last
        entry, alphas = tRNS padded with 255 (none without tRNS);
      - grey 1/2/4 bits -> TYPE_BYTE_BINARY with the ramp i * 255 / (2^depth - 1)."""
    from .core import IndexedImage
    info = png_palette_info(path)
    if info is None:
        return None
    depth, ctype, plte, trns = info
    if ctype == 3 and plte:
        n = 1 << depth
        rgb = [plte[i] if i < len(plte) else plte[-1] for i in range(n)]
        alpha = [trns[i] if trns is not None and i < len(trns) else 255 for i in range(n)]
        pal = np.array([(a << 24) | c for a, c in zip(alpha, rgb)], np.uint32)
        idx = np.asarray(im.convert("P") if im.mode != "P" else im, dtype=np.uint8)
        return IndexedImage(idx, pal, N.INDEXED8 if depth == 8 else N.BINARY1)
    if ctype == 0 and depth in (1, 2, 4):
        n = 1 << depth
        pal = np.array([0xff000000 | (i * 255 // (n - 1)) * 0x010101 for i in range(n)], np.uint32)
        grey = np.asarray(im.convert("L") if im.mode == "1" else im, dtype=np.uint8)
        return IndexedImage((grey.astype(np.uint16) * (n - 1) // 255).astype(np.uint8), pal, N.BINARY1)
    return None


def _to_array(im, path=None):
    """Decoded raster as the BufferedImage type the JDK reader returns:
    TYPE_BYTE_GRAY (H, W), TYPE_USHORT_GRAY (H, W) uint16 for a 16-bit grey
    PNG, TYPE_3BYTE_BGR (H, W, 3) or, with an alpha channel, TYPE_4BYTE_ABGR
    (H, W, 4), and for palette PNGs and 1/2/4-bit grey PNGs an IndexedImage
    (TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY) - ImageTools.resizeImage keeps that
    type and the PNG is written back with it (ImageTools.java:12-15)."""
    if path is not None and im.format == "PNG":
        r = _indexed_raster(im, path)
        if r is not None:  # TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY (kept by ImageTools)
            return r
    mode = im.mode
    if mode == "L":
        return np.asarray(im, dtype=np.uint8)
    if mode in ("I;16", "I;16B", "I;16L") or (mode == "I" and im.format == "PNG"):
        # 16-bit grey PNG (Pillow: I;16, or I in older versions): TYPE_USHORT_GRAY
        return np.ascontiguousarray(np.asarray(im).astype(np.uint16))
    if mode in ("I", "F", "1"):  # (a 1-bit PNG is an IndexedImage, above)
        return np.asarray(im.convert("L"), dtype=np.uint8)
    if mode in ("LA", "PA"):
        # grey+alpha is TYPE_CUSTOM there, drawn into TYPE_INT_ARGB: RGBA out
        # (the JDK's linear-grey -> sRGB conversion of that case is not restated)
        mode, im = "RGBA", im.convert("RGBA")
    if mode == "RGBA":
        return np.ascontiguousarray(np.asarray(im, dtype=np.uint8)[:, :, ::-1])  # TYPE_4BYTE_ABGR
    if mode != "RGB":  # CMYK, and palette images of other formats (GIF, BMP: not the PNG path)
        im = im.convert("RGB")
    rgb = np.asarray(im, dtype=np.uint8)
    return np.ascontiguousarray(rgb[:, :, ::-1])  # TYPE_3BYTE_BGR


def _refused(path, w, h, params: CompressionParams):
    """A JPEG the reference's reader refuses (arithmetic coding, hierarchical,
    not 8-bit: icx_jpeg_info's ICX_E_REFUSED).  TwelveMonkeys reports its
    dimensions from the SOF, so the dims gate (ImageCompression.java:131)
    still applies; past it reader.read throws an IIOException (the JDK's 6b:
    JERR_ARITH_NOTIMPL / JERR_SOF_UNSUPPORTED / JERR_BAD_PRECISION), which
    processImage reports as FAILED_IO_ERROR (:94-96).  Returns False when
    the dims gate skips the file."""
    if w <= params.min_width or h <= params.min_height:
        log.debug("%s - 跳過: 圖片尺寸 %dx%d 未超過最小壓縮門檻 %dx%d", path, w, h, params.min_width,
                  params.min_height)
        return False
    raise OSError(f"{path}: JPEG flavour the reader refuses (arithmetic / hierarchical / not 8-bit)")


def _open_image(path):
    """Image.open for the host readers.  A JPEG (FF D8 FF: the JDK's JPEG
    reader SPI takes it, JPEGImageReaderSpi.canDecodeInput) is read with a
    fake EOI appended, as the JDK's source manager inserts one at end of
    stream (imageioJPEG.c imageio_fill_input_buffer): a truncated scan then
    decodes with libjpeg's zero fill instead of raising.  A JPEG the host
    reader cannot open raises OSError: its reader was found, reading failed."""
    import io
    from PIL import Image
    with open(path, "rb") as f:
        head = f.read(3)
    if head != b"\xff\xd8\xff":
        return Image.open(path)
    with open(path, "rb") as f:
        data = f.read()
    try:
        return Image.open(io.BytesIO(data + b"\xff\xd9"))
    except (Image.UnidentifiedImageError, ValueError, SyntaxError) as e:
        raise OSError(f"{path}: unreadable JPEG ({e})") from e


def _device_jpeg(input_path, params: CompressionParams, reader=None):
    """The file bytes (read by `reader`: into pinned host memory when the codec
    provides it, and then pushed to the GPU by the reader's upload()) and
    header of a JPEG the device decoder supports, else None."""
    from .core import jpeg_info
    with _span("read"):
        if reader is None:
            with open(input_path, "rb") as f:
                data = f.read()
        else:
            data = reader(input_path)
    head = data[:2] if isinstance(data, bytes) else bytes(data[:2])
    if head != b"\xff\xd8":
        return None
    with _span("parse"):
        st, w, h, nc = jpeg_info(data if isinstance(data, bytes) else data.array)
    if st == N.E_REFUSED:
        _refused(input_path, w, h, params)  # raises, or returns False (the dims gate)
        return False
    if st != N.OK:
        return None
    if w > params.min_width and h > params.min_height and hasattr(reader, "upload"):
        with _span("upload"):
            data = reader.upload(data)
    if w <= params.min_width or h <= params.min_height:  # ImageCompression.java:131
        log.debug("%s - 跳過: 圖片尺寸 %dx%d 未超過最小壓縮門檻 %dx%d", input_path, w, h, params.min_width,
                  params.min_height)
        return False
    s = subsampling_factor(w, h)
    if s > 1:
        log.debug("%s - 對圖片應用二次取樣，比率: %d", os.path.basename(str(input_path)), s)
    return DecodedImage(None, "jpeg", w, h, s, data, nc)


class DeviceReader:
    """Reads JPEG files for the device decoder and pushes their bytes to the
    GPU that will decode them, on the reader thread (icx_upload: a copy
    stream of the codec's own, concurrent with the kernels of the groups
    already formed), so the decode calls of the GPU workers read
    device-resident files and carry no host-to-device copy (VERDICT r4 item
    2: the 7.8 GB of 1000 4K q95 files crossed PCIe inside the decode calls,
    serial with their kernels).  A file goes to the device with the fewest
    bytes assigned so far; the pinned staging buffer (portable: DMA-able to
    every GPU) goes back to the pool as soon as the copy is done."""

    def __init__(self, codecs):
        self.by_dev = {}
        for c in codecs:
            self.by_dev.setdefault(c.device, c)
        self.devices = sorted(self.by_dev)
        self.assigned = {d: 0 for d in self.devices}
        self.lock = threading.Lock()
        self.mean_size = 4 << 20  # running mean of staged file sizes (the estimate a chunk reserves)
        self.staged = 0

    def __call__(self, path):
        from .core import PinnedBuffer
        return PinnedBuffer.read_file(self.by_dev[self.devices[0]], path)

    def pick(self, nbytes):
        """The device with the fewest bytes assigned so far (nbytes more now)."""
        with self.lock:
            d = min(self.devices, key=lambda k: self.assigned[k])
            self.assigned[d] += nbytes
        return d

    def stage(self, pairs, params, output_dir):
        """processImage up to the decode for a chunk of (index, path) pairs,
        staged natively (icx_stage_files: stat, read, header parse, dims gate
        and the copy to HBM without the interpreter lock) on one device;
        returns their _Items.  Files that are not device JPEGs go through
        _prepare's host readers."""
        from .core import DeviceImage
        n = len(pairs)
        # reserve the chunk's estimated bytes up front: reader threads that
        # pick at the same time then spread over the devices instead of all
        # taking the one with the fewest bytes so far; corrected
        # to the actual bytes below
        est = int(self.mean_size) * n
        d = self.pick(est)
        codec = self.by_dev[d]
        jobs = (N.StageJob * n)()
        keep = []
        for k, (_, path) in enumerate(pairs):
            b = os.fsencode(path)
            keep.append(b)
            jobs[k].path = b
            jobs[k].min_size = int(params.min_size_bytes)
            jobs[k].min_width, jobs[k].min_height = int(params.min_width), int(params.min_height)
        with _span("stage"):
            st = codec._lib.icx_stage_files(codec._ctx, jobs, n)
        if st != N.OK:
            log.warning("icx_stage_files: %s", codec.last_error())
        got = sum(int(jobs[k].size) for k in range(n) if jobs[k].dev)
        with self.lock:
            self.assigned[d] += got - est
            if got:
                self.staged += n
                self.mean_size += (got / n - self.mean_size) * min(1.0, n / self.staged)
        out = []
        for k, (i, path) in enumerate(pairs):
            j = jobs[k]
            dev = DeviceImage.adopt(codec, j.dev, (j.size,)) if j.dev else None
            out.append(_staged_item(i, path, j, dev, params, output_dir, self))
        return out

    def upload(self, buf):
        """The file's bytes in HBM of the device with the fewest bytes so far;
        if the device has no room for them (or the copy fails), the pinned
        host bytes themselves: the decode call then reads them from there
        (the file used to fail with FAILED_UNKNOWN)."""
        from .core import DeviceImage
        with self.lock:
            d = min(self.devices, key=lambda k: self.assigned[k])
            self.assigned[d] += buf.size
        codec = self.by_dev[d]
        dev = None
        try:
            dev = DeviceImage(codec, (buf.size,))
            codec._check(codec._lib.icx_upload(codec._ctx, dev.ptr, buf.ptr, buf.size), "icx_upload")
        except (N.IcxError, MemoryError) as e:
            log.warning("file upload to GPU %d failed (%s): decoding from host memory", d, e)
            if dev is not None:
                dev.free()
            with self.lock:
                self.assigned[d] -= buf.size
            return buf
        buf.free()
        return dev


def _staged_item(index, path, job, dev, params: CompressionParams, output_dir, reader) -> "_Item":
    """_prepare (ImageCompression.java:53-76) from a file icx_stage_files
    staged: the same gates, results and log lines in the same order; a file
    that is not a JPEG the device decoder takes goes to _prepare's readers."""
    it = _Item(index, path)
    if not job.exists:
        log.warning("%s - 檔案不存在或不可讀，跳過", path)
        it.report = CompressionReport(CompressionResult.SKIPPED_NOT_FOUND, 0, 0)
        return it
    it.original_size = int(job.size)
    if it.original_size <= params.min_size_bytes:
        log.info("%s - 跳過: 檔案大小 %s 未超過最小壓縮門檻 %s", path, format_file_size(it.original_size),
                 format_file_size(params.min_size_bytes))
        it.report = CompressionReport(CompressionResult.SKIPPED_CONDITION_NOT_MET, it.original_size,
                                      it.original_size)
        return it
    if job.read_errno:
        log.warning("%s - 處理圖片時發生 I/O 錯誤 (可能非支援格式或檔案損毀)", path)
        it.report = CompressionReport(CompressionResult.FAILED_IO_ERROR, it.original_size, 0)
        return it
    w, h = int(job.width), int(job.height)
    if dev is None:
        if job.jpeg_status == N.E_REFUSED:
            try:
                _refused(path, w, h, params)
            except OSError as e:
                log.warning("%s - 處理圖片時發生 I/O 錯誤 (可能非支援格式或檔案損毀)", path)
                log.debug("%s", e)
                it.report = CompressionReport(CompressionResult.FAILED_IO_ERROR, it.original_size, 0)
                return it
            it.report = CompressionReport(CompressionResult.FAILED_UNSUPPORTED_FORMAT, it.original_size,
                                          it.original_size)
            return it
        if job.jpeg_status == N.OK and (w <= params.min_width or h <= params.min_height):
            log.debug("%s - 跳過: 圖片尺寸 %dx%d 未超過最小壓縮門檻 %dx%d", path, w, h, params.min_width,
                      params.min_height)
            it.report = CompressionReport(CompressionResult.FAILED_UNSUPPORTED_FORMAT, it.original_size,
                                          it.original_size)
            return it
        return _prepare(index, path, output_dir, params, reader)  # PNG, other formats, unsupported JPEG
    s = subsampling_factor(w, h)
    if s > 1:
        log.debug("%s - 對圖片應用二次取樣，比率: %d", os.path.basename(str(path)), s)
    it.decoded = DecodedImage(None, "jpeg", w, h, s, dev, int(job.ncomp))
    it.output = os.path.join(str(output_dir), os.path.basename(str(path)))
    return it


def decode_image_with_subsampling(input_path, params: CompressionParams, file_size: int,
                                  device_jpeg=False) -> Optional[DecodedImage]:
    """ImageCompression.decodeImageWithSubsampling: None when the file is at or
    below -s, has no reader, or is not larger than (-w, -i) on both axes.
    device_jpeg: leave supported JPEGs undecoded for the GPU (DecodedImage.data)."""
    from PIL import Image
    if file_size <= params.min_size_bytes:
        log.info("%s - 跳過: 檔案大小 %s 未超過最小壓縮門檻 %s", input_path, format_file_size(file_size),
                 format_file_size(params.min_size_bytes))
        return None
    if device_jpeg:  # True, or a reader callable (path -> bytes / PinnedBuffer)
        d = _device_jpeg(input_path, params, None if device_jpeg is True else device_jpeg)
        if d is False:
            return None
        if d is not None:
            return d
    try:
        with _span("host_decode"):
            im = _open_image(input_path)
    except (Image.UnidentifiedImageError, ValueError):
        log.warning("%s - 找不到對應的圖片讀取器，跳過", input_path)
        return None
    with im:
        fmt = IMAGEIO_FORMATS.get(im.format or "")
        if fmt is None:
            log.warning("%s - 找不到對應的圖片讀取器，跳過", input_path)
            return None
        width, height = im.size
        if width <= params.min_width or height <= params.min_height:
            log.debug("%s - 跳過: 圖片尺寸 %dx%d 未超過最小壓縮門檻 %dx%d", input_path, width, height,
                      params.min_width, params.min_height)
            return None
        s = subsampling_factor(width, height)
        with _span("host_decode"):
            arr = _to_array(im, input_path)
    if s > 1:  # ImageReadParam.setSourceSubsampling(s, s, 0, 0): keep pixels (x*s, y*s)
        log.debug("%s - 對圖片應用二次取樣，比率: %d", os.path.basename(str(input_path)), s)
        from .core import IndexedImage
        if isinstance(arr, IndexedImage):
            arr = IndexedImage(arr.indices[::s, ::s], arr.palette, arr.fmt)
        else:
            arr = np.ascontiguousarray(arr[::s, ::s])
    return DecodedImage(arr, fmt, width, height, s)


@dataclass
class _Item:
    index: int
    path: str
    original_size: int = 0
    decoded: Optional[DecodedImage] = None
    report: Optional[CompressionReport] = None
    output: Optional[str] = None


def _prepare(index, path, output_dir, params, device_jpeg=False) -> _Item:
    """processImage up to and including the decode (ImageCompression.java:53-76)."""
    it = _Item(index, path)
    try:
        with _span("stat"):
            ok = os.path.exists(path) and os.access(path, os.R_OK)
        if not ok:
            log.warning("%s - 檔案不存在或不可讀，跳過", path)
            it.report = CompressionReport(CompressionResult.SKIPPED_NOT_FOUND, 0, 0)
            return it
        it.original_size = os.path.getsize(path)
    except OSError:
        it.report = CompressionReport(CompressionResult.FAILED_IO_ERROR, 0, 0)
        return it
    try:
        d = decode_image_with_subsampling(path, params, it.original_size, device_jpeg)
    except MemoryError:
        it.report = CompressionReport(CompressionResult.FAILED_OUT_OF_MEMORY, it.original_size, 0)
        return it
    except OSError:
        log.warning("%s - 處理圖片時發生 I/O 錯誤 (可能非支援格式或檔案損毀)", path)
        it.report = CompressionReport(CompressionResult.FAILED_IO_ERROR, it.original_size, 0)
        return it
    except Exception:
        log.exception("%s - 處理檔案時發生未知錯誤", path)
        it.report = CompressionReport(CompressionResult.FAILED_UNKNOWN, it.original_size, 0)
        return it
    if d is None:
        should = it.original_size > params.min_size_bytes
        it.report = CompressionReport(
            CompressionResult.FAILED_UNSUPPORTED_FORMAT if should else CompressionResult.SKIPPED_CONDITION_NOT_MET,
            it.original_size, it.original_size)
        return it
    it.decoded = d
    it.output = os.path.join(str(output_dir), os.path.basename(str(path)))
    return it


def _finish(it: _Item, success: bool):
    """Result mapping after compressImageIteratively (ImageCompression.java:79-93)."""
    if success:
        comp = os.path.getsize(it.output)
        ratio = 100.0 * (it.original_size - comp) / it.original_size if it.original_size else 0.0
        log.info("%s - 處理成功 -> %s (大小: %s -> %s, 節省: %.2f%%)", it.path, it.output,
                 format_file_size(it.original_size), format_file_size(comp), ratio)
        it.report = CompressionReport(CompressionResult.COMPRESSED_SUCCESS, it.original_size, comp)
    else:
        log.warning("%s - 無法在目標大小限制下完成壓縮", it.path)
        try:
            os.remove(it.output)
        except FileNotFoundError:
            pass
        it.report = CompressionReport(CompressionResult.FAILED_COMPRESSION, it.original_size, 0)
    it.decoded = None


def _fail(it: _Item, exc: BaseException):
    if isinstance(exc, MemoryError) or getattr(exc, "status", None) == N.E_NOMEM:
        res = CompressionResult.FAILED_OUT_OF_MEMORY
    elif isinstance(exc, OSError) or getattr(exc, "status", None) == N.E_DEVICE:
        res = CompressionResult.FAILED_IO_ERROR
    else:
        res = CompressionResult.FAILED_UNKNOWN
    log.error("%s - %s", it.path, exc)
    it.report = CompressionReport(res, it.original_size, 0)
    it.decoded = None


def _host_decode(path, s):
    """libjpeg-turbo decode + source subsampling (files the device decoder
    refused), with the JDK source manager's fake EOI (_open_image)."""
    with _open_image(path) as im:
        arr = _to_array(im)
    return np.ascontiguousarray(arr[::s, ::s]) if s > 1 else arr


def decode_group(codec, items: List[_Item]):
    """Decode the group's device-decodable JPEGs on the GPU (one batch, output
    left in HBM); a file the device decoder rejects is decoded on the host."""
    todo = [it for it in items if it.decoded.image is None]
    if not todo:
        return
    # a codec that decodes into host memory only (icx.Pool: its images may
    # land on any of its devices) hands back numpy frames, which its fit uploads
    kw = {}
    if hasattr(codec, "_ctx"):  # (icx.Codec / Pool: the headers were parsed by _device_jpeg)
        kw["infos"] = [(N.OK, it.decoded.width, it.decoded.height, it.decoded.ncomp) for it in todo]
    res = codec.decode_jpg_batch([it.decoded.data for it in todo], subsampling=0,
                                 device_out=getattr(codec, "supports_device_out", True), **kw)
    for it, (st, img) in zip(todo, res):
        it.decoded.data = None
        if st == N.OK:
            it.decoded.image = img
            continue
        log.warning("%s - GPU 解碼失敗 (icx status %d)，改用主機解碼", it.path, st)
        try:  # a corrupt file fails alone, as its own processImage task would
            it.decoded.image = _host_decode(it.path, it.decoded.subsampling)
        except MemoryError as e:
            _fail(it, e)
        except OSError:  # ImageCompression.java:101-103 (IOException from reader.read)
            log.warning("%s - 處理圖片時發生 I/O 錯誤 (可能非支援格式或檔案損毀)", it.path)
            it.report = CompressionReport(CompressionResult.FAILED_IO_ERROR, it.original_size, 0)
            it.decoded = None
        except Exception as e:
            _fail(it, e)


def _jpeg_write(it: _Item, data, success: bool, n=None):
    """Write a JPEG file: bytes, or the first n bytes of a PinnedBuffer, which
    goes back to the pool afterwards."""
    try:
        with _span("write"):
            with open(it.output, "wb") as f:
                f.write(data if n is None else memoryview(data.array)[:n])
        _finish(it, success)
    except Exception as e:
        _fail(it, e)
    finally:
        if n is not None:
            data.free()


def _pinned_outputs(codec, items: List[_Item], params: CompressionParams):
    """Pinned host buffers for the group's output files (a DMA each, no
    staging copy; the writer pool writes them from there and hands them
    back), or None: a codec without pinned memory, or an allocation failure
    (pinned memory exhausted), after which the fit returns host bytes."""
    if not hasattr(codec, "_ctx"):
        return None
    from .core import PinnedBuffer
    outs = []
    try:
        for it in items:
            # (a fitting file is <= -t; and no baseline JPEG reaches 10 bytes a pixel)
            outs.append(PinnedBuffer(codec, min(params.target_max_size_bytes + 1,
                                                10 * it.decoded.image.shape[0] * it.decoded.image.shape[1] + 65536)))
    except Exception as e:  # hipHostMalloc failed: host numpy buffers instead
        log.warning("pinned output buffers unavailable (%s); using host buffers", e)
        for o in outs:
            o.free()
        return None
    return outs


def compress_jpeg_group(codec, items: List[_Item], params: CompressionParams, cache, writer=None):
    """compressJpgWithTargetSize for a group of decoded JPEGs in one device batch
    (file writes on `writer`, a host thread pool, when given)."""
    try:
        with _span("gpu_decode"):
            decode_group(codec, items)
    except Exception as e:  # context-level failure: every image of the group fails alike
        for it in items:
            _fail(it, e)
        return
    finally:
        for it in items:  # the files' bytes are no longer needed: a reader may read ahead again
            rel = getattr(it, "release", None)
            if rel is not None:
                it.release = None
                rel()
    items = [it for it in items if it.report is None]  # files whose decode failed are done
    if not items:
        return
    keys = [create_key(it.decoded.image, it.original_size) for it in items]
    with cache.lock:
        if hasattr(cache, "refresh"):  # SharedCache: entries other ranks learned meanwhile
            cache.refresh()
        cached = [cache.get(k) for k in keys]
    outs = _pinned_outputs(codec, items, params)
    try:
        with _span("gpu_fit"):
            res = codec.fit([it.decoded.image for it in items], params.target_max_size_bytes, params.quality,
                            cached=cached, outputs=[o.array for o in outs] if outs else None)
            if outs:
                for r, o in zip(res, outs):
                    r["data"] = o if r["success"] and r["status"] == N.OK else None
                    if r["data"] is None:
                        o.free()
    except Exception as e:  # context-level failure: every image of the group fails alike
        for o in outs or ():
            o.free()
        for it in items:
            _fail(it, e)
        return
    for it, key, c, r in zip(items, keys, cached, res):
        try:
            if r["status"] == N.E_NOMEM:
                raise MemoryError("device out of memory")
            if r["status"] != N.OK:
                raise OSError(f"encode failed (icx status {r['status']})")
            if r["success"]:
                if not r["cache_hit"]:
                    with cache.lock:
                        cache[key] = r["learned"]
                it.decoded = None  # the frame's HBM buffer goes back to the pool now
                pinned = not isinstance(r["data"], (bytes, bytearray))
                if writer is not None:
                    writer.submit(_jpeg_write, it, r["data"], True, r["out_len"] if pinned else None)
                    continue
                _jpeg_write(it, r["data"], True, r["out_len"] if pinned else None)
                continue
            _finish(it, r["success"])
        except Exception as e:
            _fail(it, e)
    if hasattr(cache, "flush"):  # SharedCache: the group's new entries go out as one chunk
        with cache.lock:
            cache.flush()


def _png_write(it: _Item, resized):
    try:
        from .pngio import write_png
        with _span("png_write"):
            write_png(it.output, resized)
        _finish(it, True)
    except Exception as e:
        _fail(it, e)


def compress_png_item(codec, it: _Item, params: CompressionParams, writer=None):
    """compressPngWithTargetSize (ImageCompressionPng.java:37-75): the resize on
    the device, the PNG filter + deflate + file write on `writer` (a host
    thread pool) when given, so the device worker never waits on deflate."""
    try:
        if writer is None or not hasattr(codec, "png_resize"):
            _finish(it, codec.compress_png_with_target_size(it.decoded.image, it.output, params))
            return
        resized = codec.png_resize(it.decoded.image, params)
        if resized is None:
            _finish(it, False)
            return
        it.decoded = None
        writer.submit(_png_write, it, resized)
    except Exception as e:
        _fail(it, e)


def compress_png_group(codec, items: List[_Item], params: CompressionParams, writer=None):
    """compressPngWithTargetSize for a group of PNGs: the resizes in one device
    launch (icx_png_fit_batch), filter + deflate + file write per image on
    `writer`.  A codec without the batched entry point takes them one by one."""
    if writer is None or not hasattr(codec, "png_fit_batch"):
        for it in items:
            compress_png_item(codec, it, params, writer)
        return
    try:
        with _span("gpu_png"):
            res = codec.png_fit_batch([it.decoded.image for it in items], params)
    except Exception:  # a bad image fails alone: redo the group one by one
        for it in items:
            compress_png_item(codec, it, params, writer)
        return
    for it, resized in zip(items, res):
        if resized is None:  # ImageCompressionPng.java:49-53: already fits the box
            w, h = it.decoded.image.shape[1], it.decoded.image.shape[0]
            log.info("PNG 圖片尺寸 %dx%d 未超過目標 %dx%d，不處理。", w, h, params.min_width, params.min_height)
            _finish(it, False)
            continue
        it.decoded = None
        writer.submit(_png_write, it, resized)


def compress_image_iteratively(codec, it: _Item, params, cache):
    """The format switch (ImageCompression.java:167-183) for one item."""
    fmt = it.decoded.format_name
    if fmt in ("jpeg", "jpg"):
        compress_jpeg_group(codec, [it], params, cache)
    elif fmt == "png":
        compress_png_item(codec, it, params)
    else:
        log.warning("不支援的檔案格式: %s ...", fmt)
        _finish(it, False)


def process_image(input_path, output_dir, params: CompressionParams, cache, codec) -> CompressionReport:
    """ImageCompression.processImage for one file (codec used only to compress)."""
    from .cache import LockedDict
    if not hasattr(cache, "lock"):
        cache = LockedDict(cache) if cache is not None else LockedDict()
    it = _prepare(0, str(input_path), output_dir, params, hasattr(codec, "decode_jpg_batch"))
    if it.report is None:
        compress_image_iteratively(codec, it, params, cache)
    return it.report


@dataclass
class BatchReport:
    total: int = 0
    counts: dict = field(default_factory=lambda: {r: 0 for r in CompressionResult})
    original_size: int = 0
    compressed_size: int = 0
    cache_size: int = 0
    seconds: float = 0.0
    megapixels: float = 0.0
    stages: dict = field(default_factory=dict)  # StageTimes.as_dict() when the batch recorded them

    @property
    def success(self):
        return self.counts[CompressionResult.COMPRESSED_SUCCESS]

    @property
    def skipped(self):
        return self.counts[CompressionResult.SKIPPED_CONDITION_NOT_MET] + self.counts[CompressionResult.SKIPPED_NOT_FOUND]

    @property
    def failed(self):  # CompressionBatch.java:112-115
        return self.total - self.success - self.skipped

    def add(self, rep: CompressionReport):
        self.counts[rep.result] += 1
        self.original_size += rep.original_size
        self.compressed_size += rep.compressed_size

    def to_vector(self):
        return [self.total] + [self.counts[r] for r in CompressionResult] + \
            [self.original_size, self.compressed_size]

    @classmethod
    def from_vector(cls, v):
        b = cls()
        b.total = int(v[0])
        for i, r in enumerate(CompressionResult):
            b.counts[r] = int(v[1 + i])
        b.original_size, b.compressed_size = int(v[-2]), int(v[-1])
        return b

    def log(self):
        log.info("處理結果 -> 總計: %d, 成功壓縮: %d, 跳過不壓縮: %d, 失敗: %d", self.total, self.success,
                 self.skipped, self.failed)
        saved = self.original_size - self.compressed_size
        pct = 0.0 if self.original_size == 0 else saved / self.original_size * 100.0
        log.info(" 原始檔案總大小: %s", format_file_size(self.original_size))
        log.info(" 壓縮後檔案總大小: %s", format_file_size(self.compressed_size))
        log.info(" 共節省硬碟空間: %s", format_file_size(saved))
        log.info(" 總空間節省百分比: %.2f %%", pct)


def host_cores():
    """Host cores this process may use: the scheduler affinity set, capped by
    a cgroup CPU quota when one is set (on the GPU box the affinity mask shows
    the whole machine while the job's share is a quota).  Returns (cores, how
    it was determined).  The reference sizes its pool the same way:
    Runtime.availableProcessors() (CompressionBatch.java:64-68), which in a
    container honours both the affinity mask and the cgroup quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = "sched_getaffinity"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, -(-int(quota) // int(period)))
            if q < n:
                n, how = q, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    return n, how


def read_file_list(path) -> List[str]:
    with open(path, encoding="utf-8") as f:
        return [ln.strip() for ln in f if ln.strip()]


def _file_cost(path) -> int:
    try:
        return os.path.getsize(path)
    except OSError:
        return 0  # a missing file costs a stat (SKIPPED_NOT_FOUND)


def shard(lines, rank: int, world: int, cost=_file_cost):
    """File-list sharding across ranks, balanced by cost (longest processing
    time first): files in decreasing cost (the file size: decode bytes, and
    the pixels and trials that come with them — an 8K or a noise frame costs
    about twice a smooth 4K one), each to the rank with the least cost so far
    (ties: the lower rank, then the lower line index).  Every rank computes
    the same assignment from the same list, so no exchange is needed.
    Returns this rank's (line index, path) pairs in list order."""
    if world <= 1:
        return list(enumerate(lines))
    import heapq
    costs = [cost(p) for p in lines]
    order = sorted(range(len(lines)), key=lambda i: (-costs[i], i))
    heap = [(0, r) for r in range(world)]
    mine = []
    for i in order:
        load, r = heapq.heappop(heap)
        if r == rank:
            mine.append(i)
        heapq.heappush(heap, (load + costs[i] + 1, r))  # +1: empty files still cost a task
    mine.sort()
    return [(i, lines[i]) for i in mine]


class _Feed:
    """Work for the GPU workers, per device: JPEG items (their files already
    on that device), PNG items and single other items, put one by one by the
    reader side.  A worker takes a group once group_size items of a kind are
    waiting - or whatever is waiting once the readers are done - and then up
    to group_max of them: when the readers outpace the GPU, files pile up
    while a worker is busy and its next call is larger (fewer, bigger device
    calls: a 64-file call costs its device ~2x per frame what a 1000-frame
    call does); when the GPU outpaces the readers, groups stay
    at group_size and the device waits for files either way."""

    def __init__(self, keys, group_size, group_max):
        self.cv = threading.Condition()
        self.jpeg = {k: [] for k in keys}
        self.png = []   # any device
        self.other = {k: [] for k in keys}
        self.group_size, self.group_max = group_size, group_max
        self.closed = False

    def put(self, dev, kind, its):
        with self.cv:
            if kind == "jpeg":
                self.jpeg[dev].extend(its)
            elif kind == "png":
                self.png.extend(its)
            else:
                self.other[dev].extend(its)
            self.cv.notify_all()

    def waiting(self, dev):
        with self.cv:
            return len(self.jpeg[dev])

    def close(self):
        with self.cv:
            self.closed = True
            self.cv.notify_all()

    def take(self, dev):
        """(kind, items) for a worker of `dev`, or None once closed and empty."""
        with self.cv:
            while True:
                if self.other[dev]:
                    return "other", [self.other[dev].pop(0)]
                for kind, lst in (("jpeg", self.jpeg[dev]), ("png", self.png)):
                    if len(lst) >= self.group_size or (self.closed and lst):
                        grp = lst[:self.group_max]
                        del lst[:self.group_max]
                        return kind, grp
                if self.closed:
                    return None
                self.cv.wait()


class CompressionBatch:
    """CompressionBatch.execute: decode on host threads, compress on the GPU(s).

    codecs: one icx.Codec per device this process drives (a worker thread
    each); they share one L1 learned cache (the reference's ConcurrentHashMap)."""

    def __init__(self, file_list_path, save_dir, params: CompressionParams, time_out_hr: float = 24,
                 h2_cache_path="image-compression-cache", codecs=None, group_size: int = 64,
                 decode_threads: Optional[int] = None, rank: int = 0, world: int = 1,
                 device_decode: Optional[bool] = None, stage_times: bool = False, group_max: int = 0,
                 write_threads: int = 4):
        self.file_list_path = file_list_path
        self.save_dir = save_dir
        self.params = params
        self.time_out_hr = time_out_hr
        self.h2_cache_path = h2_cache_path
        self.codecs = codecs or []
        self.group_size = max(1, group_size)
        # a GPU worker that finds more than group_size files waiting takes up
        # to group_max of them in one device call (0: group_size, fixed groups)
        self.group_max = max(self.group_size, group_max)
        self.decode_threads = decode_threads or host_cores()[0]
        # JPEG output files are written by a few threads of their own: file
        # creation in one directory serialises on the directory, so more
        # writers only add contention (1000 x 875 KB files: 1 / 2 / 4 / 8
        # threads 0.33-0.45 / 0.20-0.23 / 0.13-0.15 / 0.13-0.14 s wall for
        # 0.3-0.4 / 0.4 / 0.5 / 0.9-1.0 thread-s), and the cores go to staging
        self.write_threads = max(1, min(write_threads, self.decode_threads))
        self.rank, self.world = rank, world
        self.stage_times = StageTimes() if stage_times else None
        # JPEG decode on the GPU when every codec can (the default for icx.Codec)
        if device_decode is None:
            device_decode = bool(self.codecs) and all(hasattr(c, "decode_jpg_batch") for c in self.codecs)
        self.device_decode = device_decode
        if device_decode and self.codecs and hasattr(self.codecs[0], "_ctx"):
            from .core import PinnedBuffer
            if all(getattr(c, "supports_device_out", False) and hasattr(c, "_ctx") for c in self.codecs):
                # files go to the decoding GPU from the reader threads (DeviceReader)
                self.device_decode = DeviceReader(self.codecs)
            else:
                c0 = self.codecs[0]  # portable pinned memory: DMA-able to every codec's GPU
                self.device_decode = lambda path: PinnedBuffer.read_file(c0, path)

    def execute(self, cache=None, save_cache: bool = True) -> BatchReport:
        from .cache import CacheManager, LockedDict
        os.makedirs(self.save_dir, exist_ok=True)
        mgr = None
        if cache is None:
            mgr = CacheManager(self.h2_cache_path)
        elif not hasattr(cache, "lock"):
            cache = LockedDict(cache)
        rep = BatchReport()
        prev_stages = getattr(_tls, "stages", None)
        _tls.stages = self.stage_times
        t0 = time.perf_counter()
        try:
            if mgr is not None:  # CompressionBatch.java:49-52 (inside the try: a schema error ends the batch)
                mgr.init_schema()
                cache = mgr.load_all_to_map()
                log.info("初始化 H2 二級快取，並載入至記憶體 L1 快取。")
            lines = read_file_list(self.file_list_path)
            mine = shard(lines, self.rank, self.world)
            rep.total = len(mine)
            deadline = t0 + self.time_out_hr * 3600.0
            items = self._run(mine, cache, deadline)
            for it in items:
                if it.report is not None:
                    rep.add(it.report)
            rep.megapixels = sum(getattr(it, "mp", 0.0) for it in items)
        except sqlite3.Error:  # CompressionBatch.java:134-139: logged, the batch ends
            log.exception("執行批次壓縮時發生未預期錯誤")
        finally:
            _tls.stages = prev_stages
            rep.seconds = time.perf_counter() - t0
            if self.stage_times is not None:
                rep.stages = self.stage_times.as_dict()
            rep.cache_size = len(cache) if cache is not None else 0
            if mgr is not None:
                if cache is not None:
                    log.info("記憶體中 L1 快取最終大小: %d", len(cache))
                    if save_cache:
                        mgr.save_all_from_map(cache)
                mgr.close()
        return rep

    def _run(self, mine, cache, deadline):
        # One work queue per device when the readers push files to a GPU
        # (DeviceReader): a group's files live in that GPU's memory, so only
        # that GPU's workers take it.  Otherwise one queue for every worker.
        per_dev = isinstance(self.device_decode, DeviceReader)
        keys = sorted({getattr(c, "device", None) for c in self.codecs}) if per_dev else [None]
        feed = _Feed(keys, self.group_size, self.group_max)
        rr = [0]

        def put(kind, its, dev=None):
            if dev is None:  # host-resident work: any device, round robin
                dev = keys[rr[0] % len(keys)]
                rr[0] += 1
            feed.put(dev, kind, its)

        def dev_of(it):
            d = it.decoded.data if it.decoded is not None else None
            return getattr(getattr(d, "codec", None), "device", None) if per_dev else None

        # read-ahead bound: file bytes read (and uploaded) but not yet decoded
        inflight = threading.Semaphore(max(4 * self.group_size * max(1, len(self.codecs)), 256)) if per_dev else None

        def slots(k):  # k read-ahead slots (fewer once the deadline has passed)
            got = 0
            while got < k:
                if inflight.acquire(timeout=0.5):
                    got += 1
                elif time.perf_counter() > deadline:
                    break
            return got

        def keep_slots(its, got):  # a slot per item until its decode, the rest back now
            for it in its:
                if got and it.decoded is not None and it.decoded.data is not None:
                    it.release = inflight.release  # after its decode (compress_jpeg_group)
                    got -= 1
            for _ in range(got):
                inflight.release()

        def prepare(i, p):
            got = slots(1) if inflight is not None else 0
            it = _prepare(i, p, self.save_dir, self.params, self.device_decode)
            if inflight is not None:
                keep_slots([it], got)
            return [it]

        def prepare_chunk(pairs):  # DeviceReader: native staging, one device per chunk
            got = slots(len(pairs))
            its = self.device_decode.stage(pairs, self.params, self.save_dir)
            keep_slots(its, got)
            return its

        done_items: List[_Item] = []
        lock = threading.Lock()

        writer = _StagedPool(self.decode_threads, self.stage_times)  # PNG filter + deflate + write
        jpeg_writer = _StagedPool(self.write_threads, self.stage_times)  # JPEG file writes

        def run_group(codec, kind, its):
            if kind == "jpeg":
                compress_jpeg_group(codec, its, self.params, cache, jpeg_writer)
            elif kind == "png":
                compress_png_group(codec, its, self.params, writer)
            else:
                for it in its:
                    compress_image_iteratively(codec, it, self.params, cache)

        def gpu_worker(codec):
            _tls.stages = self.stage_times
            dev = getattr(codec, "device", None) if per_dev else None
            while True:
                with _span("queue_wait"):
                    grp = feed.take(dev)
                if grp is None:
                    return
                kind, its = grp
                if time.perf_counter() > deadline:  # shutdownNow(): unfinished tasks are dropped
                    for it in its:
                        rel = getattr(it, "release", None)
                        if rel is not None:
                            it.release = None
                            rel()
                    continue
                try:
                    run_group(codec, kind, its)
                except BaseException as e:  # a worker never dies silently: the group's open items fail
                    log.exception("GPU worker: group of %d %s files failed", len(its), kind)
                    for it in its:
                        if it.report is None:
                            _fail(it, e)

        workers = [threading.Thread(target=gpu_worker, args=(c,), daemon=True) for c in self.codecs]
        for w in workers:
            w.start()
        with cf.ThreadPoolExecutor(self.decode_threads) as pool:
            if per_dev and hasattr(self.codecs[0], "_lib") and hasattr(self.codecs[0]._lib, "icx_stage_files"):
                step = max(1, min(8, self.group_size // 4))  # files per native staging call
                futs = [pool.submit(_in_batch, self.stage_times, prepare_chunk, mine[k:k + step])
                        for k in range(0, len(mine), step)]
            else:
                futs = [pool.submit(_in_batch, self.stage_times, prepare, i, p) for i, p in mine]
            try:
                for f in cf.as_completed(futs, timeout=max(0.0, deadline - time.perf_counter())):
                    for it in f.result():
                        with lock:
                            done_items.append(it)
                        if it.report is not None:
                            continue
                        it.mp = it.decoded.width * it.decoded.height / 1e6  # source pixels
                        if not self.codecs:
                            raise RuntimeError("no GPU codec available to compress decoded images")
                        fmt = it.decoded.format_name
                        if fmt in ("jpeg", "jpg"):
                            d = dev_of(it)
                            if d not in keys:  # a host-decoded JPEG: any device's group
                                d = min(keys, key=lambda k: feed.waiting(k))
                            put("jpeg", [it], d)
                        elif fmt == "png":
                            put("png", [it])
                        else:
                            put("other", [it])
            except cf.TimeoutError:
                log.warning("執行緒池等待逾時，部分任務可能未完成。")
                for f in futs:
                    f.cancel()
        feed.close()  # workers drain what is left, then stop
        for w in workers:
            w.join(timeout=max(1.0, deadline - time.perf_counter()))
        writer.shutdown(wait=True)
        jpeg_writer.shutdown(wait=True)
        return done_items
