"""ctypes binding of libicx.so (the C ABI declared in include/icx.h).

The product path: every compute call goes through this library's HIP
kernels.  There is no CPU fallback; a missing or unloadable library raises
immediately (NativeLibraryError).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ICX_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libicx.so")

# icx_status
OK, E_INVALID, E_NOMEM, E_DEVICE, E_BUFFER, E_UNSUPPORTED, E_CORRUPT, E_NULL, E_REFUSED = range(9)
# icx_fmt (XRGB32/ARGB32: TYPE_INT_RGB/ARGB int rasters, ABGR32: TYPE_4BYTE_ABGR, RGBA32: PNG order,
# GRAY16: TYPE_USHORT_GRAY, uint16 samples)
# INDEXED8 / BINARY1: TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY, one colour-map index per byte + Image.palette
BGR24, RGB24, GRAY8, XRGB32, ARGB32, ABGR32, RGBA32, GRAY16, INDEXED8, BINARY1 = range(10)
CHANNELS = {BGR24: 3, RGB24: 3, GRAY8: 1, XRGB32: 4, ARGB32: 4, ABGR32: 4, RGBA32: 4, GRAY16: 1, INDEXED8: 1,
            BINARY1: 1}
BYTES_PER_PX = {**CHANNELS, GRAY16: 2}
# icx_set_table_layout: one DQT/DHT segment per table (623 B header) / all in one (607 B)
TABLES_SEPARATE, TABLES_GROUPED = 0, 1

EXPORTS = [
    "icx_abi_version", "icx_create", "icx_destroy", "icx_status_string", "icx_last_error",
    "icx_quality_tables", "icx_create_key", "icx_subsampling_factor", "icx_scaled_dims",
    "icx_jpeg_header_size", "icx_jpeg_header_size_layout", "icx_default_palette", "icx_inverse_colour_map",
    "icx_dither_tables", "icx_set_table_layout", "icx_compress_jpg_to_stream", "icx_find_best_quality",
    "icx_compress_jpg_with_target_size", "icx_compress_jpg_batch", "icx_resize_image",
    "icx_resize_bilinear", "icx_png_fit", "icx_num_blocks", "icx_debug_fdct",
    "icx_profile_enable", "icx_profile_reset", "icx_profile_query",
    "icx_jpeg_info", "icx_decode_jpg", "icx_decode_jpg_batch", "icx_debug_decode_coefs",
    "icx_debug_progressive_coefs", "icx_debug_recovery_coefs",
    "icx_device_alloc", "icx_device_free", "icx_memcpy", "icx_host_alloc", "icx_host_free",
    "icx_png_bound", "icx_png_encode", "icx_png_fit_batch",
    "icx_pool_create", "icx_pool_destroy", "icx_pool_size", "icx_pool_context", "icx_pool_compress_jpg_batch",
    "icx_pool_decode_jpg_batch", "icx_pool_png_fit_batch",
    "icx_device_count", "icx_debug_self_check_image", "icx_debug_corrupt_constants", "icx_upload",
    "icx_debug_decode_cmyk", "icx_stage_files",
]


# entry points added within ABI version 4 (round 5); the rest are required
LATER = {"icx_device_count", "icx_debug_self_check_image", "icx_debug_corrupt_constants", "icx_upload",
         "icx_debug_decode_cmyk", "icx_stage_files"}


class NativeLibraryError(RuntimeError):
    pass


class IcxError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__(f"icx status {status}: {msg}")


class Image(ctypes.Structure):
    _fields_ = [("px", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("stride", ctypes.c_int32), ("fmt", ctypes.c_int32),
                ("palette", ctypes.c_void_p), ("palette_len", ctypes.c_int32)]


class LearnedParams(ctypes.Structure):
    _fields_ = [("quality", ctypes.c_float), ("scale", ctypes.c_double)]


class SimilarityKey(ctypes.Structure):
    _fields_ = [("width_bucket", ctypes.c_int32), ("height_bucket", ctypes.c_int32),
                ("size_bucket", ctypes.c_int64)]


class FitJob(ctypes.Structure):
    _fields_ = [("img", Image), ("target_max_size", ctypes.c_int64), ("quality", ctypes.c_float),
                ("has_cached", ctypes.c_int32), ("cached", LearnedParams),
                ("out", ctypes.c_void_p), ("cap", ctypes.c_size_t),
                ("success", ctypes.c_int32), ("cache_hit", ctypes.c_int32),
                ("out_len", ctypes.c_size_t), ("learned", LearnedParams),
                ("encodes", ctypes.c_int32), ("status", ctypes.c_int32)]


class PngFitJob(ctypes.Structure):
    _fields_ = [("src", Image), ("min_width", ctypes.c_int32), ("min_height", ctypes.c_int32),
                ("dst", ctypes.c_void_p), ("cap", ctypes.c_size_t),
                ("out_w", ctypes.c_int32), ("out_h", ctypes.c_int32), ("resized", ctypes.c_int32),
                ("status", ctypes.c_int32)]


class StageJob(ctypes.Structure):
    """icx_stage_job (include/icx.h): one file of icx_stage_files."""
    _fields_ = [("path", ctypes.c_char_p), ("min_size", ctypes.c_int64), ("min_width", ctypes.c_int32),
                ("min_height", ctypes.c_int32), ("exists", ctypes.c_int32), ("size", ctypes.c_int64),
                ("read_errno", ctypes.c_int32), ("jpeg_status", ctypes.c_int32), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("ncomp", ctypes.c_int32), ("dev", ctypes.c_void_p),
                ("status", ctypes.c_int)]


class DecodeJob(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t), ("subsampling", ctypes.c_int32),
                ("out", ctypes.c_void_p), ("cap", ctypes.c_size_t),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("fmt", ctypes.c_int32),
                ("src_width", ctypes.c_int32), ("src_height", ctypes.c_int32),
                ("out_len", ctypes.c_size_t), ("status", ctypes.c_int32)]


_lib = None


def load():
    """Load libicx.so once; raise NativeLibraryError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(f"libicx.so not built at {LIB_PATH}; run __graft_entry__.build()")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    c = ctypes
    P = c.POINTER
    sig = {
        "icx_abi_version": (c.c_int, []),
        "icx_create": (c.c_int, [c.c_int, P(c.c_void_p)]),
        "icx_device_count": (c.c_int32, []),
        "icx_debug_self_check_image": (None, [c.c_int32, c.c_void_p, P(c.c_uint64), P(c.c_int64)]),
        "icx_debug_corrupt_constants": (c.c_int, [c.c_int32, c.c_int32]),
        "icx_upload": (c.c_int, [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]),
        "icx_debug_decode_cmyk": (c.c_int, [c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t]),
        "icx_stage_files": (c.c_int, [c.c_void_p, P(StageJob), c.c_int32]),
        "icx_destroy": (None, [c.c_void_p]),
        "icx_status_string": (c.c_char_p, [c.c_int]),
        "icx_last_error": (c.c_char_p, [c.c_void_p]),
        "icx_quality_tables": (None, [c.c_float, P(c.c_uint16), P(c.c_uint16)]),
        "icx_create_key": (None, [c.c_int32, c.c_int32, c.c_int64, P(SimilarityKey)]),
        "icx_subsampling_factor": (c.c_int32, [c.c_int32, c.c_int32]),
        "icx_scaled_dims": (None, [c.c_int32, c.c_int32, c.c_double, P(c.c_int32), P(c.c_int32)]),
        "icx_jpeg_header_size": (c.c_int32, [c.c_int32]),
        "icx_jpeg_header_size_layout": (c.c_int32, [c.c_int32, c.c_int32]),
        "icx_default_palette": (c.c_int32, [c.c_int32, P(c.c_uint32)]),
        "icx_inverse_colour_map": (None, [c.c_void_p, c.c_int32, c.c_void_p]),
        "icx_dither_tables": (None, [c.c_void_p]),
        "icx_set_table_layout": (c.c_int, [c.c_void_p, c.c_int32]),
        "icx_compress_jpg_to_stream": (c.c_int, [c.c_void_p, P(Image), c.c_float, c.c_void_p, c.c_size_t,
                                                 P(c.c_size_t)]),
        "icx_find_best_quality": (c.c_int, [c.c_void_p, P(Image), c.c_int64, c.c_float, P(c.c_float),
                                            P(c.c_float), P(c.c_int64), P(c.c_int32)]),
        "icx_compress_jpg_with_target_size": (c.c_int, [c.c_void_p, P(FitJob)]),
        "icx_compress_jpg_batch": (c.c_int, [c.c_void_p, P(FitJob), c.c_int32]),
        "icx_resize_image": (c.c_int, [c.c_void_p, P(Image), c.c_double, c.c_void_p, c.c_size_t,
                                       P(c.c_int32), P(c.c_int32)]),
        "icx_resize_bilinear": (c.c_int, [c.c_void_p, P(Image), c.c_void_p, c.c_int32, c.c_int32, c.c_int32]),
        "icx_png_fit": (c.c_int, [c.c_void_p, P(Image), c.c_int32, c.c_int32, c.c_void_p, c.c_size_t,
                                  P(c.c_int32), P(c.c_int32), P(c.c_int32)]),
        "icx_num_blocks": (c.c_int64, [c.c_int32, c.c_int32, c.c_int32]),
        "icx_debug_fdct": (c.c_int, [c.c_void_p, P(Image), P(c.c_int16), c.c_size_t]),
        "icx_profile_enable": (c.c_int, [c.c_void_p, c.c_int32]),
        "icx_profile_reset": (c.c_int, [c.c_void_p]),
        "icx_profile_query": (c.c_int, [c.c_void_p, c.c_char_p, P(c.c_int64), P(c.c_double), P(c.c_int64)]),
        "icx_jpeg_info": (c.c_int, [c.c_void_p, c.c_size_t, P(c.c_int32), P(c.c_int32), P(c.c_int32)]),
        "icx_decode_jpg": (c.c_int, [c.c_void_p, P(DecodeJob)]),
        "icx_decode_jpg_batch": (c.c_int, [c.c_void_p, P(DecodeJob), c.c_int32]),
        "icx_debug_decode_coefs": (c.c_int, [c.c_void_p, c.c_void_p, c.c_size_t, P(c.c_int16), c.c_size_t]),
        "icx_debug_progressive_coefs": (c.c_int, [c.c_void_p, c.c_size_t, P(c.c_int16), c.c_size_t]),
        "icx_debug_recovery_coefs": (c.c_int, [c.c_void_p, c.c_size_t, P(c.c_int16), c.c_size_t]),
        "icx_device_alloc": (c.c_int, [c.c_void_p, c.c_size_t, P(c.c_void_p)]),
        "icx_device_free": (c.c_int, [c.c_void_p, c.c_void_p]),
        "icx_memcpy": (c.c_int, [c.c_void_p, c.c_void_p, c.c_void_p, c.c_size_t]),
        "icx_host_alloc": (c.c_int, [c.c_void_p, c.c_size_t, P(c.c_void_p)]),
        "icx_host_free": (c.c_int, [c.c_void_p, c.c_void_p]),
        "icx_png_bound": (c.c_size_t, [P(Image)]),
        "icx_png_encode": (c.c_int, [P(Image), c.c_int32, c.c_void_p, c.c_size_t, P(c.c_size_t)]),
        "icx_png_fit_batch": (c.c_int, [c.c_void_p, P(PngFitJob), c.c_int32]),
        "icx_pool_create": (c.c_int, [P(c.c_int32), c.c_int32, P(c.c_void_p)]),
        "icx_pool_destroy": (None, [c.c_void_p]),
        "icx_pool_size": (c.c_int32, [c.c_void_p]),
        "icx_pool_context": (c.c_void_p, [c.c_void_p, c.c_int32]),
        "icx_pool_compress_jpg_batch": (c.c_int, [c.c_void_p, P(FitJob), c.c_int32]),
        "icx_pool_decode_jpg_batch": (c.c_int, [c.c_void_p, P(DecodeJob), c.c_int32]),
        "icx_pool_png_fit_batch": (c.c_int, [c.c_void_p, P(PngFitJob), c.c_int32]),
    }
    for name, (res, args) in sig.items():
        if name in LATER and not hasattr(lib, name):
            continue  # an older build (A/B runs load one through ICX_LIB)
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.icx_abi_version() != 5:
        raise NativeLibraryError("libicx ABI version mismatch")
    _lib = lib
    return lib
