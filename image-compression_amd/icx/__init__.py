"""icx — MI355X-native JPEG target-size compression (host side).

Every compute call goes to libicx.so (HIP kernels for gfx950) through the C
ABI in include/icx.h; see core.py for the mapping to the reference's classes.
"""
from ._native import BGR24, BINARY1, GRAY8, INDEXED8, RGB24, IcxError, NativeLibraryError, load  # noqa: F401
from .core import (Codec, Pool, CompressionParams, DeviceImage, CompressionReport, CompressionResult,  # noqa: F401
                   IndexedImage, LearnedParams, SimilarityKey, create_key, default_palette, quality_tables,
                   scaled_dims, subsampling_factor)
