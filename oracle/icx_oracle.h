/*
 * icx_oracle.h — CPU restatement of the reference's JPEG target-size path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product path (libicx.so) never links,
 * loads or calls it.
 *
 * What it restates (reference = PolloChang/image-compression @ 2025-07-25):
 *   A2  compressJpgWithTargetSize   ImageCompressionJpg.java:77-122
 *   A3  findBestQualityByBinarySearch ImageCompressionJpg.java:158-200
 *   A4  compressJpgToStream / tryCachedParams  :136-147, :216-238
 *   A5-A10 the JDK JPEG writer it calls (javax.imageio -> IJG libjpeg 6b):
 *          quality->tables, rgb_ycc_convert, edge expansion, h2v2_downsample,
 *          jpeg_fdct_islow, quantiser, encode_mcu_huff, marker writer
 *   A11 decodeImageWithSubsampling decimation rule  ImageCompression.java:137-155
 *   A12 ImageTools.resizeImage (Java2D bilinear)    ImageTools.java:7-26
 *   A13 CacheTools.createKey                         CacheTools.java:14-21
 *
 * Pinning: A5-A10 are checked byte for byte against libjpeg-turbo 3.1.4
 * golden files (tests/golden/, made by gen_golden.py); A3 against search
 * traces computed with that encoder.  A12 is "parity unpinned": no Java2D
 * exists in this container.
 */
#ifndef ICX_ORACLE_H
#define ICX_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* pixel formats, same numbering as include/icx.h */
enum { OR_BGR24 = 0, OR_RGB24 = 1, OR_GRAY8 = 2, OR_XRGB32 = 3, OR_ARGB32 = 4, OR_ABGR32 = 5, OR_RGBA32 = 6,
       OR_GRAY16 = 7 /* TYPE_USHORT_GRAY, native-endian uint16 */ };

/* A6: JDK quality -> natural-order tables (JPEG.convertToLinearQuality +
 * JPEGQTable.getScaledInstance(lin, true)). */
void oracle_qtables(float q, uint16_t lum[64], uint16_t chrom[64]);

/* Number of 8x8 blocks in the scan (incl. libjpeg's dummy blocks). */
long oracle_num_blocks(int w, int h, int fmt);

/* A7-A9 without quantisation: raw jpeg_fdct_islow output (x8 scaled), one
 * 64-entry block per scan block, MCU order (Y0 Y1 Y2 Y3 Cb Cr), coefficients
 * in zig-zag order.  Dummy blocks carry AC=0 and the DC of the block libjpeg
 * copies it from.  coefs must hold oracle_num_blocks()*64 entries. */
long oracle_fdct(const uint8_t* px, int w, int h, int stride, int fmt, int16_t* coefs);

/* A4: one baseline JPEG encode at quality q.  Returns 0 on success, 4 when
 * cap is too small (*len = needed size), 1 on invalid input. */
int oracle_encode(const uint8_t* px, int w, int h, int stride, int fmt, float q,
                  uint8_t* out, size_t cap, size_t* len);

/* Table marker layout (A5/A10, SURVEY.md §7 hard part 2): 0 = one DQT / DHT
 * segment per table (libjpeg 6b jcmarker.c: 623 B colour / 328 B grey
 * header, the default), 1 = all tables of a kind in one segment (607 / 324 B).
 * Process-wide. */
void oracle_set_table_layout(int grouped);

/* A3: binary search.  Trial qualities/sizes are reported (up to 8). */
float oracle_find_best_quality(const uint8_t* px, int w, int h, int stride, int fmt,
                               int64_t target, float q0,
                               float* trial_q, int64_t* trial_size, int* ntrials);

/* A12: bilinear resize (Java2D TransformHelper fixed-point semantics). */
int oracle_resize(const uint8_t* src, int sw, int sh, int sstride, int fmt,
                  uint8_t* dst, int dw, int dh, int dstride);
/* A12 for TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY sources: src = one palette
 * index per byte (a 1/2/4-bit raster unpacked), pal = its colour map
 * (0xAARRGGBB).  dst = one index per byte into the DEFAULT map of a new
 * BufferedImage of that type (oracle_default_palette: binary 0 -> the 6x6x6
 * cube + grey ramp, 1 -> black/white), dithered as Java2D's ByteIndexed
 * store does (binary: no dither).  Parity unpinned (no JDK). */
int oracle_resize_indexed(const uint8_t* src, int sw, int sh, int sstride, const uint32_t* pal, int binary,
                          uint8_t* dst, int dw, int dh, int dstride);
void oracle_default_palette(int binary, uint32_t pal[256], int* n);
void oracle_inverse_cube(const uint32_t* cmap, int n, uint8_t cube[32768]);
void oracle_dither_tables(int cmapsize, int8_t red[64], int8_t green[64], int8_t blue[64]);

/* (int)(w*scale) clamped to >= 1, per ImageTools.java:8-9 */
void oracle_scaled_dims(int w, int h, double scale, int* dw, int* dh);

/* A2 (+ A4 cache path).  have_cached selects tryCachedParams first.
 * Returns 1 on success (out/len/best_q/best_scale set), 0 if no (q, scale)
 * fits, <0 on error.  *encodes counts every full encode performed, the
 * reference's cost unit.  cached_hit is set when the cached params were used. */
int oracle_compress_jpg_with_target_size(const uint8_t* px, int w, int h, int stride, int fmt,
                                         int64_t target, float q0,
                                         int have_cached, float cached_q, double cached_scale,
                                         uint8_t* out, size_t cap, size_t* len,
                                         float* best_q, double* best_scale,
                                         int* encodes, int* cached_hit);

/* A11 subsampling factor: maxDim>4096 ? highestOneBit(floor(maxDim/4096)) : 1 */
int oracle_subsampling(int w, int h);

/* A13 cache key */
void oracle_create_key(int w, int h, int64_t file_size, int* wb, int* hb, int64_t* sb);

/* Thread-parallel batch of A2 over n images (the reference's fixed thread
 * pool, CompressionBatch.java:64-88); returns the number of encodes done. */
long oracle_fit_batch(int n, const uint8_t* const* px, const int* w, const int* h,
                      const int* stride, int fmt, int64_t target, float q0,
                      int have_cached, float cached_q, double cached_scale,
                      int nthreads, int64_t* out_sizes, float* out_q, double* out_scale);

/* ---- A11 decode (icx_oracle_decode.c): IJG 6b baseline decompression as the
 * JDK JPEGImageReader runs it (ImageCompression.java:113-155), including
 * libjpeg's recovery from damaged entropy data (truncation, bad codes,
 * restart markers out of sequence).  Status codes as include/icx.h: 0 ok,
 * 4 cap too small, 5 not read here (the host reader reads it), 6 corrupt
 * (the JDK reader throws), 8 refused (arithmetic / hierarchical / not 8-bit:
 * the JDK reader throws at read()). */
int oracle_jpeg_info(const uint8_t* jpg, size_t len, int* w, int* h, int* ncomp);
/* blocks in the scan (MCU order, dummy blocks included); -1 if unparsable */
long oracle_jpeg_num_blocks(const uint8_t* jpg, size_t len);
/* quantised coefficients after DC prediction, natural order, 64 per block */
int oracle_jpeg_coefs(const uint8_t* jpg, size_t len, int16_t* coefs, size_t nblocks);
/* decode + source subsampling s: ceil(W/s) x ceil(H/s), BGR24 or GRAY8, packed */
int oracle_jpeg_decode(const uint8_t* jpg, size_t len, int s, uint8_t* out, size_t cap, int* w,
                       int* h, int* fmt);
/* 3-component file: its luma samples alone, W x H (JCS_GRAYSCALE output) */
int oracle_jpeg_decode_luma(const uint8_t* jpg, size_t len, uint8_t* out, size_t cap, int* w, int* h);
/* 4-component (CMYK / YCCK) file: libjpeg's CMYK samples, W x H x 4 */
int oracle_jpeg_decode_cmyk(const uint8_t* jpg, size_t len, uint8_t* out, size_t cap, int* w, int* h);

#ifdef __cplusplus
}
#endif
#endif
