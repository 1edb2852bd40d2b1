/*
 * icx.h — C-ABI of the MI355X-native JPEG target-size compression path.
 *
 * Drop-in boundary for PolloChang/image-compression's per-image encode hot
 * path.  The reference has no FFI: the hot path is reached through static
 * Java functions and the javax.imageio SPI.  Each entry point
 * below replaces one of those functions; the JNI/ctypes bindings a maintainer
 * would add are in INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Pixel/output pointers may be host memory
 *    or device (HBM) memory of the context's GPU; the library detects which.
 *    The caller owns every buffer; nothing is retained past return.
 *  - Errors are status codes (no exceptions cross the ABI).  The mapping to the
 *    reference's CompressionResult (CompressionResult.java:3-11) is:
 *      ICX_E_NOMEM  -> FAILED_OUT_OF_MEMORY   (ImageCompression.java:97-100)
 *      ICX_E_DEVICE -> FAILED_IO_ERROR        (ImageCompression.java:94-96)
 *      other errors -> FAILED_UNKNOWN         (ImageCompression.java:101-104)
 *    A NULL required argument returns ICX_E_NULL, the analogue of the
 *    NullPointerException contract tested in ImageCompressionPngTest.java:76-88.
 *  - Every function is thread-safe; calls on one context are serialised on
 *    its device stream (one context per GPU per process).
 *  - Floating-point parameters keep Java's types: quality is float32, scale
 *    is float64, so results match the reference's arithmetic bit for bit.
 */
#ifndef ICX_H
#define ICX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICX_ABI_VERSION 5  /* 2: four-byte pixel formats, icx_png_encode; 3: ICX_GRAY16, icx_png_fit_batch;
                              4: icx_set_table_layout, ICX_INDEXED8 / ICX_BINARY1 (icx_image.palette);
                              5: ICX_E_REFUSED; damaged JPEGs decoded with IJG 6b's recovery */

typedef struct icx_ctx icx_ctx;

typedef enum icx_status {
    ICX_OK = 0,
    ICX_E_INVALID = 1,     /* bad dimensions / format / argument value            */
    ICX_E_NOMEM = 2,       /* host or device allocation failed                    */
    ICX_E_DEVICE = 3,      /* HIP runtime error                                   */
    ICX_E_BUFFER = 4,      /* output capacity too small; *out_len = needed bytes  */
    ICX_E_UNSUPPORTED = 5, /* valid but unsupported input (e.g. progressive JPEG) */
    ICX_E_CORRUPT = 6,     /* malformed compressed input                          */
    ICX_E_NULL = 7,        /* required pointer argument is NULL                   */
    ICX_E_REFUSED = 8      /* a JPEG the reference's reader refuses at read():
                              arithmetic coding (SOF9-11), hierarchical (SOF5-7,
                              13-15), sample precision other than 8 bits; its
                              dimensions are still reported (TwelveMonkeys reads
                              the SOF itself), -> FAILED_IO_ERROR               */
} icx_status;

/* Pixel layouts.  ICX_BGR24 is java.awt.image.BufferedImage.TYPE_3BYTE_BGR,
 * the type the JDK JPEG reader returns for YCbCr JPEGs; ICX_GRAY8 is
 * TYPE_BYTE_GRAY (1-component JPEG).
 * Four-byte pixels (the PNG path: ImageTools.java:12-15 keeps the source
 * type, TYPE_CUSTOM -> TYPE_INT_ARGB / TYPE_INT_RGB) are accepted by the
 * resize / PNG entry points only; rows and px must be 4-byte aligned.  The
 * JPEG entry points return ICX_E_UNSUPPORTED for them (the JDK JPEG writer
 * refuses alpha rasters).  Byte order in memory (little-endian ints):
 *   ICX_XRGB32  TYPE_INT_RGB    int 0x00RRGGBB: B, G, R, 0 (alpha ignored, written 0)
 *   ICX_ARGB32  TYPE_INT_ARGB   int 0xAARRGGBB: B, G, R, A
 *   ICX_ABGR32  TYPE_4BYTE_ABGR bytes A, B, G, R (ImageIO's reading of an RGBA PNG)
 *   ICX_RGBA32  bytes R, G, B, A (PNG colour type 6 row order)
 * ICX_GRAY16 is TYPE_USHORT_GRAY (a 16-bit grey PNG as the JDK reads it):
 * native-endian uint16 samples, rows and px 2-byte aligned; resize / PNG
 * entry points only.  Java2D's bilinear loops carry it through 8-bit
 * IntArgbPre (UshortGray.h: the high byte in, gray * 257 out), and so does
 * icx_resize_image; icx_png_encode writes it as a 16-bit grey PNG.
 * ICX_INDEXED8 is TYPE_BYTE_INDEXED (an 8-bit palette PNG as the JDK reads
 * it) and ICX_BINARY1 TYPE_BYTE_BINARY (a 1/2/4-bit palette or grey PNG):
 * one colour-map index per byte (a packed raster unpacked), the colour map in
 * icx_image.palette (0xAARRGGBB, palette_len entries; <= 256, <= 16 for
 * BINARY1).  ImageTools.resizeImage keeps the type, so the resized image gets
 * Java2D's DEFAULT map of a new BufferedImage of that type (INDEXED8: the
 * 6x6x6 cube + grey ramp of icx_default_palette, dithered; BINARY1: black /
 * white): resize and PNG entry points only. */
typedef enum icx_fmt {
    ICX_BGR24 = 0,
    ICX_RGB24 = 1,
    ICX_GRAY8 = 2,
    ICX_XRGB32 = 3,
    ICX_ARGB32 = 4,
    ICX_ABGR32 = 5,
    ICX_RGBA32 = 6,
    ICX_GRAY16 = 7,
    ICX_INDEXED8 = 8,
    ICX_BINARY1 = 9
} icx_fmt;

/* A decoded image (BufferedImage).  stride in bytes. */
typedef struct icx_image {
    const uint8_t* px;
    int32_t width;
    int32_t height;
    int32_t stride;
    int32_t fmt; /* icx_fmt */
    const uint32_t* palette; /* ICX_INDEXED8 / ICX_BINARY1: host colour map (0xAARRGGBB), else ignored */
    int32_t palette_len;
} icx_image;

/* The colour map of `new BufferedImage(w, h, TYPE_BYTE_INDEXED)` (binary = 0:
 * 256 entries) or TYPE_BYTE_BINARY (binary = 1: 2 entries); returns the
 * entry count. */
int32_t icx_default_palette(int32_t binary, uint32_t pal[256]);
/* What Java2D derives from a colour map for storing into it: the inverse map
 * of 32x32x32 cells (AWT initCubemap, index = (r>>3)<<10 | (g>>3)<<5 | b>>3)
 * and the ordered-dither error tables of a 256-entry map
 * (make_dither_arrays: red, green, blue, [(y & 7) * 8 + (x & 7)]). */
void icx_inverse_colour_map(const uint32_t* pal, int32_t n, uint8_t cube[32768]);
void icx_dither_tables(int8_t err[3][64]);

/* learn/LearnedParams.java:8  record LearnedParams(float quality, double scale) */
typedef struct icx_learned_params {
    float quality;
    double scale;
} icx_learned_params;

/* learn/jpg/SimilarityKey.java:9  record SimilarityKey(int, int, long) */
typedef struct icx_similarity_key {
    int32_t width_bucket;
    int32_t height_bucket;
    int64_t size_bucket;
} icx_similarity_key;

/* ---------------------------------------------------------------- context */
/* One context per GPU per process: owns the HIP stream, workspace pool and
 * staging buffers.  device = HIP ordinal. */
icx_status icx_create(int device, icx_ctx** out);
void icx_destroy(icx_ctx* ctx);
const char* icx_status_string(icx_status s);

/* Several GPUs behind one handle, for a host process that drives every GPU of
 * the node (a JVM's CompressionBatch thread pool, CompressionBatch.java:64-88):
 * one context per listed device (ordinals may repeat: several contexts on one
 * GPU).  The pool's batched calls split the jobs into per-device shares
 * balanced by pixels (decode: compressed bytes), run them concurrently on one
 * host thread per device and fill in every job's results as the single-context
 * call would.  Pool calls take host buffers only (a job with a device pointer
 * gets ICX_E_INVALID); icx_pool_context(pool, i) is device i's own context for
 * device-resident work.  The return value is the first context-level failure,
 * else ICX_OK. */
typedef struct icx_pool icx_pool;
icx_status icx_pool_create(const int32_t* devices, int32_t ndev, icx_pool** out);
void icx_pool_destroy(icx_pool* pool);
int32_t icx_pool_size(const icx_pool* pool);
icx_ctx* icx_pool_context(icx_pool* pool, int32_t i);
/* GPUs visible to this process (0 when there are none): the CLI's default
 * device list when one process drives the node. */
int32_t icx_device_count(void);
/* icx_create's device self-check: the first context on
 * a device encodes a fixed 16x16 BGR24 and a fixed 16x16 GRAY8 frame at
 * quality 0.75 there and compares the files with known answers (length and
 * 64-bit FNV-1a digest, pinned against the CPU oracle by the tests); every
 * context compares the device's digest of the encoder's constant tables with
 * the host's (~0.1 ms).  A mismatch fails icx_create with ICX_E_DEVICE, so a
 * constant table missing or wrong on one GPU cannot silently corrupt that
 * GPU's output (ICX_SELF_CHECK=0 skips both).  Debug
 * helpers: the known-answer image (px: 16*16*3 or 16*16 bytes) and its
 * expected file; and a hook that overwrites (on = 1) or restores (on = 0)
 * the encoder's constant Huffman tables on `device`. */
void icx_debug_self_check_image(int32_t grey, uint8_t* px, uint64_t* digest, int64_t* len);
icx_status icx_debug_corrupt_constants(int32_t device, int32_t on);
/* Last error text recorded on this context (never NULL). */
const char* icx_last_error(const icx_ctx* ctx);
int icx_abi_version(void);

/* ------------------------------------------------------- pure host helpers */
/* A6: JPEG.convertToLinearQuality + JPEGQTable.K1Luminance/K2Chrominance
 * .getScaledInstance(lin, true), natural order; the tables the JDK writer
 * uses for setCompressionQuality(q) (ImageCompressionJpg.java:140-143). */
void icx_quality_tables(float quality, uint16_t lum[64], uint16_t chrom[64]);

/* A13: CacheTools.createKey (CacheTools.java:14-21). */
void icx_create_key(int32_t width, int32_t height, int64_t file_size, icx_similarity_key* key);

/* A11: ImageCompression.decodeImageWithSubsampling's factor
 * (ImageCompression.java:140-153): maxDim > 4096 ? highestOneBit(floor(maxDim/4096)) : 1. */
int32_t icx_subsampling_factor(int32_t width, int32_t height);

/* A12 dims: ImageTools.java:8-9, max(1, (int)(w*scale)). */
void icx_scaled_dims(int32_t width, int32_t height, double scale, int32_t* out_w, int32_t* out_h);

/* Exact JPEG file size this library writes for a given entropy-segment size
 * (headers + EOI).  Header layout: SOI, JFIF APP0, DQT per table, SOF0, DHT per
 * table, SOS (623 B for 3 components, 328 B for grey). */
int32_t icx_jpeg_header_size(int32_t fmt);

/* Marker layout of the writer's tables (A5; SURVEY.md §7 hard part 2: the
 * JDK's grouping cannot be checked without a JVM, so both are available).
 * ICX_TABLES_SEPARATE (default): one DQT segment per quantisation table and
 * one DHT segment per Huffman table, as libjpeg 6b's jcmarker.c writes the
 * tables the JDK hands it (623 / 328 B).  ICX_TABLES_GROUPED: every
 * quantisation table in one DQT segment and every Huffman table in one DHT
 * segment (607 / 324 B).  The entropy-coded data is the same; the size every
 * search decision compares against -t (ImageCompressionJpg.java:176) is not. */
enum { ICX_TABLES_SEPARATE = 0, ICX_TABLES_GROUPED = 1 };
int32_t icx_jpeg_header_size_layout(int32_t fmt, int32_t layout);
/* Layout of every later encode on this context (ICX_E_INVALID for others). */
icx_status icx_set_table_layout(icx_ctx* ctx, int32_t layout);

/* ------------------------------------------------------------- hot path */
/* A4  ImageCompressionJpg.compressJpgToStream (ImageCompressionJpg.java:136-147):
 * one baseline JPEG encode at float quality q.  Writes the complete file to
 * out (host or device).  ICX_E_BUFFER if cap < size (then *out_len = size). */
icx_status icx_compress_jpg_to_stream(icx_ctx* ctx, const icx_image* img, float quality,
                                      uint8_t* out, size_t cap, size_t* out_len);

/* A3  ImageCompressionJpg.findBestQualityByBinarySearch (:158-200).
 * Returns the best quality (or -1.0f) in *best_quality.  trial_q/trial_size
 * (each >= 8 entries, may be NULL) receive the trial sequence. */
icx_status icx_find_best_quality(icx_ctx* ctx, const icx_image* img, int64_t target_max_size,
                                 float initial_quality, float* best_quality, float* trial_q,
                                 int64_t* trial_size, int32_t* ntrials);

/* A2  ImageCompressionJpg.compressJpgWithTargetSize (:77-122), including the
 * cache-hit branch tryCachedParams (:216-238).  The Map<SimilarityKey,
 * LearnedParams> stays on the caller's side: pass cache.get(key) in `cached`
 * (has_cached = 1 on a hit); on return `learned` is what the reference would
 * cache.put (valid when success && !cache_hit). */
typedef struct icx_fit_job {
    /* inputs */
    icx_image img;
    int64_t target_max_size; /* CompressionParams.targetMaxSizeBytes */
    float quality;           /* CompressionParams.quality (search upper bound) */
    int32_t has_cached;
    icx_learned_params cached;
    uint8_t* out; /* host or device */
    size_t cap;
    /* outputs */
    int32_t success;   /* compressJpgWithTargetSize's return value */
    int32_t cache_hit; /* tryCachedParams wrote the file */
    size_t out_len;
    icx_learned_params learned;
    int32_t encodes;   /* trial encodes performed (cache probe + search trials) */
    icx_status status;
} icx_fit_job;

icx_status icx_compress_jpg_with_target_size(icx_ctx* ctx, icx_fit_job* job);

/* Batched A2 for throughput: the images are processed together, sharing
 * kernel launches.  Per-job results/status are filled in; the return value is
 * ICX_OK unless a context-level failure occurred. */
icx_status icx_compress_jpg_batch(icx_ctx* ctx, icx_fit_job* jobs, int32_t n);
icx_status icx_pool_compress_jpg_batch(icx_pool* pool, icx_fit_job* jobs, int32_t n);

/* A12  ImageTools.resizeImage (ImageTools.java:7-26): Java2D bilinear resize
 * to (max(1,(int)(w*scale)), max(1,(int)(h*scale))).  dst gets the same fmt,
 * tightly packed (stride = w*channels).  Alpha formats are interpolated in
 * premultiplied form and composited SrcOver onto the new (transparent)
 * image, as Java2D's TransformHelper + IntArgbPre mask blit do. */
icx_status icx_resize_image(icx_ctx* ctx, const icx_image* src, double scale, uint8_t* dst,
                            size_t cap, int32_t* out_w, int32_t* out_h);

/* Bilinear resize to explicit dims (dstride in bytes). */
icx_status icx_resize_bilinear(icx_ctx* ctx, const icx_image* src, uint8_t* dst, int32_t dst_w,
                               int32_t dst_h, int32_t dst_stride);

/* The resize step of ImageCompressionPng.compressPngWithTargetSize
 * (ImageCompressionPng.java:37-75): if w <= min_w && h <= min_h sets
 * *resized = 0 (the reference returns false); else scales by
 * min(min_w/w, min_h/h) into dst and sets *resized = 1. */
icx_status icx_png_fit(icx_ctx* ctx, const icx_image* src, int32_t min_width, int32_t min_height,
                       uint8_t* dst, size_t cap, int32_t* out_w, int32_t* out_h,
                       int32_t* resized);

/* Batched icx_png_fit: the resizes of all jobs share one launch (a group of
 * PNGs of a CompressionBatch, ImageCompressionPng.java:57-70 per image).
 * Per-job results/status are filled in; a job whose image already fits the
 * box gets resized = 0 and nothing written.  Sources and destinations may be
 * host or device memory.  Returns ICX_OK unless a context-level failure
 * occurred. */
typedef struct icx_png_fit_job {
    /* inputs */
    icx_image src;
    int32_t min_width, min_height; /* CompressionParams.minWidth / minHeight */
    uint8_t* dst;                  /* host or device; packed rows of out_w * channels (may be NULL
                                      for an image that already fits the box) */
    size_t cap;
    /* outputs */
    int32_t out_w, out_h;
    int32_t resized;               /* 0: the reference returns false (ImageCompressionPng.java:49-53) */
    icx_status status;
} icx_png_fit_job;
icx_status icx_png_fit_batch(icx_ctx* ctx, icx_png_fit_job* jobs, int32_t n);
icx_status icx_pool_png_fit_batch(icx_pool* pool, icx_png_fit_job* jobs, int32_t n);

/* The PNG write of ImageCompressionPng (ImageCompressionPng.java:70,
 * ImageIO.write(img, "png", file)) for host pixels: 8-bit grey (GRAY8), RGB
 * (BGR24/RGB24/XRGB32), RGBA (ARGB32/ABGR32/RGBA32) or 16-bit grey (GRAY16).
 * Restates OpenJDK's PNGImageWriter: per row RowFilter.filterRow's choice
 * (None costs the sum of the unsigned sample bytes; Sub, Up, Average and
 * Paeth the sum of |unwrapped int difference|; ties keep the lower type), one
 * zlib stream at `level` (0-9; -1 = the writer's default, 4) cut into IDAT
 * chunks of 32768 bytes.  Needs cap >= icx_png_bound(img); *out_len = file
 * bytes. */
size_t icx_png_bound(const icx_image* img);
icx_status icx_png_encode(const icx_image* img, int32_t level, uint8_t* out, size_t cap, size_t* out_len);

/* ------------------------------------------------------------- decode (A11) */
/* ImageCompression.decodeImageWithSubsampling (ImageCompression.java:107-165)
 * for JPEG: the JDK JPEGImageReader (IJG 6b: ISLOW IDCT, fancy upsampling,
 * ycc_rgb_convert) with ImageReadParam.setSourceSubsampling(s, s, 0, 0) —
 * pixels (x*s, y*s) of the full decode — and ignoreMetadata = true.
 * Baseline/extended-sequential Huffman JPEGs with one interleaved scan
 * (4:2:0, 4:2:2, 4:4:4, 4:4:0, 4:1:1; CMYK / YCCK with 1x1 components) or
 * one grey component, with or without restart intervals, and progressive
 * files of the same layouts.  Damaged sequential files decode as the JDK's
 * reader decodes them (IJG 6b's recovery: a truncated scan ends in grey MCUs,
 * a bad Huffman code reads as 0, restart markers out of sequence are
 * resynchronised), so a file is ICX_E_CORRUPT only where that reader throws.
 * ICX_E_REFUSED: arithmetic / hierarchical / not 8-bit (the reader throws at
 * read()); anything else returns ICX_E_UNSUPPORTED (another reader's file). */
typedef struct icx_decode_job {
    /* inputs */
    const uint8_t* data;   /* the whole JPEG file; host or device memory */
    size_t len;
    int32_t subsampling;   /* s >= 1; 0 = the reference's rule icx_subsampling_factor(w, h) */
    uint8_t* out;          /* host or device; rows of width*channels bytes, packed */
    size_t cap;
    /* outputs */
    int32_t width, height; /* decoded image: ceil(W/s) x ceil(H/s) */
    int32_t fmt;           /* ICX_BGR24 (TYPE_3BYTE_BGR) or ICX_GRAY8 (TYPE_BYTE_GRAY) */
    int32_t src_width, src_height; /* SOF dimensions (reader.getWidth(0)/getHeight(0)) */
    size_t out_len;        /* width*height*channels */
    icx_status status;
} icx_decode_job;

/* Header-only parse (host memory): SOF dimensions and components.  Returns
 * ICX_OK when the device decoder supports the file, ICX_E_UNSUPPORTED or
 * ICX_E_REFUSED (with the dimensions filled in) when it does not,
 * ICX_E_CORRUPT otherwise. */
icx_status icx_jpeg_info(const uint8_t* data, size_t len, int32_t* width, int32_t* height, int32_t* ncomp);

icx_status icx_decode_jpg(icx_ctx* ctx, icx_decode_job* job);
/* Batched decode: all files of the batch share the launches.  Per-job status
 * is filled in; the return value is ICX_OK unless a context-level failure
 * occurred. */
icx_status icx_decode_jpg_batch(icx_ctx* ctx, icx_decode_job* jobs, int32_t n);
icx_status icx_pool_decode_jpg_batch(icx_pool* pool, icx_decode_job* jobs, int32_t n);

/* ------------------------------------------------------------ device memory */
/* Buffers in the context GPU's HBM, so a decoded frame can stay on the device
 * between icx_decode_jpg_batch and icx_compress_jpg_batch (pass the pointer
 * as icx_decode_job.out and then as icx_image.px). */
icx_status icx_device_alloc(icx_ctx* ctx, size_t bytes, void** ptr);
icx_status icx_device_free(icx_ctx* ctx, void* ptr);
/* Pinned (page-locked, portable) host buffers: file bytes read straight into
 * one upload by DMA at link speed, with no staging copy. */
icx_status icx_host_alloc(icx_ctx* ctx, size_t bytes, void** ptr);
icx_status icx_host_free(icx_ctx* ctx, void* ptr);
/* Synchronous copy between any two of host / this context's device memory. */
icx_status icx_memcpy(icx_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Host -> this context's device memory, synchronous (the bytes are in HBM
 * when it returns), on a copy stream of its own and without waiting for a
 * batch call running on the context: reader threads push file bytes to the
 * GPU while the decode / encode kernels of other files run (the files ->
 * files path; the decode then reads device-resident files). */
icx_status icx_upload(icx_ctx* ctx, void* dst, const void* src, size_t bytes);

/* ------------------------------------------------------------- file staging */
/* The reader side of the files -> files path (CompressionBatch.java:64-88,
 * ImageCompression.java:53-76 / 113-126) without an interpreter lock: per
 * job, exists && readable (stat + access), the file size, and - for files
 * larger than min_size (-s) - one read into pinned memory, the JPEG header
 * parse of icx_jpeg_info and, for a JPEG the device decoder takes whose
 * dimensions pass the gate (w > min_width && h > min_height), one copy of the
 * whole file to this context's device (icx_device_alloc'd: the caller frees
 * `dev`, typically after icx_decode_jpg_batch read it).  Every decision
 * (skips, format fallbacks) stays with the caller.  jpeg_status: -1 = not
 * read or no JPEG SOI, else icx_jpeg_info's status.  read_errno: the read's
 * errno (-> FAILED_IO_ERROR).  Returns ICX_OK unless the device failed. */
typedef struct icx_stage_job {
    const char* path;                /* in */
    int64_t min_size;                /* in: -s */
    int32_t min_width, min_height;   /* in: -w, -i */
    int32_t exists;                  /* out */
    int64_t size;
    int32_t read_errno;
    int32_t jpeg_status;
    int32_t width, height, ncomp;
    void* dev;
    icx_status status;
} icx_stage_job;
icx_status icx_stage_files(icx_ctx* ctx, icx_stage_job* jobs, int32_t n);

/* ------------------------------------------------------- parity / metrics */
/* A 4-component (CMYK / YCCK) baseline file decoded to libjpeg's CMYK samples
 * (jdcolor.c: YCCK through ycck_cmyk_convert, CMYK as stored), 4 bytes a
 * pixel, W x H, host or device `out` - the samples icx_decode_jpg converts
 * to BGR24 (debug / parity). */
icx_status icx_debug_decode_cmyk(icx_ctx* ctx, const uint8_t* data, size_t len, uint8_t* out, size_t cap);
/* Quantised coefficients after DC prediction (natural order, 64 per block,
 * scan/MCU block order incl. dummy blocks) as the device decoder produced them. */
icx_status icx_debug_decode_coefs(icx_ctx* ctx, const uint8_t* data, size_t len, int16_t* coefs, size_t ncoefs);
/* Host-only: the progressive (SOF2) entropy decode the device decoder's
 * progressive path runs on host threads (every scan, jdphuff.c semantics),
 * same layout as icx_debug_decode_coefs (DC value in [0]).  ICX_E_INVALID for
 * a sequential file; no context and no GPU needed. */
icx_status icx_debug_progressive_coefs(const uint8_t* data, size_t len, int16_t* coefs, size_t ncoefs);
/* Host-only: the sequential entropy decode with IJG 6b's recovery (truncated
 * scans, bad codes, restart resynchronisation) that the device decoder runs
 * on host threads for the files its own decode flags; same layout as
 * icx_debug_decode_coefs.  ICX_E_INVALID for a progressive file. */
icx_status icx_debug_recovery_coefs(const uint8_t* data, size_t len, int16_t* coefs, size_t ncoefs);

/* Raw jpeg_fdct_islow coefficients (x8 scale, before quantisation) in scan
 * block order (MCU: Y0 Y1 Y2 Y3 Cb Cr), zig-zag within each block: the
 * device-resident layout the search re-quantises every trial. */
int64_t icx_num_blocks(int32_t width, int32_t height, int32_t fmt);
icx_status icx_debug_fdct(icx_ctx* ctx, const icx_image* img, int16_t* coefs, size_t ncoefs);

/* Per-kernel timing with HIP events recorded on the context's stream around
 * every launch of the named kernel ("fdct", "huff", "scan", "ffcount",
 * "decide", "stuff", "resize").  Enabling adds one event pair per launch. */
icx_status icx_profile_enable(icx_ctx* ctx, int32_t on);
icx_status icx_profile_reset(icx_ctx* ctx);
icx_status icx_profile_query(icx_ctx* ctx, const char* kernel, int64_t* launches, double* total_ms,
                             int64_t* units);

#ifdef __cplusplus
}
#endif
#endif /* ICX_H */
