// icx_png.cpp — the PNG write of the PNG path, native (host threads).
//
// Reference: ImageCompressionPng.java:70, ImageIO.write(resized, "png", file)
// -> the JDK PNGImageWriter (OpenJDK 21 java.desktop, not in /root/reference;
// restated here from its published source, unverifiable offline: SURVEY.md
// §8c).  What is restated:
//   - RowFilter.filterRow: the five filters of each row are costed over the
//     row's bytes in PNG sample order with the bytesPerPixel bytes left of the
//     row and the previous row of the first row reading as zero.  None costs
//     the sum of the unsigned bytes; Sub, Up, Average and Paeth the sum of
//     |curr - predictor| as ints (the unwrapped difference, not the residual
//     byte); the first strictly smaller cost wins (ties keep the lower type);
//   - PNGImageWriter's default deflate level, 4 (DEFAULT_COMPRESSION_LEVEL),
//     one zlib stream (java.util.zip.Deflater: zlib's default strategy,
//     window and memory level);
//   - IDATOutputStream: the stream is cut into IDAT chunks of 32768 bytes
//     (the last one shorter).
// The deflate bytes also depend on the JDK's zlib build, so PNG parity is on
// decoded pixels, dimensions, colour type and bit depth, with the filter
// choice pinned row for row against tests/png_ref.py.
//
// Output colour type follows the raster: GRAY8 -> 0 (grey, 8 bits), GRAY16
// -> 0 (grey, 16 bits, TYPE_USHORT_GRAY), BGR24 / RGB24 / XRGB32 -> 2 (RGB),
// ARGB32 / ABGR32 / RGBA32 -> 6 (RGBA), no interlace.  Palette rasters
// (INDEXED8: TYPE_BYTE_INDEXED, 8 bits; BINARY1: TYPE_BYTE_BINARY, 1/2/4 bits
// by map size) follow PNGMetadata.initialize for an IndexColorModel: a map
// that is the grey ramp i * 255 / (2^depth - 1) becomes grey (colour type 0,
// or 4 with alpha at 8 bits), anything else a palette (3) with PLTE = the
// whole map and tRNS = its alphas when it has any; RowFilter uses filter 0
// for every palette row.  The new images of ImageTools.resizeImage carry the
// default maps: INDEXED8 -> an 8-bit palette PNG of the 6x6x6 cube + grey
// ramp, BINARY1 -> a 1-bit grey PNG.  Rows are converted,
// filtered and deflated one at a time (three row buffers), straight into the
// caller's buffer: no image-sized temporary.  The caller's thread does the
// work; ctypes releases the GIL, so the batch driver's writer pool runs one
// image per thread.
#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "icx_context.h"

namespace {

// How a palette raster is written (PNGMetadata.initialize for an IndexColorModel).
struct PalOut {
    int depth = 8;     // bits per sample
    int ctype = 3;     // 0 grey, 4 grey + alpha, 3 palette
    bool alpha = false;
};

PalOut pal_out(const icx_image* img)
{
    PalOut o;
    const int n = img->palette_len;
    if (img->fmt == ICX_BINARY1) o.depth = n <= 2 ? 1 : n <= 4 ? 2 : 4;
    const int scale = 255 / ((1 << o.depth) - 1);
    bool grey = true;
    for (int i = 0; i < n; i++) {
        const uint32_t c = img->palette[i];
        const uint32_t r = c >> 16 & 255, g = c >> 8 & 255, b = c & 255;
        if (r != (uint32_t)(i * scale & 255) || r != g || r != b) grey = false;
        if ((c >> 24) != 255) o.alpha = true;
    }
    o.ctype = grey && o.alpha && o.depth == 8 ? 4 : grey && !o.alpha ? 0 : 3;
    return o;
}

// Bytes per pixel of the PNG row (RowFilter's bytesPerPixel) and of the source.
int png_bpp(int fmt)
{
    switch (fmt) {
    case ICX_GRAY8: case ICX_INDEXED8: case ICX_BINARY1: return 1;
    case ICX_GRAY16: return 2;
    case ICX_BGR24: case ICX_RGB24: case ICX_XRGB32: return 3;
    default: return 4;
    }
}

int src_bpp(int fmt)
{
    return fmt == ICX_GRAY8 || fmt == ICX_INDEXED8 || fmt == ICX_BINARY1 ? 1 : fmt == ICX_GRAY16 ? 2
                                                                        : fmt <= ICX_RGB24 ? 3 : 4;
}

// Bytes of one PNG row (without the filter byte).
size_t png_row_bytes(const icx_image* img)
{
    if (img->fmt == ICX_INDEXED8 || img->fmt == ICX_BINARY1) {
        const PalOut o = pal_out(img);
        return o.ctype == 4 ? 2 * (size_t)img->width : ((size_t)img->width * o.depth + 7) / 8;
    }
    return (size_t)img->width * png_bpp(img->fmt);
}

// A palette row -> PNG samples: indices packed MSB first at `depth` bits,
// grey levels (the ramp's index is the level) or grey + alpha pairs.
void convert_pal_row(const uint8_t* s, const icx_image* img, const PalOut& o, uint8_t* d)
{
    const int w = img->width;
    if (o.ctype == 4) {
        for (int x = 0; x < w; x++) {
            const uint32_t c = img->palette[s[x] < img->palette_len ? s[x] : 0];
            d[2 * x] = (uint8_t)(c & 255);
            d[2 * x + 1] = (uint8_t)(c >> 24);
        }
        return;
    }
    if (o.depth == 8) {
        memcpy(d, s, (size_t)w);
        return;
    }
    memset(d, 0, ((size_t)w * o.depth + 7) / 8);
    const int per = 8 / o.depth;
    for (int x = 0; x < w; x++)
        d[x / per] |= (uint8_t)((s[x] & ((1 << o.depth) - 1)) << (8 - o.depth * (x % per + 1)));
}

// Source row -> PNG sample order (R, G, B[, A] or grey).
void convert_row(const uint8_t* s, int w, int fmt, uint8_t* d)
{
    switch (fmt) {
    case ICX_GRAY8: memcpy(d, s, (size_t)w); break;
    case ICX_GRAY16:  // native-endian (little) uint16 -> big-endian PNG samples
        for (int x = 0; x < w; x++) { d[2 * x] = s[2 * x + 1]; d[2 * x + 1] = s[2 * x]; }
        break;
    case ICX_RGB24: memcpy(d, s, (size_t)w * 3); break;
    case ICX_RGBA32: memcpy(d, s, (size_t)w * 4); break;
    case ICX_BGR24:
        for (int x = 0; x < w; x++) { d[3 * x] = s[3 * x + 2]; d[3 * x + 1] = s[3 * x + 1]; d[3 * x + 2] = s[3 * x]; }
        break;
    case ICX_XRGB32:  // bytes B, G, R, X
        for (int x = 0; x < w; x++) { d[3 * x] = s[4 * x + 2]; d[3 * x + 1] = s[4 * x + 1]; d[3 * x + 2] = s[4 * x]; }
        break;
    case ICX_ARGB32:  // bytes B, G, R, A
        for (int x = 0; x < w; x++) {
            d[4 * x] = s[4 * x + 2]; d[4 * x + 1] = s[4 * x + 1]; d[4 * x + 2] = s[4 * x]; d[4 * x + 3] = s[4 * x + 3];
        }
        break;
    case ICX_ABGR32:  // bytes A, B, G, R
        for (int x = 0; x < w; x++) {
            d[4 * x] = s[4 * x + 3]; d[4 * x + 1] = s[4 * x + 2]; d[4 * x + 2] = s[4 * x + 1]; d[4 * x + 3] = s[4 * x];
        }
        break;
    }
}

inline int paeth(int a, int b, int c)
{
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// RowFilter.filterRow: filters `cur` (prev: the previous row in PNG sample
// order, zeros for the first) into out[0] = type, out[1..n] = residuals.
void filter_row(const uint8_t* cur, const uint8_t* prev, int n, int bpp, uint8_t* out)
{
    // the badness of all five filters in one pass
    long cost[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const int x = cur[i], a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
        cost[0] += x;                           // None: the unsigned bytes themselves
        cost[1] += std::abs(x - a);             // the others: |curr - predictor| as ints
        cost[2] += std::abs(x - b);
        cost[3] += std::abs(x - ((a + b) >> 1));
        cost[4] += std::abs(x - paeth(a, b, c));
    }
    int best = 0;
    for (int f = 1; f < 5; f++)
        if (cost[f] < cost[best]) best = f;
    out[0] = (uint8_t)best;
    uint8_t* r = out + 1;
    for (int i = 0; i < n; i++) {
        const int x = cur[i], a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
        int p = 0;
        switch (best) {
        case 1: p = a; break;
        case 2: p = b; break;
        case 3: p = (a + b) >> 1; break;
        case 4: p = paeth(a, b, c); break;
        }
        r[i] = (uint8_t)(x - p);
    }
}

void put32(uint8_t* p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

// One chunk at p: length, tag, the `len` data bytes already at p + 8, CRC.
size_t close_chunk(uint8_t* p, const char* tag, size_t len)
{
    put32(p, (uint32_t)len);
    memcpy(p + 4, tag, 4);
    const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), p + 4, (uInt)(len + 4));
    put32(p + 8 + len, crc);
    return 12 + len;
}

}  // namespace

extern "C" {

// The whole filtered image (raw bytes) up to 1 GiB: zlib's 32-bit counters.
constexpr size_t kMaxRaw = (size_t)1 << 30;
constexpr size_t kIdat = 32768;  // IDATOutputStream chunk length
constexpr int kDefaultLevel = 4; // PNGImageWriter.DEFAULT_COMPRESSION_LEVEL

// A palette raster's colour map as validate() (icx_runtime.cpp) takes it:
// 1..256 entries for INDEXED8, 1..16 for BINARY1 (IndexColorModel of a
// TYPE_BYTE_BINARY raster: at most 4 bits per pixel).
static bool palette_ok(const icx_image* img)
{
    if (img->fmt != ICX_INDEXED8 && img->fmt != ICX_BINARY1) return true;
    const int maxn = img->fmt == ICX_BINARY1 ? 16 : 256;
    return img->palette && img->palette_len >= 1 && img->palette_len <= maxn;
}

size_t icx_png_bound(const icx_image* img)
{
    if (!img || img->width <= 0 || img->height <= 0) return 0;
    if (!palette_ok(img)) return 0;
    const size_t raw = (size_t)img->height * (png_row_bytes(img) + 1);
    if (raw > kMaxRaw) return 0;
    const size_t z = (size_t)compressBound((uLong)raw);
    return 8 + 25 + z + 12 * (z / kIdat + 1) + 12 + 64 + 12 + 3 * 256 + 12 + 256;  // + PLTE, tRNS
}

icx_status icx_png_encode(const icx_image* img, int32_t level, uint8_t* out, size_t cap, size_t* out_len)
{
    if (!img || !img->px || !out || !out_len) return ICX_E_NULL;
    if (img->width <= 0 || img->height <= 0 || img->fmt < ICX_BGR24 || img->fmt > ICX_BINARY1 ||
        img->stride < img->width * src_bpp(img->fmt) || level < -1 || level > 9)
        return ICX_E_INVALID;
    if (icx::is_device_ptr(img->px)) return ICX_E_INVALID;  // host rows only
    if (!palette_ok(img)) return ICX_E_INVALID;             // no map, or more entries than the depth holds
    const size_t need = icx_png_bound(img);
    if (need == 0) return ICX_E_UNSUPPORTED;  // over kMaxRaw
    *out_len = need;
    if (cap < need) return ICX_E_BUFFER;
    const bool pal = img->fmt == ICX_INDEXED8 || img->fmt == ICX_BINARY1;
    const PalOut po = pal ? pal_out(img) : PalOut{};
    const int bpp = pal && po.ctype == 4 ? 2 : png_bpp(img->fmt);
    const int n = (int)png_row_bytes(img);
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    memcpy(out, sig, 8);
    size_t pos = 8;
    uint8_t* ih = out + pos + 8;
    put32(ih, (uint32_t)img->width);
    put32(ih + 4, (uint32_t)img->height);
    ih[8] = pal ? (uint8_t)po.depth : img->fmt == ICX_GRAY16 ? 16 : 8;                // bit depth
    ih[9] = pal ? (uint8_t)po.ctype : (uint8_t)(bpp <= 2 ? 0 : bpp == 3 ? 2 : 6);    // colour type
    ih[10] = ih[11] = ih[12] = 0;                             // deflate, adaptive filtering, no interlace
    pos += close_chunk(out + pos, "IHDR", 13);
    if (pal && po.ctype == 3) {  // PLTE = the whole map, tRNS = its alphas
        uint8_t* p = out + pos + 8;
        for (int i = 0; i < img->palette_len; i++) {
            p[3 * i] = (uint8_t)(img->palette[i] >> 16);
            p[3 * i + 1] = (uint8_t)(img->palette[i] >> 8);
            p[3 * i + 2] = (uint8_t)img->palette[i];
        }
        pos += close_chunk(out + pos, "PLTE", 3 * (size_t)img->palette_len);
        if (po.alpha) {
            p = out + pos + 8;
            for (int i = 0; i < img->palette_len; i++) p[i] = (uint8_t)(img->palette[i] >> 24);
            pos += close_chunk(out + pos, "tRNS", (size_t)img->palette_len);
        }
    }

    z_stream z{};
    if (deflateInit(&z, level < 0 ? kDefaultLevel : level) != Z_OK) return ICX_E_NOMEM;
    std::vector<uint8_t> rows(3 * (size_t)n + 1);
    uint8_t *cur = rows.data(), *prev = cur + n, *filt = prev + n;
    memset(prev, 0, (size_t)n);
    // deflate straight into IDAT chunks of kIdat data bytes: a full chunk is
    // closed (length, tag, CRC) and the next one opened behind it
    uint8_t* idat = out + pos;
    // this chunk's data capacity: kIdat, or less when the caller's buffer ends
    // first (then a full chunk means the buffer is exhausted)
    auto room = [&](size_t at) -> size_t { return cap > at + 32 ? std::min(kIdat, cap - at - 32) : 0; };
    size_t ccap = room(pos);
    z.next_out = idat + 8;
    z.avail_out = (uInt)ccap;
    int zr = Z_OK;
    bool finished = false;
    for (int y = 0; y < img->height && zr == Z_OK; y++) {
        if (pal) convert_pal_row(img->px + (size_t)y * img->stride, img, po, cur);
        else convert_row(img->px + (size_t)y * img->stride, img->width, img->fmt, cur);
        if (pal && po.ctype == 3) {  // RowFilter: "Use type 0 for palette images"
            filt[0] = 0;
            memcpy(filt + 1, cur, (size_t)n);
        } else {
            filter_row(cur, prev, n, bpp, filt);
        }
        z.next_in = filt;
        z.avail_in = (uInt)n + 1;
        const int flush = y + 1 == img->height ? Z_FINISH : Z_NO_FLUSH;
        for (;;) {
            zr = deflate(&z, flush);
            if (zr == Z_STREAM_END) {
                finished = true;
                zr = Z_OK;
                break;
            }
            if (zr != Z_OK && zr != Z_BUF_ERROR) break;
            zr = Z_OK;
            if (z.avail_out > 0) break;  // input consumed (NO_FLUSH) - next row
            // chunk full: close it, open the next one
            if (ccap < kIdat) { zr = Z_BUF_ERROR; break; }
            pos += close_chunk(idat, "IDAT", kIdat);
            idat = out + pos;
            ccap = room(pos);
            if (ccap == 0) { zr = Z_BUF_ERROR; break; }
            z.next_out = idat + 8;
            z.avail_out = (uInt)ccap;
        }
        std::swap(cur, prev);
    }
    const size_t last = ccap - z.avail_out;
    const bool ok = finished && z.avail_in == 0 && zr == Z_OK;
    deflateEnd(&z);
    if (!ok) return ICX_E_BUFFER;
    if (last > 0) pos += close_chunk(idat, "IDAT", last);
    pos += close_chunk(out + pos, "IEND", 0);
    *out_len = pos;
    return ICX_OK;
}

}  // extern "C"
