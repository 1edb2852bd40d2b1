// icx_png.cpp — the PNG write of the PNG path, native (host threads).
//
// Reference: ImageCompressionPng.java:70, ImageIO.write(resized, "png", file)
// -> the JDK PNGImageWriter: per row an adaptive filter (None, Sub, Up,
// Average, Paeth) and one zlib stream.  The writer's exact heuristic and
// deflate settings are not pinnable here (no JDK): parity is
// on decoded pixels and dimensions, and the filter choice is the one of the
// previous Python writer (tests/png_ref.py): the least sum of |residual byte
// read as signed|, ties to the lower filter type.
//
// Output colour type follows the raster: GRAY8 -> 0 (grey), BGR24 / RGB24 /
// XRGB32 -> 2 (RGB), ARGB32 / ABGR32 / RGBA32 -> 6 (RGBA), 8 bits per sample,
// no interlace.  Rows are converted, filtered and deflated one at a time
// (three row buffers), straight into the caller's buffer: no image-sized
// temporary.  The caller's thread does the work; ctypes releases the GIL, so
// the batch driver's writer pool runs one image per thread.
#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "icx_context.h"

namespace {

int png_channels(int fmt)
{
    switch (fmt) {
    case ICX_GRAY8: return 1;
    case ICX_BGR24: case ICX_RGB24: case ICX_XRGB32: return 3;
    default: return 4;
    }
}

int src_channels(int fmt) { return fmt == ICX_GRAY8 ? 1 : fmt <= ICX_RGB24 ? 3 : 4; }

// Source row -> PNG sample order (R, G, B[, A] or grey).
void convert_row(const uint8_t* s, int w, int fmt, uint8_t* d)
{
    switch (fmt) {
    case ICX_GRAY8: memcpy(d, s, (size_t)w); break;
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

// Filters `cur` (prev: the previous raw row, zeros for the first) into
// out[0] = type, out[1..n] = residuals.
void filter_row(const uint8_t* cur, const uint8_t* prev, int n, int bpp, uint8_t* out)
{
    // costs of all five filters in one pass
    long cost[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const int x = cur[i], a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
        cost[0] += std::abs((int)(int8_t)(uint8_t)x);
        cost[1] += std::abs((int)(int8_t)(uint8_t)(x - a));
        cost[2] += std::abs((int)(int8_t)(uint8_t)(x - b));
        cost[3] += std::abs((int)(int8_t)(uint8_t)(x - ((a + b) >> 1)));
        cost[4] += std::abs((int)(int8_t)(uint8_t)(x - paeth(a, b, c)));
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

// One IDAT chunk holds the whole zlib stream: raw (filtered) data up to 1 GiB.
constexpr size_t kMaxRaw = (size_t)1 << 30;

size_t icx_png_bound(const icx_image* img)
{
    if (!img || img->width <= 0 || img->height <= 0) return 0;
    const size_t raw = (size_t)img->height * ((size_t)img->width * png_channels(img->fmt) + 1);
    if (raw > kMaxRaw) return 0;
    return 8 + 25 + 12 + (size_t)compressBound((uLong)raw) + 12 + 64;
}

icx_status icx_png_encode(const icx_image* img, int32_t level, uint8_t* out, size_t cap, size_t* out_len)
{
    if (!img || !img->px || !out || !out_len) return ICX_E_NULL;
    if (img->width <= 0 || img->height <= 0 || img->fmt < ICX_BGR24 || img->fmt > ICX_RGBA32 ||
        img->stride < img->width * src_channels(img->fmt) || level < -1 || level > 9)
        return ICX_E_INVALID;
    if (icx::is_device_ptr(img->px)) return ICX_E_INVALID;  // host rows only
    const size_t need = icx_png_bound(img);
    if (need == 0) return ICX_E_UNSUPPORTED;  // over kMaxRaw
    *out_len = need;
    if (cap < need) return ICX_E_BUFFER;
    const int ch = png_channels(img->fmt);
    const int n = img->width * ch;
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    memcpy(out, sig, 8);
    size_t pos = 8;
    uint8_t* ih = out + pos + 8;
    put32(ih, (uint32_t)img->width);
    put32(ih + 4, (uint32_t)img->height);
    ih[8] = 8;                                         // bit depth
    ih[9] = (uint8_t)(ch == 1 ? 0 : ch == 3 ? 2 : 6);  // colour type
    ih[10] = ih[11] = ih[12] = 0;                      // deflate, adaptive filtering, no interlace
    pos += close_chunk(out + pos, "IHDR", 13);

    z_stream z{};
    if (deflateInit(&z, level) != Z_OK) return ICX_E_NOMEM;
    std::vector<uint8_t> rows(3 * (size_t)n + 1);
    uint8_t *cur = rows.data(), *prev = cur + n, *filt = prev + n;
    memset(prev, 0, (size_t)n);
    uint8_t* idat = out + pos;
    z.next_out = idat + 8;
    z.avail_out = (uInt)std::min<size_t>(cap - pos - 8 - 12 - 12, 0xFFFFFFFFu);
    int zr = Z_OK;
    bool finished = false;
    for (int y = 0; y < img->height && zr == Z_OK; y++) {
        convert_row(img->px + (size_t)y * img->stride, img->width, img->fmt, cur);
        filter_row(cur, prev, n, ch, filt);
        z.next_in = filt;
        z.avail_in = (uInt)n + 1;
        zr = deflate(&z, y + 1 == img->height ? Z_FINISH : Z_NO_FLUSH);
        if (zr == Z_STREAM_END) {
            finished = true;
            zr = Z_OK;
        }
        std::swap(cur, prev);
    }
    const size_t zlen = z.total_out;
    const bool ok = finished && z.avail_in == 0;
    deflateEnd(&z);
    if (!ok) return ICX_E_BUFFER;
    pos += close_chunk(idat, "IDAT", zlen);
    pos += close_chunk(out + pos, "IEND", 0);
    *out_len = pos;
    return ICX_OK;
}

}  // extern "C"
