// icx_runtime.cpp — host runtime behind include/icx.h.
//
// Owns one HIP stream, a device workspace arena and a pinned staging arena
// per context, builds the binary-search trees (all float32 decisions of
// ImageCompressionJpg.java:158-200 are evaluated here, in Java's order of
// operations), and drives the batched stage loop of compressJpgWithTargetSize
// (ImageCompressionJpg.java:77-122) on the device: per stage one FDCT launch,
// then the quality trials as a fixed sequence of launches with the search
// state kept in HBM (no host round trip between trials), then one host
// synchronisation to decide which images move on to the next 0.85x scale.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/icx.h"
#include "icx_context.h"
#include "icx_internal.h"
#include "icx_kernels.h"

using namespace icx;

namespace {

// ------------------------------------------------------------ constants
// JPEGQTable.K1Luminance / K2Chrominance (ITU-T T.81 Annex K.1/K.2), natural order.
const int kK1[64] = {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                     14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                     18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int kK2[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                     24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// zig-zag position -> natural index (jpeg_natural_order)
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// Annex K.3 standard Huffman tables (JPEGHuffmanTable.Std*): counts per length 1..16, symbols.
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChrVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

// ------------------------------------------------------- float32 quality math
// Java float arithmetic; volatile locals keep every product/sum rounded to
// float32 (no contraction, no extended precision).
float linear_quality(float q)  // JPEG.convertToLinearQuality
{
    if (q <= 0.0f) q = 0.01f;
    if (q > 1.0f) q = 1.0f;
    if (q < 0.5f) {
        volatile float r = 0.5f / q;
        return r;
    }
    volatile float t = q * 2.0f;
    volatile float r = 2.0f - t;
    return r;
}

void scaled_table(const int* base, float lin, uint16_t* out)  // JPEGQTable.getScaledInstance(lin, true)
{
    for (int i = 0; i < 64; i++) {
        volatile float p = (float)base[i] * lin;
        volatile float s = p + 0.5f;
        int sv = (int)s;
        out[i] = (uint16_t)std::min(255, std::max(1, sv));
    }
}

void make_node(float q, QNode& n)
{
    uint16_t t[2][64];
    const float lin = linear_quality(q);
    scaled_table(kK1, lin, t[0]);
    scaled_table(kK2, lin, t[1]);
    n.mid = q;
    n.child_fit = n.child_nofit = -1;
    n.pad = 0;
    for (int c = 0; c < 2; c++) {
        for (int k = 0; k < 64; k++) {
            const uint32_t div = (uint32_t)t[c][kZigzag[k]] << 3;
            volatile float r = 1.0f / (float)div;
            volatile float b = ((float)(div >> 1) + 0.5f) * r;
            n.qf[c][k] = make_float4((float)(div - (div >> 1)), r, b, 0.0f);
        }
        for (int i = 0; i < 64; i++) n.qt[c][i] = t[c][i];
    }
}

// Tree of findBestQualityByBinarySearch: a node is the loop state (lo, hi, i)
// at the top of an iteration that performs an encode.
int build_tree(float lo, float hi, int iter, std::vector<QNode>& nodes, int& depth)
{
    if (iter >= MAX_TRIALS) return -1;
    volatile float sum = lo + hi;
    volatile float mid = sum / 2.0f;  // (lowQuality + highQuality) / 2.0f
    if (mid < 0.01f) return -1;       // midQuality < 0.01f -> break
    const int idx = (int)nodes.size();
    nodes.emplace_back();
    make_node(mid, nodes[idx]);
    depth = std::max(depth, iter + 1);
    volatile float dfit = hi - mid;   // fits: lowQuality = mid
    volatile float dno = mid - lo;    // too big: highQuality = mid
    const int cf = dfit < 0.01f ? -1 : build_tree(mid, hi, iter + 1, nodes, depth);
    const int cn = dno < 0.01f ? -1 : build_tree(lo, mid, iter + 1, nodes, depth);
    nodes[idx].child_fit = cf;
    nodes[idx].child_nofit = cn;
    return idx;
}

// bytes per pixel of a raster (GRAY16: one 2-byte sample)
int channels(int fmt)
{
    return fmt == ICX_GRAY8 || fmt == ICX_INDEXED8 || fmt == ICX_BINARY1 ? 1 : fmt == ICX_GRAY16 ? 2
                                                                        : fmt <= ICX_RGB24 ? 3 : 4;
}

bool is_palette(int fmt) { return fmt == ICX_INDEXED8 || fmt == ICX_BINARY1; }

// --- default colour maps of the palette types (BufferedImage.java's
// TYPE_BYTE_INDEXED / TYPE_BYTE_BINARY constructors) and what Java2D derives
// from a map for storing into it (OpenJDK java.desktop; no JDK here to pin
// them, parity unpinned: DESIGN.md §6)
int default_palette(bool binary, uint32_t* pal)
{
    if (binary) {  // IndexColorModel(1, 2, {0, 0xff} x 3)
        pal[0] = 0xff000000u;
        pal[1] = 0xffffffffu;
        return 2;
    }
    int n = 0;  // 6x6x6 cube (r outer), then a grey ramp from 18 in steps of 256 / 40
    for (int r = 0; r <= 255; r += 51)
        for (int g = 0; g <= 255; g += 51)
            for (int b = 0; b <= 255; b += 51) pal[n++] = 0xff000000u | (uint32_t)r << 16 | (uint32_t)g << 8 | (uint32_t)b;
    const int step = 256 / (256 - n);
    for (int v = 3 * step; n < 256; n++, v += step) pal[n] = 0xff000000u | (uint32_t)v * 0x010101u;
    return 256;
}

// initCubemap (32 cells per axis): the map's entries seed a 15-bit RGB cube
// in the order 0, n-1, 1, n-2, ...; then breadth first, level by level, every
// cell of the previous level claims its unclaimed neighbours (+r, -r, +g, -g,
// +b, -b) for its entry - an L1 flood fill in which the first claim wins.
std::vector<uint8_t> inverse_cube(const uint32_t* pal, int n)
{
    std::vector<uint8_t> cube(32768, 0);
    std::vector<uint8_t> claimed(32768, 0);
    std::vector<std::pair<uint16_t, uint8_t>> level, next;
    auto claim = [&](std::vector<std::pair<uint16_t, uint8_t>>& to, int cell, int idx) {
        if (claimed[cell]) return;
        claimed[cell] = 1;
        cube[cell] = (uint8_t)idx;
        to.emplace_back((uint16_t)cell, (uint8_t)idx);
    };
    auto cell_of = [](uint32_t c) { return (int)((c >> 9 & 0x7c00) | (c >> 6 & 0x03e0) | (c >> 3 & 0x001f)); };
    for (int i = 0; i < (n + 1) / 2; i++) {
        claim(level, cell_of(pal[i]), i);
        claim(level, cell_of(pal[n - 1 - i]), n - 1 - i);
    }
    static const int kMask[3] = {0x7c00, 0x03e0, 0x001f}, kStep[3] = {0x0400, 0x0020, 0x0001};
    while (!level.empty()) {
        next.clear();
        for (const auto& e : level)
            for (int a = 0; a < 3; a++) {
                if ((e.first & kMask[a]) + kStep[a] <= kMask[a]) claim(next, e.first + kStep[a], e.second);
                if ((e.first & kMask[a]) >= kStep[a]) claim(next, e.first - kStep[a], e.second);
            }
        level.swap(next);
    }
    return cube;
}

// calculatePrimaryColorsApproximation: the eight corner cells hold colours
// within 5 of their corners' primaries
bool represents_primaries(const uint32_t* pal, const std::vector<uint8_t>& cube)
{
    for (int c = 0; c < 8; c++) {
        const int r = c & 4 ? 31 : 0, g = c & 2 ? 31 : 0, b = c & 1 ? 31 : 0;
        const uint32_t p = pal[cube[(r << 10) | (g << 5) | b]];
        const int want[3] = {r ? 255 : 0, g ? 255 : 0, b ? 255 : 0};
        const int got[3] = {(int)(p >> 16 & 255), (int)(p >> 8 & 255), (int)(p & 255)};
        for (int k = 0; k < 3; k++)
            if (std::abs(got[k] - want[k]) > 5) return false;
    }
    return true;
}

// make_dither_arrays(256): the 8x8 recursive ordered-dither matrix scaled to
// [-e/2, e - e/2) with e = (int)(256 / cbrt(256)) = 40; green mirrored
// left-right, blue top-bottom
void dither_tables(int8_t (&d)[3][64])
{
    const int e = (int)(256 / std::pow(256.0, 1.0 / 3.0)), lo = -e / 2, hi = e - e / 2;
    int m[8][8];
    m[0][0] = 0;
    for (int k = 1; k < 8; k <<= 1)
        for (int i = 0; i < k; i++)
            for (int j = 0; j < k; j++) {
                const int v = m[i][j] * 4;
                m[i][j] = v;
                m[i + k][j + k] = v + 1;
                m[i][j + k] = v + 2;
                m[i + k][j] = v + 3;
            }
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            const auto at = [&](int yy, int xx) { return (int8_t)(m[yy][xx] * (hi - lo) / 64 + lo); };
            d[0][y * 8 + x] = at(y, x);
            d[1][y * 8 + x] = at(y, 7 - x);
            d[2][y * 8 + x] = at(7 - y, x);
        }
}

void geometry(ImgDesc& d, int w, int h, int fmt, int layout = ICX_TABLES_SEPARATE)
{
    d.w = w;
    d.h = h;
    d.fmt = fmt;
    d.ncomp = fmt == ICX_GRAY8 ? 1 : 3;
    d.ywb = (w + 7) / 8;
    d.yhb = (h + 7) / 8;
    if (d.ncomp == 1) {
        d.mcux = d.ywb;
        d.mcuy = d.yhb;
        d.nblocks = (int64_t)d.mcux * d.mcuy;
        d.hdr_len = layout == ICX_TABLES_GROUPED ? HDR_GRAY_GROUPED : HDR_GRAY;
    } else {
        d.mcux = (w + 15) / 16;
        d.mcuy = (h + 15) / 16;
        d.nblocks = (int64_t)d.mcux * d.mcuy * 6;
        d.hdr_len = layout == ICX_TABLES_GROUPED ? HDR_COLOR_GROUPED : HDR_COLOR;
    }
    d.nchunks = (int)((d.nblocks + CHUNK_BLOCKS - 1) / CHUNK_BLOCKS);
    d.tiles_x = (uint32_t)((d.mcux + 15) / 16);
    d.tiles_xm = d.tiles_x > 1 ? (uint32_t)(((1ull << 32) + d.tiles_x - 1) / d.tiles_x) : 0u;
}

int64_t fdct_tiles(const ImgDesc& d)
{
    return d.ncomp == 1 ? (int64_t)((d.mcux + 15) / 16) * d.mcuy : (int64_t)((d.mcux + 15) / 16) * d.mcuy;
}

// candidate-list region: COEF_SLOTS int32 entries for every block of every
// FDCT tile (16 colour MCUs = 96 blocks, or 16 grey blocks), partial tiles included
size_t coef_bytes(const ImgDesc& d)
{
    return (size_t)fdct_tiles(d) * (d.ncomp == 1 ? 16 : 96) * COEF_SLOTS * 4;
}

// worst-case entropy bytes after stuffing
uint64_t worst_file(const ImgDesc& d) { return (uint64_t)d.hdr_len + (uint64_t)d.nblocks * (MAX_BLOCK_BITS / 8) * 2 + 16; }

}  // namespace

namespace {

// ---------------------------------------------------------------- batch driver
struct Item {
    icx_fit_job* job;
    int kind;              // 0 BGR, 1 RGB, 2 GRAY
    int nch;
    ImgDesc orig;          // geometry of the original image
    const uint8_t* dpx;    // original pixels on device
    uint8_t* dresize;
    uint8_t* dout;
    bool host_out;
    int root;              // search tree root for this job's quality bound
    int depth;
    int cached_node;
    double coef_scale;     // scale whose coefficients are resident, NaN = none
    int64_t entries;       // candidate-list entries of the resident coefficients (padded)
    bool done, found, hit;
    float best_q;
    double best_scale;
    int encodes;
};

enum class Mode { Fit, Encode, Search, Fdct };

struct Batch {
    icx_ctx* c;
    std::vector<Item> it;
    std::vector<QNode> nodes;
    ImgDesc* d_desc = nullptr;
    ImgState* d_state = nullptr;
    QNode* d_nodes = nullptr;
    std::vector<ImgDesc> desc;
    std::vector<ImgState> state;
    ImgState* h_state = nullptr;  // pinned mirror for downloads
    int huff_launches = 0;        // trial launches so far: odd ones walk the images in reverse (launch_huff)
    // The stage's small uploads (descriptors, states, launch plans) share one
    // pinned block and go in one copy per launch group (flush before launches).
    std::unique_ptr<Uploader> up;
};

struct DPlan {
    Plan p;
    int64_t total;
};


// Build a launch plan over `ids` with per-image work counts.
icx_status make_plan(Batch& B, const std::vector<int>& ids, const std::vector<int64_t>& counts, DPlan& out)
{
    std::vector<int64_t> pre(ids.size() + 1, 0);
    for (size_t i = 0; i < ids.size(); i++) pre[i + 1] = pre[i] + counts[i];
    std::vector<int32_t> ids32(ids.begin(), ids.end());
    ids32.push_back(0);
    out.p.ids = B.up->put(ids32.data(), ids32.size());
    out.p.prefix = B.up->put(pre.data(), pre.size());
    out.p.m = (int32_t)ids.size();
    out.p.uniform = 0;
    out.p.identity = 1;
    for (size_t i = 0; i < ids.size(); i++) out.p.identity &= ids[i] == (int)i;
    if (!counts.empty() && counts[0] > 0 && counts[0] < (1 << 30) && ids.size() < 65536 &&
        std::all_of(counts.begin(), counts.end(), [&](int64_t v) { return v == counts[0]; }))
        out.p.uniform = (int32_t)counts[0];
    out.total = pre.back();
    return B.up->overflow ? fail(B.c, ICX_E_NOMEM, "upload staging exhausted") : ICX_OK;
}

// A new stage: descriptors and states go into a fresh upload block (with room
// for the stage's launch plans); the copy happens at the first launch.
void new_stage(Batch& B)
{
    const size_t m = B.desc.size();
    const size_t bytes = Uploader::need<ImgDesc>(m) + Uploader::need<ImgState>(m) +
                         12 * (Uploader::need<int32_t>(m + 1) + Uploader::need<int64_t>(m + 1));
    B.up.reset(new Uploader(B.c, bytes));
}

// Wait for the stream: the stage decisions sit on the critical path between
// two device stages, and a blocking wait's wake-up latency (scheduler-
// dependent, 20 us to several hundred on a busy host) is idle device time.
// So poll - tightly for the first 50 us, then yielding the core to the
// decode / writer pools between polls - and block only once the stage has
// run for 2 ms, where a wake-up is small against the stage itself.
hipError_t stream_wait(hipStream_t st)
{
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        const auto dt = clk::now() - t0;
        if (dt < std::chrono::microseconds(50)) {
#if defined(__x86_64__) || defined(__i386__)
            __builtin_ia32_pause();
#endif
        } else if (dt < std::chrono::milliseconds(2)) {
            sched_yield();
        } else {
            return hipStreamSynchronize(st);
        }
    }
}

icx_status sync_states(Batch& B)
{
    HostSpan hs{B.c, "host.sync"};
    icx_ctx* c = B.c;
    hipError_t e = hipMemcpyAsync(B.h_state, B.d_state, sizeof(ImgState) * B.state.size(), hipMemcpyDeviceToHost,
                                  c->stream);
    if (e == hipSuccess) e = stream_wait(c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "state download");
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(c, e, "kernel launch");
    memcpy(B.state.data(), B.h_state, sizeof(ImgState) * B.state.size());
    return ICX_OK;  // profile events are resolved once, when the call ends
}

icx_status push_desc_state(Batch& B)
{
    new_stage(B);
    B.d_desc = B.up->put(B.desc.data(), B.desc.size());
    B.d_state = B.up->put(B.state.data(), B.state.size());
    if (B.c->dev.overflow) return fail(B.c, ICX_E_NOMEM, "device workspace overrun (workspace sizing)");
    return B.up->overflow ? fail(B.c, ICX_E_NOMEM, "upload staging exhausted") : ICX_OK;
}

// Point image i's descriptor at its pixels for `scale` (resizing on device).
void stage_pixels(Batch& B, int i, double scale)
{
    icx_ctx* c = B.c;
    Item& I = B.it[i];
    ImgDesc& d = B.desc[i];
    const ImgDesc keep = d;
    if (scale < 1.0) {
        int32_t dw, dh;
        icx_scaled_dims(I.orig.w, I.orig.h, scale, &dw, &dh);
        {
            Timed tm(c, "resize", (int64_t)dw * dh);
            launch_resize(I.dpx, I.orig.w, I.orig.h, I.orig.stride, I.orig.fmt, I.dresize, dw, dh, dw * I.nch,
                          c->stream);
        }
        geometry(d, dw, dh, I.orig.fmt, c->table_layout);
        d.px = I.dresize;
        d.stride = dw * I.nch;
    } else {
        geometry(d, I.orig.w, I.orig.h, I.orig.fmt, c->table_layout);
        d.px = I.dpx;
        d.stride = I.orig.stride;
    }
    // buffers and limits stay those sized for the original image
    d.coefs = keep.coefs;
    d.coff = keep.coff;
    d.ncoef = keep.ncoef;
    d.cand_node = keep.cand_node;
    for (int k = 0; k < 2; k++) {
        d.scratch[k] = keep.scratch[k];
        d.chunk_bits[k] = keep.chunk_bits[k];
        d.chunk_off[k] = keep.chunk_off[k];
        d.chunk_ff[k] = keep.chunk_ff[k];
        d.chunk_ffa[k] = keep.chunk_ffa[k];
    }
    d.chunk_ffoff = keep.chunk_ffoff;
    d.ovf = keep.ovf;
    d.out = keep.out;
    d.cap = keep.cap;
    d.target = keep.target;
}

icx_status run_fdct(Batch& B, const std::vector<int>& ids)
{
    for (int kind = 0; kind < 3; kind++) {
        std::vector<int> sel;
        std::vector<int64_t> cnt;
        for (int i : ids)
            if (B.it[i].kind == kind) {
                sel.push_back(i);
                cnt.push_back(fdct_tiles(B.desc[i]));
            }
        if (sel.empty()) continue;
        DPlan P;
        icx_status s = make_plan(B, sel, cnt, P);
        if (s) return s;
        int64_t px = 0;
        for (int i : sel) px += (int64_t)B.desc[i].w * B.desc[i].h;
        if ((s = B.up->flush())) return s;
        {
            Timed tm(B.c, "fdct", px, true);
            launch_fdct(B.d_desc, B.d_state, B.d_nodes, P.p, P.total, kind, B.c->stream);
        }
        if (B.c->prof) {  // list sizes for the byte accounting (the FDCT keeps no count)
            Timed tm(B.c, "count", (int64_t)sel.size(), true);
            launch_list_count(B.d_desc, B.d_state, P.p, B.c->stream);
        }
    }
    return ICX_OK;
}

// After the synchronisation of a stage whose FDCT covered `ids`: the list
// entries each image's FDCT wrote (device counter), and the FDCT's algorithmic
// bytes - pixels read + lists, list offsets and lengths written.
void credit_fdct(Batch& B, const std::vector<int>& ids)
{
    int64_t bytes = 0;
    for (int i : ids) {
        const ImgDesc& d = B.desc[i];
        int64_t e = 0;
        for (int k = 0; k < ENT_SLOTS; k++) e += (int64_t)B.state[i].list_entries[k];
        B.it[i].entries = e;
        bytes += (int64_t)d.w * d.h * B.it[i].nch + 4 * B.it[i].entries + 5 * d.nblocks;
    }
    if (B.c->prof) B.c->stats["fdct.bytes"].units += bytes;
}

// Blocks actually quantised+coded by the trials of `ids` since their state
// was initialised (inactive images exit k_huff at once): the huff kernel's
// algorithmic work - and bytes: every trial reads each block's list (padded
// entries), its offset and its length, and writes its bitstream (the trial
// that fits is the file: no re-encode) with the chunks' bit counts and 0xFF
// bins - credited after the stage's synchronisation.
void credit_huff(Batch& B, const std::vector<int>& ids)
{
    if (!B.c->prof) return;
    int64_t blocks = 0, bytes = 0;
    for (int i : ids) {
        blocks += (int64_t)B.state[i].ntrials * B.desc[i].nblocks;
        bytes += (int64_t)B.state[i].ntrials * (4 * B.it[i].entries + 5 * B.desc[i].nblocks) +
                 (int64_t)B.state[i].huff_wbytes;
    }
    B.c->stats["huff"].units += blocks;
    B.c->stats["huff.bytes"].units += bytes;
}

// `depth` trials (k_huff + k_scan with its search step) for the images in ids,
// then - finals - the final file of every image whose search has a best
// trial (k_ffscan / k_stuff skip the others), all without a host round trip:
// the stage's one synchronisation then also returns the files' lengths.
icx_status run_trials(Batch& B, const std::vector<int>& ids, int depth, bool finals)
{
    std::vector<int64_t> cnt;
    for (int i : ids) cnt.push_back(B.desc[i].nchunks);
    DPlan P;
    icx_status s = make_plan(B, ids, cnt, P);
    if (s || (s = B.up->flush())) return s;
    icx_ctx* c = B.c;
    for (int t = 0; t < depth; t++) {
        { Timed tm(c, "huff", 0, true); launch_huff(B.d_desc, B.d_state, B.d_nodes, P.p, P.total, (B.huff_launches++) & 1, c->stream); }
        { Timed tm(c, "scan", (int64_t)ids.size(), true); launch_scan(B.d_desc, B.d_state, B.d_nodes, P.p, c->stream); }
    }
    if (finals) {
        { Timed tm(c, "ffscan", (int64_t)ids.size(), true); launch_ffscan(B.d_desc, B.d_state, P.p, c->stream); }
        { Timed tm(c, "stuff", P.total, true); launch_stuff(B.d_desc, B.d_state, B.d_nodes, P.p, P.total, c->stream); }
    }
    return ICX_OK;
}

void init_state(ImgState& s, int node, bool force)
{
    memset(&s, 0, sizeof(s));
    s.node = node;
    s.best_node = -1;
    s.cur = 0;
    s.best_buf = 1;
    s.active = node >= 0;
    s.force = force;
}

int kind_of(int fmt) { return fmt == ICX_BGR24 ? 0 : fmt == ICX_RGB24 ? 1 : 2; }

icx_status validate(const icx_image* img)
{
    if (!img || !img->px) return ICX_E_NULL;
    if (img->width <= 0 || img->height <= 0 || img->width > 65535 || img->height > 65535) return ICX_E_INVALID;
    if (img->fmt < ICX_BGR24 || img->fmt > ICX_BINARY1) return ICX_E_INVALID;
    if (is_palette(img->fmt) && (!img->palette || img->palette_len < 1 ||
                                 img->palette_len > (img->fmt == ICX_BINARY1 ? 16 : 256)))
        return ICX_E_INVALID;
    if (img->stride < img->width * channels(img->fmt)) return ICX_E_INVALID;
    if (channels(img->fmt) == 4 && (((uintptr_t)img->px | (uintptr_t)img->stride) & 3)) return ICX_E_INVALID;
    if (channels(img->fmt) == 2 && (((uintptr_t)img->px | (uintptr_t)img->stride) & 1)) return ICX_E_INVALID;
    return ICX_OK;
}

// Core driver.  mode Fit: A2 per job; Encode: A4 (job.quality, forced);
// Search: A3 only (no output); Fdct: coefficients only (debug).
icx_status run_batch(icx_ctx* c, icx_fit_job* jobs, int n, Mode mode, int16_t* fdct_out = nullptr,
                     ImgState* search_out = nullptr)
{
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    HostSpan call{c, "host.call_fit"};  // the whole call, wall time (profiling)
    hipError_t he = hipSetDevice(c->device);
    if (he != hipSuccess) return hip_fail(c, he, "hipSetDevice");
    std::vector<int> order;
    for (int i = 0; i < n; i++) {
        icx_fit_job& j = jobs[i];
        j.success = 0;
        j.cache_hit = 0;
        j.out_len = 0;
        j.learned.quality = -1.0f;
        j.learned.scale = 0.0;
        j.encodes = 0;
        j.status = validate(&j.img);
        if (j.status == ICX_OK && j.img.fmt > ICX_GRAY8) j.status = ICX_E_UNSUPPORTED;  // JPEG: no alpha rasters
        if (j.status == ICX_OK && mode != Mode::Search && mode != Mode::Fdct && !j.out) j.status = ICX_E_NULL;
        if (j.status == ICX_OK) order.push_back(i);
    }
    // ---- device workspace per image (what the sub-batch loop below takes);
    // host inputs and outputs are staged separately (stage_bytes), in one of
    // two arenas that alternate between sub-batches
    auto out_staging = [&](const icx_fit_job& j) -> size_t {
        if (!(mode == Mode::Fit || mode == Mode::Encode) || is_device_ptr(j.out)) return 0;
        ImgDesc g{};
        geometry(g, j.img.width, j.img.height, j.img.fmt);
        return std::min<uint64_t>(worst_file(g), j.cap);
    };
    auto stage_bytes = [&](const icx_fit_job& j) -> size_t {
        const size_t px = (size_t)j.img.width * j.img.height * channels(j.img.fmt);
        return (is_device_ptr(j.img.px) ? 0 : align_up(px, 256)) + align_up(out_staging(j), 256);
    };
    auto workspace = [&](const icx_fit_job& j) -> size_t {
        ImgDesc g{};
        geometry(g, j.img.width, j.img.height, j.img.fmt);
        const size_t px = (size_t)j.img.width * j.img.height * channels(j.img.fmt);
        size_t per = coef_bytes(g) + ((size_t)g.nchunks * CHUNK_BLOCKS + 1) * 5 + 512 + (size_t)g.nblocks * BLOCK_WORDS * 4 + 1024 +
                     2 * ((size_t)g.nchunks * CHUNK_WORDS + 1) * 4 +
                     (size_t)g.nchunks * (2 * 4 + 2 * 8 + 2 * 4 + 2 * 32 + 8) + 64 + 8 * 256 + 4096;
        if (mode == Mode::Fit) per += px;  // resize buffer
        return per;
    };
    // Sub-batches of about equal size: as few as the budget allows (the two
    // staging arenas count against it).
    size_t all_need = 0, all_stage = 0;
    for (int i : order) {
        all_need += workspace(jobs[i]) + 2 * stage_bytes(jobs[i]);
        all_stage += stage_bytes(jobs[i]);
    }
    size_t nsub = std::max<size_t>(1, (all_need + c->budget - 1) / c->budget);
    // Host buffers: sub-batches of ~512 MB of uploads (up to 16), so that all
    // but the first upload and the last sub-batch's kernels and downloads
    // overlap (the link moves ~57 GB/s, the kernels ~30x that)
    if (all_stage > 0)
        nsub = std::max(nsub, std::min<size_t>({16, order.size(), (all_stage + (512u << 20) - 1) / (512u << 20)}));
    const size_t share = (all_need + nsub - 1) / nsub;
    std::vector<std::vector<int>> subs;
    std::vector<size_t> sub_need;
    size_t stage_max = 0;
    for (size_t pos = 0; pos < order.size();) {
        std::vector<int> sub;
        size_t need = 1 << 20, acct = 1 << 20, st = 0;
        while (pos < order.size()) {
            const icx_fit_job& j = jobs[order[pos]];
            const size_t per = workspace(j), sb = stage_bytes(j);
            if (!sub.empty() && (acct + per + 2 * sb > c->budget || acct - (1 << 20) >= share)) break;
            need += per;
            acct += per + 2 * sb;
            st += sb;
            sub.push_back(order[pos++]);
        }
        stage_max = std::max(stage_max, st);
        subs.push_back(std::move(sub));
        sub_need.push_back(need);
    }
    // ---- host staging: uploads of sub-batch s+1 (io_up) run while s
    // computes; downloads of s (io_down) while s+1 computes
    struct HostIO {
        std::vector<uint8_t*> px, out;
        bool up = false, down = false, wait = false;
    };
    std::vector<HostIO> hio(subs.size());
    struct IoDrain {  // every exit waits for the copies that touch the caller's buffers
        icx_ctx* c;
        ~IoDrain()
        {
            if (c->io_up) hipStreamSynchronize(c->io_up);
            if (c->io_down) hipStreamSynchronize(c->io_down);
        }
    } io_drain{c};
    if (stage_max > 0) {
        if (!c->io_up) {
            hipError_t e = hipStreamCreateWithFlags(&c->io_up, hipStreamNonBlocking);
            if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->io_down, hipStreamNonBlocking);
            for (int b = 0; b < 2 && e == hipSuccess; b++) {
                e = hipEventCreateWithFlags(&c->ev_up[b], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_down[b], hipEventDisableTiming);
            }
            if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming);
            if (e != hipSuccess) return hip_fail(c, e, "host I/O streams");
        }
        // both arenas reserved before any work: a re-allocation (hipFree)
        // would synchronise the device in the middle of the pipeline
        for (int b = 0; b < 2 && b < (int)subs.size(); b++) {
            hipError_t e = c->stage[b].reserve(stage_max + 4096);
            if (e != hipSuccess) {
                for (int i : order) jobs[i].status = ICX_E_NOMEM;
                (void)hipGetLastError();
                return fail(c, ICX_E_NOMEM, "host staging allocation failed");
            }
        }
    }
    auto prefetch = [&](size_t si) -> icx_status {
        if (si >= subs.size() || stage_max == 0) return ICX_OK;
        const std::vector<int>& sub = subs[si];
        HostIO& H = hio[si];
        DevArena& A = c->stage[si & 1];
        A.used = 0;
        H.px.assign(sub.size(), nullptr);
        H.out.assign(sub.size(), nullptr);
        // the arena's last reader (sub-batch si-2's downloads) must be done
        hipError_t e = hipStreamWaitEvent(c->io_up, c->ev_down[si & 1], 0);
        for (size_t k = 0; k < sub.size() && e == hipSuccess; k++) {
            const icx_fit_job& j = jobs[sub[k]];
            if (!is_device_ptr(j.img.px)) {
                const size_t row = (size_t)j.img.width * channels(j.img.fmt);
                H.px[k] = (uint8_t*)A.take(row * j.img.height);
                e = (size_t)j.img.stride == row  // packed rows: one linear copy
                        ? hipMemcpyAsync(H.px[k], j.img.px, row * j.img.height, hipMemcpyHostToDevice, c->io_up)
                        : hipMemcpy2DAsync(H.px[k], row, j.img.px, j.img.stride, row, j.img.height,
                                           hipMemcpyHostToDevice, c->io_up);
                H.up = true;
            }
            if (out_staging(j)) {
                H.out[k] = (uint8_t*)A.take(out_staging(j));
                H.down = true;
            }
        }
        // ev_up orders c->stream behind the arena's reuse: behind the uploads,
        // and (recorded after the wait on ev_down above) behind sub-batch
        // si-2's downloads from the same arena.  Recorded whenever the arena
        // is written here at all - a sub-batch with device inputs and host
        // outputs uploads nothing, but its kernels still overwrite the bytes
        // si-2's downloads may be reading.
        H.wait = H.up || H.down;
        if (e == hipSuccess && H.wait) e = hipEventRecord(c->ev_up[si & 1], c->io_up);
        return e == hipSuccess ? ICX_OK : hip_fail(c, e, "input upload");
    };
    if (icx_status ps = prefetch(0)) return ps;
    for (size_t si = 0; si < subs.size(); si++) {
        std::unique_ptr<HostSpan> prep(new HostSpan{c, "host.prep"});  // until the first launch
        const std::vector<int>& sub = subs[si];
        const size_t need = sub_need[si];
        if (c->prof) {  // sub-batches per call and their workspace (reported by bench.py)
            c->stats["subbatch"].launches++;
            c->stats["subbatch"].units += (int64_t)(need >> 20);
        }
        hipError_t e = c->dev.reserve(need + ((size_t)sub.size() + 8) * 4096 + (16 << 20));
        if (e != hipSuccess) {
            for (int i : sub) jobs[i].status = ICX_E_NOMEM;
            (void)hipGetLastError();
            c->err = "device workspace allocation failed";
            if (icx_status ps = prefetch(si + 1)) return ps;  // the next sub-batch still needs its inputs
            continue;
        }
        c->dev.used = 0;
        c->dev.overflow = false;
        e = c->host.reserve(64 << 20);
        if (e != hipSuccess) return hip_fail(c, e, "hipHostMalloc");
        c->host.used = 0;

        Batch B;
        B.c = c;
        const int m = (int)sub.size();
        B.it.resize(m);
        B.desc.assign(m, ImgDesc{});
        B.state.assign(m, ImgState{});
        int max_depth = 0;
        std::map<uint32_t, int> tree_of_q;   // bit pattern of q0 -> root
        std::map<uint32_t, int> depth_of_q;
        std::map<uint32_t, int> single_of_q; // fixed-quality node
        auto single = [&](float q) {
            uint32_t key;
            memcpy(&key, &q, 4);
            auto f = single_of_q.find(key);
            if (f != single_of_q.end()) return f->second;
            int idx = (int)B.nodes.size();
            B.nodes.emplace_back();
            make_node(q, B.nodes[idx]);
            single_of_q[key] = idx;
            return idx;
        };
        for (int k = 0; k < m; k++) {
            icx_fit_job& j = jobs[sub[k]];
            Item& I = B.it[k];
            I.job = &j;
            I.kind = kind_of(j.img.fmt);
            I.nch = channels(j.img.fmt);
            I.done = I.found = I.hit = false;
            I.best_q = -1.0f;
            I.best_scale = 0;
            I.encodes = 0;
            I.coef_scale = NAN;
            I.entries = 0;
            I.root = I.cached_node = -1;
            I.depth = 0;
            ImgDesc& d = B.desc[k];
            geometry(d, j.img.width, j.img.height, j.img.fmt, c->table_layout);
            d.stride = j.img.stride;
            d.target = j.target_max_size;
            d.coefs = (int32_t*)c->dev.take(coef_bytes(d));
            d.coff = (uint32_t*)c->dev.take(((size_t)d.nchunks * CHUNK_BLOCKS + 1) * 4);  // + the dummy slot (store_list_meta)
            d.ncoef = (uint8_t*)c->dev.take((size_t)d.nchunks * CHUNK_BLOCKS + 1);
            d.ovf = (uint32_t*)c->dev.take((size_t)d.nblocks * BLOCK_WORDS * 4 + 1024);
            for (int b = 0; b < 2; b++) {
                d.scratch[b] = (uint32_t*)c->dev.take(((size_t)d.nchunks * CHUNK_WORDS + 1) * 4);
                d.chunk_bits[b] = (uint32_t*)c->dev.take((size_t)d.nchunks * 4);
                d.chunk_off[b] = (uint64_t*)c->dev.take(((size_t)d.nchunks + 1) * 8);
                d.chunk_ff[b] = (uint32_t*)c->dev.take((size_t)d.nchunks * 4);
                d.chunk_ffa[b] = (uint32_t*)c->dev.take((size_t)d.nchunks * 32);
            }
            d.chunk_ffoff = (uint64_t*)c->dev.take((size_t)d.nchunks * 8);
            // input pixels (host rows: uploaded into the staging arena by prefetch)
            if (hio[si].px.empty() || !hio[si].px[k]) {
                I.dpx = j.img.px;
            } else {
                I.dpx = hio[si].px[k];
                d.stride = (int32_t)((size_t)j.img.width * I.nch);
            }
            d.px = I.dpx;
            I.orig = d;
            I.dresize = (mode == Mode::Fit) ? (uint8_t*)c->dev.take((size_t)j.img.width * j.img.height * I.nch)
                                            : nullptr;
            // output
            I.host_out = false;
            I.dout = nullptr;
            if (mode == Mode::Fit || mode == Mode::Encode) {
                if (hio[si].out.empty() || !hio[si].out[k]) {
                    I.dout = j.out;
                    d.cap = j.cap;
                } else {  // staging bound >= any file we can produce
                    I.dout = hio[si].out[k];
                    I.host_out = true;
                    d.cap = std::min<uint64_t>(worst_file(d), j.cap);
                }
            }
            d.out = I.dout;
            I.orig = d;
            // quality nodes
            if (mode == Mode::Fit || mode == Mode::Search) {
                uint32_t key;
                memcpy(&key, &j.quality, 4);
                auto f = tree_of_q.find(key);
                if (f == tree_of_q.end()) {
                    int depth = 0;
                    int root = build_tree(0.0f, j.quality, 0, B.nodes, depth);
                    tree_of_q[key] = root;
                    depth_of_q[key] = depth;
                    f = tree_of_q.find(key);
                }
                I.root = f->second;
                I.depth = depth_of_q[key];
                max_depth = std::max(max_depth, I.depth);
                if (mode == Mode::Fit && j.has_cached) I.cached_node = single(j.cached.quality);
            } else if (mode == Mode::Encode) {
                I.cached_node = single(j.quality);
            }
        }
        // Candidate filter of each image: per coefficient, the smallest
        // quantiser threshold over every node a trial of this image can reach
        // (cached probe + search tree).  The FDCT keeps only coefficients at or
        // above it - every one that can quantise to nonzero in some trial.  No
        // reachable node (debug FDCT): all-zero thresholds keep every coefficient.
        std::map<std::pair<int, int>, int> cand_of;
        for (int k = 0; k < m; k++) {
            Item& I = B.it[k];
            const auto key = std::make_pair(I.root, I.cached_node);
            auto f = cand_of.find(key);
            if (f == cand_of.end()) {
                QNode cn{};
                std::vector<int> todo;
                if (I.root >= 0) todo.push_back(I.root);
                if (I.cached_node >= 0) todo.push_back(I.cached_node);
                bool first = true;
                while (!todo.empty()) {
                    const int n = todo.back();
                    todo.pop_back();
                    for (int c = 0; c < 2; c++)
                        for (int z = 0; z < 64; z++)
                            cn.qf[c][z].x = first ? B.nodes[n].qf[c][z].x : std::min(cn.qf[c][z].x, B.nodes[n].qf[c][z].x);
                    first = false;
                    if (B.nodes[n].child_fit >= 0) todo.push_back(B.nodes[n].child_fit);
                    if (B.nodes[n].child_nofit >= 0) todo.push_back(B.nodes[n].child_nofit);
                }
                cn.child_fit = cn.child_nofit = -1;
                B.nodes.push_back(cn);
                f = cand_of.emplace(key, (int)B.nodes.size() - 1).first;
            }
            B.desc[k].cand_node = f->second;
            I.orig.cand_node = f->second;
        }
        B.d_nodes = (QNode*)c->dev.take(sizeof(QNode) * B.nodes.size());
        B.h_state = (ImgState*)c->host.take(sizeof(ImgState) * m);
        if (!B.h_state) return fail(c, ICX_E_NOMEM, "pinned staging exhausted");
        icx_status s = upload(c, B.d_nodes, B.nodes.data(), sizeof(QNode) * B.nodes.size());
        if (s) return s;
        // this sub-batch's pixels have landed (and the arena's previous
        // downloads have drained) before its first kernel; the next
        // sub-batch's upload starts behind them on io_up
        if (hio[si].wait && (e = hipStreamWaitEvent(c->stream, c->ev_up[si & 1], 0)) != hipSuccess)
            return hip_fail(c, e, "hipStreamWaitEvent");
        if ((s = prefetch(si + 1))) return s;

        std::vector<int> all(m);
        for (int k = 0; k < m; k++) all[k] = k;
        prep.reset();

        if (mode == Mode::Fdct) {
            for (int k = 0; k < m; k++) init_state(B.state[k], -1, false);
            if ((s = push_desc_state(B)) || (s = run_fdct(B, all)) || (s = sync_states(B))) return s;
            const ImgDesc& d0 = B.desc[0];
            std::vector<int32_t> raw(coef_bytes(d0) / 4);
            std::vector<uint32_t> off((size_t)d0.nblocks);
            std::vector<uint8_t> cnt((size_t)d0.nblocks);
            e = hipMemcpy(raw.data(), d0.coefs, raw.size() * 4, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(off.data(), d0.coff, off.size() * 4, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(cnt.data(), d0.ncoef, cnt.size(), hipMemcpyDeviceToHost);
            if (e != hipSuccess) return hip_fail(c, e, "coef download");
            for (int64_t blk = 0; blk < d0.nblocks; blk++) {  // lists -> block-major zig-zag
                if (cnt[blk] != 64 || (size_t)off[blk] * 4 + 64 > raw.size())
                    return fail(c, ICX_E_DEVICE, "debug FDCT list is not complete");
                for (int i = 0; i < 64; i++) {
                    const uint32_t v = (uint32_t)raw[(size_t)off[blk] * 4 + i], cb = v & ~0x3FFu;
                    float cf;
                    std::memcpy(&cf, &cb, 4);
                    fdct_out[blk * 64 + ((v >> 3) & 63)] = (int16_t)cf;
                }
            }
            continue;
        }

        if (mode == Mode::Encode) {  // A4: one forced encode
            for (int k = 0; k < m; k++) init_state(B.state[k], B.it[k].cached_node, true);
            if ((s = push_desc_state(B)) || (s = run_fdct(B, all)) || (s = run_trials(B, all, 1, true)) ||
                (s = sync_states(B)))
                return s;
            credit_fdct(B, all);
            credit_huff(B, all);
            for (int k = 0; k < m; k++) {
                B.it[k].found = B.state[k].best_node >= 0;
                B.it[k].best_q = jobs[sub[k]].quality;
                B.it[k].best_scale = 1.0;
                B.it[k].encodes = B.state[k].ntrials;
            }
        } else {
            // ---- stage 0: tryCachedParams (ImageCompressionJpg.java:82-89, :216-238)
            std::vector<int> probe;
            if (mode == Mode::Fit)
                for (int k = 0; k < m; k++)
                    if (B.it[k].cached_node >= 0) probe.push_back(k);
            for (int k = 0; k < m; k++) init_state(B.state[k], -1, false);
            if (!probe.empty()) {
                for (int k : probe) {
                    const double sc = jobs[sub[k]].cached.scale;
                    stage_pixels(B, k, sc < 1.0 ? sc : 1.0);
                    init_state(B.state[k], B.it[k].cached_node, false);
                    B.it[k].coef_scale = sc < 1.0 ? sc : 1.0;
                }
                if ((s = push_desc_state(B)) || (s = run_fdct(B, probe)) || (s = run_trials(B, probe, 1, true)) ||
                    (s = sync_states(B)))
                    return s;
                credit_fdct(B, probe);
                credit_huff(B, probe);
                for (int k : probe) {
                    B.it[k].encodes += B.state[k].ntrials;
                    if (B.state[k].best_node >= 0) {
                        Item& I = B.it[k];
                        I.found = I.hit = I.done = true;
                        I.best_q = jobs[sub[k]].cached.quality;
                        I.best_scale = jobs[sub[k]].cached.scale;
                    }
                }
            }
            // ---- scale loop (ImageCompressionJpg.java:91-115)
            std::vector<int> pend;
            for (int k = 0; k < m; k++)
                if (!B.it[k].done) pend.push_back(k);
            const double STEP = 0.85;
            for (double scale = 1.0; scale > 0.1 && !pend.empty(); scale = (scale == 1.0) ? STEP : scale * STEP) {
                std::vector<int> need_fdct;
                int depth = 0;
                for (int k : pend) {
                    if (!(B.it[k].coef_scale == scale)) {
                        stage_pixels(B, k, scale);
                        need_fdct.push_back(k);
                        B.it[k].coef_scale = scale;
                    }
                    init_state(B.state[k], B.it[k].root, false);
                    depth = std::max(depth, B.it[k].depth);
                }
                if ((s = push_desc_state(B)) || (s = run_fdct(B, need_fdct)) ||
                    (s = run_trials(B, pend, depth, mode != Mode::Search)) || (s = sync_states(B)))
                    return s;
                credit_fdct(B, need_fdct);
                credit_huff(B, pend);
                std::vector<int> rest;
                for (int k : pend) {
                    Item& I = B.it[k];
                    I.encodes += B.state[k].ntrials;
                    if (mode == Mode::Search) {  // A3 only: report the first scale's search
                        I.done = true;
                        I.found = B.state[k].best_node >= 0;
                        I.best_q = I.found ? B.nodes[B.state[k].best_node].mid : -1.0f;
                        continue;
                    }
                    if (B.state[k].best_node >= 0) {
                        I.found = I.done = true;
                        I.best_q = B.nodes[B.state[k].best_node].mid;
                        I.best_scale = scale;
                    } else {
                        rest.push_back(k);
                    }
                }
                if (mode == Mode::Search) break;
                pend.swap(rest);
            }
        }
        // ---- results + host outputs (downloads on io_down, behind this
        // sub-batch's kernels; they overlap the next sub-batch)
        HostSpan res{c, "host.results"};
        if (hio[si].down) {
            if ((e = hipEventRecord(c->ev_done, c->stream)) != hipSuccess ||
                (e = hipStreamWaitEvent(c->io_down, c->ev_done, 0)) != hipSuccess)
                return hip_fail(c, e, "output download");
        }
        for (int k = 0; k < m; k++) {
            Item& I = B.it[k];
            icx_fit_job& j = *I.job;
            j.encodes = I.encodes;
            if (mode == Mode::Search) {
                j.learned.quality = I.best_q;
                j.success = I.found;
                j.status = ICX_OK;
                continue;
            }
            if (!I.found) {
                j.success = 0;
                j.status = ICX_OK;
                continue;
            }
            j.success = 1;
            j.cache_hit = I.hit;
            j.learned.quality = I.best_q;
            j.learned.scale = I.best_scale;
            j.out_len = (size_t)B.state[k].out_len;
            if (B.state[k].status == 4 || j.out_len > j.cap) {
                j.status = ICX_E_BUFFER;
                continue;
            }
            j.status = ICX_OK;
            if (I.host_out) {
                e = hipMemcpyAsync(j.out, I.dout, j.out_len, hipMemcpyDeviceToHost, c->io_down);
                if (e != hipSuccess) return hip_fail(c, e, "output download");
            }
        }
        if (hio[si].down && (e = hipEventRecord(c->ev_down[si & 1], c->io_down)) != hipSuccess)
            return hip_fail(c, e, "output download");
        e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "hipStreamSynchronize");
        if (search_out && m > 0 && sub[0] == 0) *search_out = B.state[0];  // trial record of job 0
    }
    resolve_profile(c);  // off the critical path: the device is idle between calls anyway
    return ICX_OK;
}

}  // namespace

// ============================================================ C ABI
namespace {
// Constant tables of the encoder (zig-zag, Huffman codes, marker templates,
// dither errors): built once per process, uploaded once per DEVICE
// (__constant__ symbols live on every device: a pool over several GPUs
// needs them on each).
struct Consts {
    uint8_t nat2zz[64], zz2nat[64];
    uint32_t dc[2][16] = {}, ac[2][256] = {};
    uint8_t hdr[4][HDR_COLOR] = {};
    int8_t dith[3][64];
};
const Consts& consts();

// The self-check's known-answer images: a 16x16 BGR24 frame and a 16x16
// GRAY8 frame of busy content (every AC table is reached), encoded at
// quality 0.75 with the default table layout.  Their files' length and
// 64-bit FNV-1a digest are pinned against the CPU oracle by
// tests/test_capi.py (test_self_check_vectors_match_oracle).
constexpr float kSelfCheckQ = 0.75f;
void self_check_image(int grey, uint8_t* px)
{
    const int nch = grey ? 1 : 3;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++)
            for (int c = 0; c < nch; c++)
                px[(y * 16 + x) * nch + c] = (uint8_t)((x * 37 + y * 91 + c * 53 + x * y * 13 + ((x ^ y) & 5) * 29) & 255);
}
constexpr uint64_t kSelfCheckDigest[2] = {0x937d6de3e49b4eb4ull, 0xae63ed12585b37ccull};  // [colour, grey]
constexpr int64_t kSelfCheckLen[2] = {776, 470};
uint64_t fnv1a64(const uint8_t* p, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

// Device self-check of a new context: a constant table
// missing or wrong on this device (an upload to the wrong device, a stale
// symbol) fails icx_create instead of corrupting this GPU's output.
//  * the first context on a device: one colour and one grey 16x16 encode,
//    compared with the known answers (the whole encoder, tables included);
//  * every context: the device's digest of its constant tables
//    (k_const_digest) against the host's, ~0.1 ms.
bool self_check_off()
{
    const char* e = getenv("ICX_SELF_CHECK");
    return e && atoi(e) == 0;
}

icx_status self_check_encode(icx_ctx* c)
{
    uint8_t px[2][16 * 16 * 3];
    uint8_t out[2][2048];
    icx_fit_job j[2] = {};
    for (int g = 0; g < 2; g++) {
        self_check_image(g, px[g]);
        j[g].img = icx_image{px[g], 16, 16, g ? 16 : 48, g ? ICX_GRAY8 : ICX_BGR24, nullptr, 0};
        j[g].quality = kSelfCheckQ;
        j[g].out = out[g];
        j[g].cap = sizeof(out[g]);
        j[g].target_max_size = INT64_MAX;
    }
    const icx_status s = run_batch(c, j, 2, Mode::Encode);
    if (s != ICX_OK) return s;
    for (int g = 0; g < 2; g++) {
        if (j[g].status != ICX_OK) return fail(c, ICX_E_DEVICE, "device self-check: encode failed");
        if ((int64_t)j[g].out_len != kSelfCheckLen[g] || fnv1a64(out[g], j[g].out_len) != kSelfCheckDigest[g])
            return fail(c, ICX_E_DEVICE, g ? "device self-check: grey known answer differs"
                                           : "device self-check: colour known answer differs");
    }
    return ICX_OK;
}
}  // namespace

namespace {
const Consts& consts()
{
    static std::once_flag once;
    static Consts K;
    std::call_once(once, [] {
        uint8_t* nat2zz = K.nat2zz;
        uint8_t* zz2nat = K.zz2nat;
        for (int k = 0; k < 64; k++) {
            zz2nat[k] = kZigzag[k];
            nat2zz[kZigzag[k]] = (uint8_t)k;
        }
        auto& dc = K.dc;
        auto& ac = K.ac;
        auto derive = [](const uint8_t* bits, const uint8_t* vals, uint32_t* tbl) {
            unsigned code = 0;
            int k = 0;
            for (int l = 1; l <= 16; l++) {
                for (int i = 0; i < bits[l - 1]; i++, k++) tbl[vals[k]] = (code++ << 8) | (uint32_t)l;
                code <<= 1;
            }
        };
        derive(kDcLumBits, kDcVals, dc[0]);
        derive(kDcChrBits, kDcVals, dc[1]);
        derive(kAcLumBits, kAcLumVals, ac[0]);
        derive(kAcChrBits, kAcChrVals, ac[1]);
        auto& hdr = K.hdr;
        for (int g = 0; g < 4; g++) {
            const int nc = (g & 1) ? 3 : 1;
            const bool grouped = g >= 2;  // ICX_TABLES_GROUPED: one DQT and one DHT segment
            std::vector<uint8_t> h;
            auto put = [&](std::initializer_list<int> v) { for (int x : v) h.push_back((uint8_t)x); };
            put({0xFF, 0xD8});
            // APP0 as the JDK's JFIFMarkerSegment writes it: JFIF 1.02, aspect-ratio units, 1x1
            put({0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00, 0x01, 0x02, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00});
            const int nt = nc == 3 ? 2 : 1;
            for (int t = 0; t < nt; t++) {
                if (t == 0 || !grouped) put({0xFF, 0xDB, 0x00, 2 + (grouped ? nt : 1) * 65});
                put({t});
                for (int i = 0; i < 64; i++) h.push_back(0);  // DQT payload patched on device
            }
            put({0xFF, 0xC0, 0x00, 8 + 3 * nc, 8, 0, 0, 0, 0, nc});
            if (nc == 1) put({1, 0x11, 0});
            else put({1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1});
            auto count = [](const uint8_t* bits) {
                int cnt = 0;
                for (int i = 0; i < 16; i++) cnt += bits[i];
                return cnt;
            };
            // grouped: one segment whose length covers every table of the header
            int all = 2 * 17 + count(kDcLumBits) + count(kAcLumBits);
            if (nc == 3) all += 2 * 17 + count(kDcChrBits) + count(kAcChrBits);
            bool first = true;
            auto dht = [&](int idx, const uint8_t* bits, const uint8_t* vals) {
                const int cnt = count(bits);
                if (!grouped) put({0xFF, 0xC4, (19 + cnt) >> 8, (19 + cnt) & 255});
                else if (first) put({0xFF, 0xC4, (2 + all) >> 8, (2 + all) & 255});
                first = false;
                put({idx});
                for (int i = 0; i < 16; i++) h.push_back(bits[i]);
                for (int i = 0; i < cnt; i++) h.push_back(vals[i]);
            };
            dht(0x00, kDcLumBits, kDcVals);
            dht(0x10, kAcLumBits, kAcLumVals);
            if (nc == 3) {
                dht(0x01, kDcChrBits, kDcVals);
                dht(0x11, kAcChrBits, kAcChrVals);
            }
            if (nc == 1) put({0xFF, 0xDA, 0x00, 0x08, 1, 1, 0x00, 0, 63, 0});
            else put({0xFF, 0xDA, 0x00, 0x0C, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0});
            if ((int)h.size() != (nc == 3 ? (grouped ? HDR_COLOR_GROUPED : HDR_COLOR)
                                          : (grouped ? HDR_GRAY_GROUPED : HDR_GRAY))) abort();
            memcpy(hdr[g], h.data(), h.size());
        }
        dither_tables(K.dith);
    });
    return K;
}
}  // namespace

extern "C" {

int icx_abi_version(void) { return ICX_ABI_VERSION; }

const char* icx_status_string(icx_status s)
{
    switch (s) {
    case ICX_OK: return "ok";
    case ICX_E_INVALID: return "invalid argument";
    case ICX_E_NOMEM: return "out of memory";
    case ICX_E_DEVICE: return "device error";
    case ICX_E_BUFFER: return "output buffer too small";
    case ICX_E_UNSUPPORTED: return "unsupported input";
    case ICX_E_CORRUPT: return "corrupt input";
    case ICX_E_NULL: return "null argument";
    case ICX_E_REFUSED: return "a JPEG flavour the reference's reader refuses";
    }
    return "unknown";
}

const char* icx_last_error(const icx_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }


int32_t icx_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

void icx_debug_self_check_image(int32_t grey, uint8_t* px, uint64_t* digest, int64_t* len)
{
    const int g = grey ? 1 : 0;
    if (px) self_check_image(g, px);
    if (digest) *digest = kSelfCheckDigest[g];
    if (len) *len = kSelfCheckLen[g];
}

icx_status icx_debug_corrupt_constants(int32_t device, int32_t on)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return ICX_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return ICX_E_DEVICE;
    const Consts& K = consts();
    Consts bad = K;
    if (on) bad.ac[0][0x01] ^= 0x100;  // the luma AC code of run 0 / size 1: wrong bits, same length
    return upload_constants(bad.nat2zz, bad.zz2nat, bad.dc, bad.ac, bad.hdr, bad.dith) == hipSuccess ? ICX_OK
                                                                                                      : ICX_E_DEVICE;
}

icx_status icx_create(int device, icx_ctx** out)
{
    if (!out) return ICX_E_NULL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return ICX_E_DEVICE;
    }
    if (device < 0 || device >= n) return ICX_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return ICX_E_DEVICE;
    icx_ctx* c = new icx_ctx();
    c->device = device;
    c->hpool.host = true;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return ICX_E_DEVICE;
    }
    static std::mutex up_mu;
    static std::vector<int> up_done;
    const Consts& K = consts();
    hipError_t up = hipSuccess;
    {
        std::lock_guard<std::mutex> lk(up_mu);
        if (std::find(up_done.begin(), up_done.end(), device) == up_done.end()) {
            up = upload_constants(K.nat2zz, K.zz2nat, K.dc, K.ac, K.hdr, K.dith);
            if (up == hipSuccess) up_done.push_back(device);
        }
    }
    if (up != hipSuccess) {
        hipStreamDestroy(c->stream);
        delete c;
        return ICX_E_DEVICE;
    }
    // Sub-batch workspace: two fifths of the free HBM at creation (a 4K image
    // needs ~190 MB, so ~110 GB of a 288 GB MI355X holds 500+ frames per
    // sub-batch and the host synchronises a few times per call, not per
    // handful of images: 1000 4K frames in two sub-batches instead of three,
    // -1.2 % step time).  The arena is reserved per call at what it needs.
    size_t free_b = 0, total_b = 0;
    size_t budget_mb = 16384;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
        budget_mb = std::max<size_t>(2048, (free_b / 5 * 2) >> 20);
    if (const char* env = getenv("ICX_WORKSPACE_MB")) budget_mb = (size_t)atoll(env);
    c->budget = budget_mb << 20;
    if (!self_check_off()) {
        // (up_mu: one digest buffer per device; the first context's encode check)
        std::lock_guard<std::mutex> lk(up_mu);
        static std::vector<std::pair<int, uint64_t*>> digest_buf;
        static std::vector<int> encode_checked;
        uint64_t* d_dig = nullptr;
        for (auto& b : digest_buf)
            if (b.first == device) d_dig = b.second;
        hipError_t e = hipSuccess;
        if (!d_dig && (e = hipMalloc(&d_dig, sizeof(uint64_t))) == hipSuccess) digest_buf.push_back({device, d_dig});
        uint64_t got = 0;
        if (e == hipSuccess) {
            launch_const_digest(d_dig, c->stream);
            e = hipMemcpyAsync(&got, d_dig, sizeof(got), hipMemcpyDeviceToHost, c->stream);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        const uint64_t want = const_digest_host(K.nat2zz, K.zz2nat, K.dc, K.ac, K.hdr, K.dith);
        icx_status st = e != hipSuccess ? ICX_E_DEVICE : got != want ? ICX_E_DEVICE : ICX_OK;
        if (st == ICX_OK && std::find(encode_checked.begin(), encode_checked.end(), device) == encode_checked.end()) {
            st = self_check_encode(c);
            if (st == ICX_OK) encode_checked.push_back(device);
        }
        if (st != ICX_OK) {
            (void)hipGetLastError();
            icx_destroy(c);
            return ICX_E_DEVICE;
        }
    }
    *out = c;
    return ICX_OK;
}


void icx_destroy(icx_ctx* ctx)
{
    if (!ctx) return;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
    for (auto e : ctx->evpool) hipEventDestroy(e);
    for (auto p : ctx->d_inv)
        if (p) hipFree(p);
    hipStreamDestroy(ctx->stream);
    for (int k = 0; k < ctx->n_dec_aux; k++) {
        hipStreamSynchronize(ctx->dec_aux[k]);
        hipStreamDestroy(ctx->dec_aux[k]);
        hipEventDestroy(ctx->ev_dec_aux[k]);
        if (ctx->ev_dec_wr[k]) hipEventDestroy(ctx->ev_dec_wr[k]);
    }
    if (ctx->ev_dec_split) hipEventDestroy(ctx->ev_dec_split);
    for (int k = 0; k < icx_ctx::UP_STREAMS; k++)
        if (ctx->up_stream[k]) {
            hipStreamSynchronize(ctx->up_stream[k]);
            hipStreamDestroy(ctx->up_stream[k]);
        }
    if (ctx->io_up) {
        hipStreamSynchronize(ctx->io_up);
        hipStreamSynchronize(ctx->io_down);
        hipStreamDestroy(ctx->io_up);
        hipStreamDestroy(ctx->io_down);
        for (int b = 0; b < 2; b++) {
            if (ctx->ev_up[b]) hipEventDestroy(ctx->ev_up[b]);
            if (ctx->ev_down[b]) hipEventDestroy(ctx->ev_down[b]);
        }
        if (ctx->ev_done) hipEventDestroy(ctx->ev_done);
    }
    delete ctx;
}

void icx_quality_tables(float quality, uint16_t lum[64], uint16_t chrom[64])
{
    const float lin = linear_quality(quality);
    if (lum) scaled_table(kK1, lin, lum);
    if (chrom) scaled_table(kK2, lin, chrom);
}

void icx_create_key(int32_t width, int32_t height, int64_t file_size, icx_similarity_key* key)
{
    if (!key) return;
    key->width_bucket = width / 100;
    key->height_bucket = height / 100;
    key->size_bucket = file_size / 102400;
}

int32_t icx_subsampling_factor(int32_t width, int32_t height)
{
    const int maxd = std::max(width, height);
    int s = 1;
    if (maxd > 4096) s = (int)std::floor((double)maxd / 4096);
    if (s > 1) {  // Integer.highestOneBit
        int hb = 1;
        while (hb <= s / 2) hb <<= 1;
        s = hb;
    }
    return s;
}

void icx_scaled_dims(int32_t width, int32_t height, double scale, int32_t* out_w, int32_t* out_h)
{
    const int nw = (int)(width * scale), nh = (int)(height * scale);
    if (out_w) *out_w = std::max(1, nw);
    if (out_h) *out_h = std::max(1, nh);
}

int32_t icx_jpeg_header_size(int32_t fmt) { return fmt == ICX_GRAY8 ? HDR_GRAY : HDR_COLOR; }

int32_t icx_default_palette(int32_t binary, uint32_t pal[256])
{
    if (!pal) return 0;
    return default_palette(binary != 0, pal);
}

void icx_inverse_colour_map(const uint32_t* pal, int32_t n, uint8_t cube[32768])
{
    if (!pal || !cube || n < 1 || n > 256) return;
    const std::vector<uint8_t> c = inverse_cube(pal, n);
    memcpy(cube, c.data(), c.size());
}

void icx_dither_tables(int8_t err[3][64])
{
    if (!err) return;
    int8_t d[3][64];
    dither_tables(d);
    memcpy(err, d, sizeof(d));
}

int32_t icx_jpeg_header_size_layout(int32_t fmt, int32_t layout)
{
    const bool grouped = layout == ICX_TABLES_GROUPED;
    return fmt == ICX_GRAY8 ? (grouped ? HDR_GRAY_GROUPED : HDR_GRAY) : (grouped ? HDR_COLOR_GROUPED : HDR_COLOR);
}

icx_status icx_set_table_layout(icx_ctx* ctx, int32_t layout)
{
    if (!ctx) return ICX_E_NULL;
    if (layout != ICX_TABLES_SEPARATE && layout != ICX_TABLES_GROUPED) return fail(ctx, ICX_E_INVALID, "table layout");
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->table_layout = layout;
    return ICX_OK;
}

int64_t icx_num_blocks(int32_t width, int32_t height, int32_t fmt)
{
    if (width <= 0 || height <= 0) return 0;
    ImgDesc d{};
    geometry(d, width, height, fmt);
    return d.nblocks;
}

icx_status icx_compress_jpg_to_stream(icx_ctx* ctx, const icx_image* img, float quality, uint8_t* out, size_t cap,
                                      size_t* out_len)
{
    if (!ctx || !img || !out || !out_len) return ICX_E_NULL;
    icx_fit_job j{};
    j.img = *img;
    j.quality = quality;
    j.out = out;
    j.cap = cap;
    j.target_max_size = INT64_MAX;
    icx_status s = run_batch(ctx, &j, 1, Mode::Encode);
    if (s) return s;
    *out_len = j.out_len;
    return j.status;
}

icx_status icx_find_best_quality(icx_ctx* ctx, const icx_image* img, int64_t target_max_size, float initial_quality,
                                 float* best_quality, float* trial_q, int64_t* trial_size, int32_t* ntrials)
{
    if (!ctx || !img || !best_quality) return ICX_E_NULL;
    icx_fit_job j{};
    j.img = *img;
    j.quality = initial_quality;
    j.target_max_size = target_max_size;
    ImgState st{};
    icx_status s = run_batch(ctx, &j, 1, Mode::Search, nullptr, &st);
    if (s) return s;
    if (j.status) return j.status;
    *best_quality = j.learned.quality;
    const int nt = std::min<int>(st.ntrials, MAX_TRIALS);
    for (int i = 0; i < nt; i++) {
        if (trial_q) trial_q[i] = st.trial_q[i];
        if (trial_size) trial_size[i] = st.trial_size[i];
    }
    if (ntrials) *ntrials = nt;
    return ICX_OK;
}

icx_status icx_compress_jpg_with_target_size(icx_ctx* ctx, icx_fit_job* job)
{
    if (!ctx || !job) return ICX_E_NULL;
    icx_status s = run_batch(ctx, job, 1, Mode::Fit);
    return s ? s : job->status;
}

icx_status icx_compress_jpg_batch(icx_ctx* ctx, icx_fit_job* jobs, int32_t n)
{
    if (!ctx || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    return run_batch(ctx, jobs, n, Mode::Fit);
}

icx_status icx_debug_fdct(icx_ctx* ctx, const icx_image* img, int16_t* coefs, size_t ncoefs)
{
    if (!ctx || !img || !coefs) return ICX_E_NULL;
    icx_status v = validate(img);
    if (v) return v;
    if ((int64_t)ncoefs < icx_num_blocks(img->width, img->height, img->fmt) * 64) return ICX_E_BUFFER;
    icx_fit_job j{};
    j.img = *img;
    icx_status s = run_batch(ctx, &j, 1, Mode::Fdct, coefs);
    return s ? s : j.status;
}

// Source pixels the bilinear taps of a w -> dw resize read along one axis
// (the algorithmic read bytes of k_resize: each touched pixel once).
static int64_t touched(int sw, int dw, int64_t x0l, int64_t dxl)
{
    int64_t n = 0;
    int last = -1;
    for (int dx = 0; dx < dw; dx++) {
        const int64_t xl = x0l + (int64_t)dx * dxl - ((int64_t)1 << 31);
        const int xw = (int)(xl >> 32);
        const int xa = xw < 0 ? 0 : xw, xb = xw < 0 ? 0 : std::min(xw + 1, sw - 1);
        for (int x : {xa, xb})
            if (x > last) {
                n++;
                last = x;
            }
    }
    return n;
}

// A palette raster's resize arguments: its colour map (padded to 256 entries
// with opaque black) copied into the workspace, and the inverse map of the
// destination type's default map (built and uploaded at first use).
static hipError_t palette_args(icx_ctx* c, const icx_image& img, ResizeArgs& a)
{
    if (!is_palette(img.fmt)) return hipSuccess;
    const int b = img.fmt == ICX_BINARY1;
    hipError_t e = hipSuccess;
    if (!c->d_inv[b]) {
        uint32_t pal[256];
        const int n = default_palette(b, pal);
        const std::vector<uint8_t> cube = inverse_cube(pal, n);
        c->inv_prims[b] = represents_primaries(pal, cube);
        if ((e = hipMalloc(&c->d_inv[b], cube.size())) != hipSuccess) return e;
        if ((e = hipMemcpy(c->d_inv[b], cube.data(), cube.size(), hipMemcpyHostToDevice)) != hipSuccess) return e;
    }
    uint32_t pal[256];
    for (int i = 0; i < 256; i++) pal[i] = i < img.palette_len ? img.palette[i] : 0xff000000u;
    uint32_t* dp = (uint32_t*)c->dev.take(sizeof(pal));
    if ((e = hipMemcpy(dp, pal, sizeof(pal), hipMemcpyHostToDevice)) != hipSuccess) return e;
    a.pal = dp;
    a.inv = c->d_inv[b];
    a.prims = c->inv_prims[b];
    return hipSuccess;
}

icx_status icx_resize_bilinear(icx_ctx* ctx, const icx_image* src, uint8_t* dst, int32_t dst_w, int32_t dst_h,
                               int32_t dst_stride)
{
    if (!ctx || !src || !dst) return ICX_E_NULL;
    icx_status v = validate(src);
    if (v) return v;
    const int nch = channels(src->fmt);
    if (dst_w <= 0 || dst_h <= 0 || dst_stride < dst_w * nch) return ICX_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    const bool din = is_device_ptr(src->px), dout = is_device_ptr(dst);
    size_t need = (1 << 20) + 2048;
    if (!din) need += (size_t)src->width * nch * src->height + 256;
    if (!dout) need += (size_t)dst_stride * dst_h + 256;
    hipError_t e = ctx->dev.reserve(need);
    if (e != hipSuccess) return hip_fail(ctx, e, "resize workspace");
    ctx->dev.used = 0;
    ctx->dev.overflow = false;
    const uint8_t* s = src->px;
    int sstride = src->stride;
    if (!din) {
        const size_t row = (size_t)src->width * nch;
        uint8_t* st = (uint8_t*)ctx->dev.take(row * src->height);
        e = hipMemcpy2DAsync(st, row, src->px, src->stride, row, src->height, hipMemcpyHostToDevice, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "resize upload");
        s = st;
        sstride = (int)row;
    }
    uint8_t* d = dout ? dst : (uint8_t*)ctx->dev.take((size_t)dst_stride * dst_h);
    {
        ResizeArgs a = resize_args(s, src->width, src->height, sstride, src->fmt, d, dst_w, dst_h, dst_stride);
        if ((e = palette_args(ctx, *src, a)) != hipSuccess) return hip_fail(ctx, e, "resize palette");
        if (ctx->prof)
            ctx->stats["resize.bytes"].units += (touched(src->width, dst_w, a.x0l, a.dxl) *
                                                     touched(src->height, dst_h, a.y0l, a.dyl) +
                                                 (int64_t)dst_w * dst_h) * nch;
        Timed tm(ctx, "resize", (int64_t)dst_w * dst_h, true);
        launch_resize_one(a, ctx->stream);
    }
    if (!dout) {
        e = hipMemcpyAsync(dst, d, (size_t)dst_stride * dst_h, hipMemcpyDeviceToHost, ctx->stream);
        if (e != hipSuccess) return hip_fail(ctx, e, "resize download");
    }
    e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(ctx, e, "resize");
    resolve_profile(ctx);
    return ICX_OK;
}

icx_status icx_resize_image(icx_ctx* ctx, const icx_image* src, double scale, uint8_t* dst, size_t cap,
                            int32_t* out_w, int32_t* out_h)
{
    if (!ctx || !src || !dst) return ICX_E_NULL;
    icx_status v = validate(src);
    if (v) return v;
    if (!(scale > 0.0)) return ICX_E_INVALID;
    int32_t dw, dh;
    icx_scaled_dims(src->width, src->height, scale, &dw, &dh);
    if (out_w) *out_w = dw;
    if (out_h) *out_h = dh;
    const size_t need = (size_t)dw * dh * channels(src->fmt);
    if (cap < need) return ICX_E_BUFFER;
    return icx_resize_bilinear(ctx, src, dst, dw, dh, dw * channels(src->fmt));
}

icx_status icx_png_fit(icx_ctx* ctx, const icx_image* src, int32_t min_width, int32_t min_height, uint8_t* dst,
                       size_t cap, int32_t* out_w, int32_t* out_h, int32_t* resized)
{
    if (!ctx || !src || !src->px || !dst || !resized) return ICX_E_NULL;
    icx_png_fit_job j{};
    j.src = *src;
    j.min_width = min_width;
    j.min_height = min_height;
    j.dst = dst;
    j.cap = cap;
    icx_status s = icx_png_fit_batch(ctx, &j, 1);
    if (s == ICX_OK) s = j.status;
    *resized = j.resized;
    if (out_w) *out_w = j.out_w;
    if (out_h) *out_h = j.out_h;
    return s;
}

icx_status icx_png_fit_batch(icx_ctx* ctx, icx_png_fit_job* jobs, int32_t n)
{
    if (!ctx || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    // ImageCompressionPng.java:45-66: the box test and scale per image
    std::vector<int> todo;
    for (int i = 0; i < n; i++) {
        icx_png_fit_job& j = jobs[i];
        j.resized = 0;
        j.out_w = j.out_h = 0;
        j.status = validate(&j.src);
        if (j.status) continue;
        if (j.src.width <= j.min_width && j.src.height <= j.min_height) {  // :49-53, the reference returns false
            j.out_w = j.src.width;
            j.out_h = j.src.height;
            continue;
        }
        if (!j.dst) {  // needed only for an image that is resized
            j.status = ICX_E_NULL;
            continue;
        }
        const double scale = std::min((double)j.min_width / j.src.width, (double)j.min_height / j.src.height);
        if (!(scale > 0.0)) {
            j.status = ICX_E_INVALID;
            continue;
        }
        icx_scaled_dims(j.src.width, j.src.height, scale, &j.out_w, &j.out_h);  // ImageTools.java:8-9
        if (j.cap < (size_t)j.out_w * j.out_h * channels(j.src.fmt)) {
            j.status = ICX_E_BUFFER;
            continue;
        }
        todo.push_back(i);
    }
    // by format (one kernel instantiation per launch), then in workspace-sized groups
    std::stable_sort(todo.begin(), todo.end(), [&](int a, int b) { return jobs[a].src.fmt < jobs[b].src.fmt; });
    size_t pos = 0;
    while (pos < todo.size()) {
        const int fmt = jobs[todo[pos]].src.fmt;
        std::vector<int> grp;
        size_t need = 1 << 20;
        while (pos < todo.size() && jobs[todo[pos]].src.fmt == fmt) {
            const icx_png_fit_job& j = jobs[todo[pos]];
            const size_t nch = channels(fmt);
            size_t per = 4096 + 2048;
            if (!is_device_ptr(j.src.px)) per += (size_t)j.src.width * j.src.height * nch + 256;
            if (!is_device_ptr(j.dst)) per += (size_t)j.out_w * j.out_h * nch + 256;
            if (!grp.empty() && need + per > ctx->budget) break;
            need += per;
            grp.push_back(todo[pos++]);
        }
        hipError_t e = ctx->dev.reserve(need + grp.size() * (sizeof(ResizeArgs) + 8) + 4096);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            for (int i : grp) jobs[i].status = ICX_E_NOMEM;
            continue;
        }
        ctx->dev.used = 0;
        ctx->dev.overflow = false;
        const int m = (int)grp.size();
        std::vector<ResizeArgs> args(m);
        std::vector<int64_t> prefix(m + 1, 0);
        std::vector<uint8_t*> dl(m, nullptr);  // device staging of host destinations
        int64_t dpx = 0, algo = 0, uniform = -1;
        for (int k = 0; k < m && e == hipSuccess; k++) {
            const icx_png_fit_job& j = jobs[grp[k]];
            const int nch = channels(fmt);
            const uint8_t* sp = j.src.px;
            int sstride = j.src.stride;
            if (!is_device_ptr(sp)) {
                const size_t row = (size_t)j.src.width * nch;
                uint8_t* st = (uint8_t*)ctx->dev.take(row * j.src.height);
                e = hipMemcpy2DAsync(st, row, sp, j.src.stride, row, j.src.height, hipMemcpyHostToDevice, ctx->stream);
                sp = st;
                sstride = (int)row;
            }
            uint8_t* dp = j.dst;
            if (!is_device_ptr(dp)) dp = dl[k] = (uint8_t*)ctx->dev.take((size_t)j.out_w * j.out_h * nch);
            args[k] = resize_args(sp, j.src.width, j.src.height, sstride, fmt, dp, j.out_w, j.out_h, j.out_w * nch);
            if (e == hipSuccess) e = palette_args(ctx, j.src, args[k]);
            const int64_t tiles = resize_tiles(j.out_w, j.out_h);
            prefix[k + 1] = prefix[k] + tiles;
            uniform = uniform < 0 || uniform == tiles ? tiles : 0;
            dpx += (int64_t)j.out_w * j.out_h;
            if (ctx->prof)
                algo += (touched(j.src.width, j.out_w, args[k].x0l, args[k].dxl) *
                             touched(j.src.height, j.out_h, args[k].y0l, args[k].dyl) +
                         (int64_t)j.out_w * j.out_h) * nch;
        }
        ResizeArgs* d_args = (ResizeArgs*)ctx->dev.take(sizeof(ResizeArgs) * m);
        int64_t* d_prefix = (int64_t*)ctx->dev.take(sizeof(int64_t) * (m + 1));
        if (e == hipSuccess) e = hipMemcpyAsync(d_args, args.data(), sizeof(ResizeArgs) * m, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_prefix, prefix.data(), sizeof(int64_t) * (m + 1), hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) {
            if (ctx->prof) ctx->stats["resize.bytes"].units += algo;
            Timed tm(ctx, "resize", dpx, true);
            launch_resize_batch(fmt, d_args, d_prefix, m, prefix[m], uniform > 0 ? uniform : 0, ctx->stream);
        }
        for (int k = 0; k < m && e == hipSuccess; k++) {
            if (!dl[k]) continue;
            const icx_png_fit_job& j = jobs[grp[k]];
            e = hipMemcpyAsync(j.dst, dl[k], (size_t)j.out_w * j.out_h * channels(fmt), hipMemcpyDeviceToHost,
                               ctx->stream);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e == hipSuccess) e = hipGetLastError();
        if (e != hipSuccess) {
            for (int i : grp) jobs[i].status = ICX_E_DEVICE;
            return hip_fail(ctx, e, "png fit batch");
        }
        for (int i : grp) jobs[i].resized = 1;
    }
    resolve_profile(ctx);
    return ICX_OK;
}

icx_status icx_profile_enable(icx_ctx* ctx, int32_t on)
{
    if (!ctx) return ICX_E_NULL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->prof = on != 0;
    return ICX_OK;
}

icx_status icx_profile_reset(icx_ctx* ctx)
{
    if (!ctx) return ICX_E_NULL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    ctx->stats.clear();
    return ICX_OK;
}

icx_status icx_profile_query(icx_ctx* ctx, const char* kernel, int64_t* launches, double* total_ms, int64_t* units)
{
    if (!ctx || !kernel) return ICX_E_NULL;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    auto f = ctx->stats.find(kernel);
    const KStat z;
    const KStat& s = f == ctx->stats.end() ? z : f->second;
    if (launches) *launches = s.launches;
    if (total_ms) *total_ms = s.ms;
    if (units) *units = s.units;
    return ICX_OK;
}

}  // extern "C"
