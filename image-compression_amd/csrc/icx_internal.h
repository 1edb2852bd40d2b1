// icx_internal.h — device-visible data structures of the MI355X JPEG path.
//
// HBM layout per image:
//   px          u8 BGR/RGB/grey rows (caller's buffer, or the resize buffer)
//   coefs       sparse jpeg_fdct_islow output (raw, x8): per scan block
//               (MCU order Y0 Y1 Y2 Y3 Cb Cr) a list of 32-bit entries
//               float_bits(c) | (chroma << 9) | (k << 3) in zig-zag order k
//               (|c| <= 8192 < 2^14 for 8-bit samples, so the float's low 10
//               mantissa bits are free; entry & ~0x3FF is c as a float,
//               entry & 0x3F8 the byte offset of the block's 8-B quantiser
//               entry in k_huff's [component][k] table) — entry 0 is the DC, then every
//               AC coefficient that can quantise to nonzero in ANY trial this
//               image may run (|c| >= the smallest threshold over the image's
//               reachable quality nodes, `cand_node`), padded (any bits) to a
//               multiple of 4.  The lists of one FDCT tile are packed back to
//               back inside the tile's region (room for 64 entries per block);
//               block b's list starts at entry 4 * coff[b] and holds ncoef[b]
//               entries.  Written once per visited scale by the FDCT, re-read
//               by every quality trial (quantisation happens there).
//   scratch[2]  per-chunk packed Huffman bitstreams (chunk = CHUNK_BLOCKS
//               scan blocks, MSB-first 32-bit words, chunk-local bit 0),
//               double-buffered: [best] holds the best fitting trial so the
//               final file is stuffed from it without a re-encode.
//   chunk_bits/off/ff [2]  per-chunk bit counts, exclusive bit offsets and
//               0xFF-byte counts of the owned bytes (bytes whose first bit
//               lies in the chunk), for byte stuffing.
//   chunk_ffa[2] per chunk, 8 counts: byte-long runs of 1-bits lying wholly
//               inside the chunk, binned by chunk-local start bit mod 8 —
//               the chunk's 0xFF count for each possible byte alignment,
//               resolved by k_scan once the chunk's global offset is known.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace icx {

// k_huff: one workgroup (256 threads, one per block) per chunk of 256 scan
// blocks.  (Round 4 measured one wave per 64-block chunk, four chunks per
// workgroup sharing the coding tables, no workgroup barrier after the table
// load: k_huff +2...5 %, step +7 % with the 4x chunk count in k_scan/k_stuff;
// profiles/NOTES.md §9.)
constexpr int CHUNK_BLOCKS = 256;  // scan blocks per Huffman chunk
constexpr int HUFF_THREADS = CHUNK_BLOCKS;
constexpr int MAX_BLOCK_BITS = 1664;     // >= 22 (DC) + 63 * 26 (AC) bits, multiple of 32
constexpr int BLOCK_WORDS = MAX_BLOCK_BITS / 32;               // 52
constexpr int CHUNK_WORDS = CHUNK_BLOCKS * BLOCK_WORDS;        // 13312 words = 52 KiB

constexpr int COEF_SLOTS = 64;           // int32 entries reserved per block in `coefs` (tile regions)
constexpr int FD_TILE_PX = 128;          // FDCT tile width in pixels (8 colour MCUs)
constexpr int MAX_TRIALS = 8;            // findBestQualityByBinarySearch loop bound (:167)
constexpr int HDR_COLOR = 623;           // SOI+APP0+2 DQT+SOF0+4 DHT+SOS
constexpr int HDR_GRAY = 328;            // SOI+APP0+DQT+SOF0+2 DHT+SOS
// ICX_TABLES_GROUPED: one DQT segment for every quantisation table, one DHT
// for every Huffman table (3 + 12 B less for colour, 4 B less for grey)
constexpr int HDR_COLOR_GROUPED = 607;
constexpr int HDR_GRAY_GROUPED = 324;
// offsets inside the header template that k_stuff patches: the chroma DQT
// payload and the SOF0 marker (the luma DQT payload starts at 25 in both)
constexpr int hdr_dqt1(bool grouped) { return grouped ? 90 : 94; }
constexpr int hdr_sof(bool colour, bool grouped) { return colour ? (grouped ? 154 : 158) : 89; }

// One trial quality: a node of the binary-search tree of
// findBestQualityByBinarySearch (ImageCompressionJpg.java:158-200), or a fixed
// quality (compressJpgToStream / tryCachedParams).  Everything float-dependent
// is evaluated on the host with Java's float32 semantics.
struct QNode {
    float mid;             // quality of this trial
    int32_t child_fit;     // next node when size <= target (lo = mid), -1 = stop
    int32_t child_nofit;   // next node when size >  target (hi = mid), -1 = stop
    int32_t pad;
    // Quantiser of zig-zag coefficient k, table c ([0]=lum [1]=chroma), for the
    // divisor d = q<<3 (jcdctmgr.c: |c| -> (|c| + d/2) / d, truncating):
    // per (component, k): x = thr = d - d/2 (the quotient is nonzero iff
    // |c| >= thr), y = fl(1/d), z = fl((d/2 + 0.5) * y): floor(fma(|c|, y, z))
    // is the quotient exactly for |c| < 2^15 (error << 0.5/d); w unused.
    // Interleaved so the trial kernel loads one 16-B entry per index.
    float4 qf[2][64];
    uint16_t qt[2][64];    // quantisation tables, natural order (DQT payload)
};

struct ImgDesc {
    const uint8_t* px;     // pixels for the current stage (original or resized)
    int32_t w, h, stride, fmt;
    int32_t ncomp, mcux, mcuy, ywb, yhb;
    int32_t nchunks, hdr_len, cand_node;  // cand_node: QNode whose thr[] filters the FDCT's lists
    // FDCT tiles per tile row (16 MCUs / 16 grey blocks each) and its
    // reciprocal for a multiply-high division (tiles_xm = ceil(2^32 / tiles_x),
    // exact for tile * tiles_x < 2^32; 0 when tiles_x == 1)
    uint32_t tiles_x, tiles_xm;
    int64_t nblocks;
    int64_t target;
    int32_t* coefs;        // candidate lists, COEF_SLOTS entries reserved per block (see above)
    uint32_t* coff;        // start of each block's list, in 4-entry (16-B) units
    uint8_t* ncoef;        // list length per block (1..64)
    uint32_t* scratch[2];
    uint32_t* chunk_bits[2];
    uint64_t* chunk_off[2];   // nchunks + 1 entries
    uint32_t* chunk_ff[2];
    uint32_t* chunk_ffa[2];   // nchunks * 8 entries
    uint64_t* chunk_ffoff;    // nchunks entries (final stuffing pass)
    uint32_t* ovf;            // per-block spill of Huffman words beyond the LDS slot
    uint8_t* out;
    uint64_t cap;
};

constexpr int ENT_SLOTS = 16;

struct ImgState {
    int32_t node;          // node of the pending trial, -1 = none
    int32_t best_node;     // node of the best fitting trial, -1 = none
    int32_t cur;           // scratch buffer the next trial writes
    int32_t best_buf;      // scratch buffer holding the best trial
    int32_t active;        // a trial is pending
    int32_t ntrials;
    int32_t force;         // single encode: accept regardless of size
    int32_t status;        // 0 ok, 4 = output buffer too small
    int64_t best_size;
    int64_t out_len;
    uint64_t total_bits[2];
    // candidate-list entries the last FDCT wrote (padded; algorithmic bytes),
    // spread over ENT_SLOTS counters so the FDCT waves' atomics rarely collide
    uint64_t list_entries[ENT_SLOTS];
    uint32_t ff_total[2];
    // bytes k_huff wrote for this state's trials: each trial's stream words
    // (at least total_bits / 8) and its per-chunk bit counts and 0xFF bins
    uint64_t huff_wbytes;
    float trial_q[MAX_TRIALS + 1];
    int64_t trial_size[MAX_TRIALS + 1];
};

// A launch plan: the images taking part (ids into desc/state arrays) and
// the exclusive prefix of work items (tiles or chunks) per image.
// Profiling: events a launch wrapper (icx_kernels.hip) hands to
// hipExtLaunchKernelGGL, which timestamps the dispatch itself - no marker
// packets between the kernels.  Set by Timed (icx_context.h) for one launch.
struct LaunchTiming {
    hipEvent_t a = nullptr, b = nullptr;
    bool used = false;
};
extern thread_local LaunchTiming g_launch_timing;

struct Plan {
    const int32_t* ids;
    const int64_t* prefix;  // m + 1 entries
    int32_t m;
    int32_t uniform;        // > 0: every slot holds this many items (2-D launches, no slot search)
    int32_t identity;       // ids[i] == i for every slot
    int32_t width = 0;      // decoder: > 0 = 2-D launch (x < width items, y = slot; items past a slot's count exit)
};

}  // namespace icx
