// icx_decode.h — data structures and the entropy-decoding state machine of
// the device JPEG decoder (row A11 of SURVEY.md §8a).
//
// Replaces the JDK JPEGImageReader decode reached from
// ImageCompression.decodeImageWithSubsampling (core/ImageCompression.java:
// 107-165); the arithmetic is IJG libjpeg 6b's baseline decompression, the
// same algorithm oracle/icx_oracle_decode.c restates on the CPU.
//
// Parallel Huffman decoding without restart markers uses self-synchronisation
// (a Huffman decoder started at an arbitrary bit soon falls onto the true
// symbol boundaries): the unstuffed entropy stream of an image is cut into
// subsequences of DEC_SUB_BITS bits, one per thread.  A decoder state is
// (bit position, block-in-MCU, zig-zag index) at a symbol boundary;
// walk(E[j], subsequence j) gives the state at which the decode leaves
// subsequence j.  The entry states E[] are the fixed point of
// E[j+1] = walk(E[j]) from the known E[0]; the sync kernel iterates it, the
// first launch over every subsequence and each later one over a worklist of
// the subsequences whose entry changed (so re-walks pack densely into waves);
// it settles in a few launches because wrong starts resynchronise quickly.
// Restart intervals need no special case: every RSTn marker is replaced by
// DEC_PAD bytes of 0xFF, and an all-ones look-ahead is never a valid JPEG code
// (T.81 C.2 forbids all-ones codes), so the decode of an interval ends with an
// invalid code whose only transition is a jump to the next interval start.
// A decoder started at a wrong state also meets invalid codes mid-interval
// (e.g. nine 1-bits where a luma DC code is due); there it resumes one bit
// later instead of ending, so wrong paths keep resynchronising rather than
// collapsing into the end state.  The true path of a valid stream never meets
// an invalid code more than 7 bits before its interval's end.
//
// Everything here is __host__ __device__ so tests/dec_emu.cpp can run the same
// state machine serially on the CPU.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <type_traits>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define ICX_HD __host__ __device__ __forceinline__
#else
#define ICX_HD inline
#endif

namespace icx {

constexpr int DEC_SUB_BITS = 1024;   // bits per subsequence (one thread)
// First-level look-up width.  9 bits since the symbol pairs (round 5): the
// write pass's first levels (32-bit entries) then take 8 KiB of LDS, so with
// its 32 KiB of block slots four workgroups still fit a CU; 0.8 % of q95
// symbols have longer codes (0.3-0.5 % at 10 bits), and pairs must fit 9
// bits.  Decode per 1000 / 200 4K q95 frames: 10 bits 80.4 / 18.9 ms, 9 bits
// 78.0 / 18.5 ms (profiles/r5/ab_r5d_dec_lut.txt).
#ifndef ICX_DEC_LUT_BITS
#define ICX_DEC_LUT_BITS 9
#endif
constexpr int DEC_LUT_BITS = ICX_DEC_LUT_BITS;  // Huffman fast-lookup width
// k_dec_write workgroup size.  The pass is LDS-limited (a 128-B block slot
// per lane + the first-level tables): 256 lanes = 40 KiB, four workgroups =
// 16 waves per CU.  576 lanes (80 KiB, meant as two workgroups = 18 waves)
// measured +28 % decode: one workgroup per CU (profiles/r4/ab_r4zb_dec_write.txt).
#ifndef ICX_DEC_WRITE_NT
#define ICX_DEC_WRITE_NT 256
#endif
constexpr int DEC_WRITE_NT = ICX_DEC_WRITE_NT;
constexpr int DEC_TILE = 4096;       // stuffed bytes per unstuff tile (256 threads x 16)
#ifndef ICX_DEC_UNSTUFF_TILES
#define ICX_DEC_UNSTUFF_TILES 4
#endif
#ifndef ICX_DEC_SCATTER_TILES
#define ICX_DEC_SCATTER_TILES 4  // with the compacted masks (ICX_SCATTER_COMPACT): 1 / 2 / 4 / 8 tiles 7.4 / 6.7 / 6.35 / 8.3 ms unstuffing per 1000 frames, per-lane masks 7.1 (ab_r5ak_dec_scatter_compact.txt, ab_r5al_dec_unstuff_tiles8.txt)
#endif
constexpr int DEC_UNSTUFF_TILES = ICX_DEC_UNSTUFF_TILES;  // consecutive tiles per k_unstuff_count workgroup
constexpr int DEC_SCATTER_TILES = ICX_DEC_SCATTER_TILES;  // ... per k_unstuff_scatter workgroup (4: +10 %, r4e)
constexpr int DEC_PAD = 8;           // 0xFF bytes standing in for each RSTn marker
constexpr int DEC_TAIL = 16;         // 0xFF bytes after the last interval
constexpr uint32_t DEC_END = 0xFFFFFFFFu;

// One Huffman table prepared for decoding (jdhuff.c jpeg_make_d_derived_tbl),
// two-level: lut[the next DEC_LUT_BITS bits] is (length << 8) | symbol for
// codes of at most DEC_LUT_BITS bits; for such a prefix of longer codes it is
// DEC_SUB | k and lut2[k][the following 16 - DEC_LUT_BITS bits] holds
// (length << 8) | symbol.  0 = no valid code.  Tables with more than DEC_NSUB
// long-code prefixes mark the rest DEC_SLOW and decode those codes with the
// canonical maxcode loop (DecSlow).  8 second-level tables: -0.4 / -0.35 ms
// per 1000 / 200 4K frames against 16 (the smaller LDS image of the tables;
// profiles/r5/ab_r5f_dec.txt).
#ifndef ICX_DEC_NSUB
#define ICX_DEC_NSUB 8
#endif
constexpr int DEC_NSUB = ICX_DEC_NSUB;  // second-level tables per Huffman table (a power of two)
constexpr uint32_t DEC_SUB = 0x2000u, DEC_SLOW = 0x4000u;
struct DecHuff {
    uint16_t lut[1 << DEC_LUT_BITS];
    uint16_t lut2[DEC_NSUB][1 << (16 - DEC_LUT_BITS)];
};
struct DecSlow {
    int32_t maxcode[17];   // largest code of length l, -1 if none
    int32_t valoff[17];    // index into vals of code c of length l: valoff[l] + c
    uint8_t vals[256];
};

// The same table for the walks themselves (k_dec_init, k_dec_sync, k_dec_write):
// each entry says what the symbol does instead of what it is - bits 0..4 the
// bits it consumes (code length + extra bits, at most 16 + 15), bits 5..11
// what it adds to the zig-zag index (DC 1; AC run + 1, ZRL 16, EOB and the
// other size-0 symbols 64, which ends the block), bits 12..15 the extra bits
// (the magnitude category: the value is the last of the consumed bits).  0 =
// no valid code here (also a DC size over 11, jdhuff.c's "bad DC").  A 10-bit
// prefix of longer codes consumes 0 bits: DEC_LEAN_LONG | k << 5 (second
// level lut2[k]) or DEC_LEAN_LONG | DEC_LEAN_SLOW (canonical maxcode loop).
// One step is then a look-up, a skip and an add; no symbol decoding.
//
// Symbol pairs (round 5).  A first-level entry of an AC table also says, in
// its high half, what the NEXT symbol does when that symbol's whole code lies
// inside the same look-ahead (first symbol's code + extra bits + the second's
// code <= DEC_LUT_BITS): bits 16..20 the bits it consumes, code + extra (0 =
// no pair), 21..24 its extra bits, 25..31 its zig-zag advance - the fields a
// step adds as they are (round 5: code length and extra bits were separate
// fields until the consumed total saved the state-only walks an add and a
// bit-field extract per step).  A walk applies both symbols in
// one step unless the first ends the block (z + advance >= 64: the next
// symbol is then the next block's DC).  Over 4K q95 content a 10-bit window
// pairs 40 % (smooth) / 32 % (noise) of the symbol steps away
// (scripts/dec_pair_stats.cpp).  Every walker (warm-up, sync, write pass, the
// CPU emulator) steps the same way, so the states they visit - subsequence
// exits, checkpoints, piece starts - are the same pair-step boundaries; two
// walks that resynchronise on different phases of a pair meet again at the
// next block end, where no pair reaches across.
constexpr uint32_t DEC_LEAN_LONG = 0x400u, DEC_LEAN_SLOW = 0x200u;
constexpr int DEC_PAIR_SHIFT = 16;
struct DecLean {
    uint32_t lut[1 << DEC_LUT_BITS];                     // (pair << 16) | entry
    uint16_t lut2[DEC_NSUB][1 << (16 - DEC_LUT_BITS)];  // entries of codes longer than 10 bits (no pairs)
};
ICX_HD uint16_t dec_lean_entry(int len, int sym, bool ac)
{
    if (!ac) return sym > 11 ? (uint16_t)0 : (uint16_t)((len + sym) | (1 << 5) | (sym << 12));
    const int sz = sym & 15, run = sym >> 4;
    const int zadd = sz ? run + 1 : (run == 15 ? 16 : 64);
    return (uint16_t)((len + sz) | (zadd << 5) | (sz << 12));
}

// Per-image tables.  Components share tables (Cb/Cr normally do): h[] holds
// the distinct ones, sel[2*c] / sel[2*c+1] index the DC / AC table of component c.
struct DecTab {
    DecHuff h[4];
    DecLean lean[4];  // h[] as state-transition entries (DecLean), for the state-only walks
    DecSlow slow[4];
    uint16_t qt[4][64];    // dequantisation tables, natural order, per component
    uint8_t sel[8];
    uint8_t ntab;
    uint8_t pad[7];
};

// Per-image descriptor (host-built, read-only on the device).
struct DecDesc {
    const uint8_t* scan;   // entropy-coded segment (stuffed), device
    int64_t scan_len;
    uint8_t* ent;          // unstuffed stream + pads, 4-byte aligned
    int64_t ent_cap;       // bytes allocated for ent
    uint32_t* tile_cnt;    // per unstuff tile: output bytes, then exclusive offsets
    uint32_t* tile_rst;    // per unstuff tile: RSTn markers, then exclusive offsets
    uint32_t* seg;         // interval start byte offsets in ent (nseg_max entries)
    uint64_t* est;         // entry state per subsequence (nsub_max + 1)
    uint64_t* ck;          // sync-walk checkpoints, DEC_CK_MAX per subsequence (dec_sync_walk)
    uint32_t* wl[2];       // subsequences to re-walk in the next sync launch (ping-pong)
    uint32_t* wl_cnt;      // entries appended to image i's worklist by sync launch r: wl_cnt[r * images + i]
    uint32_t* ncnt;        // blocks completed inside each subsequence
    uint32_t* boff;        // blocks completed before each subsequence
    int16_t* coefs;        // nblocks x 64, natural order, quantised; [0] = DC difference
    int32_t* dc;           // nblocks: DC differences (write pass), then DC values (k_dec_dc)
    uint8_t* plane[4];     // IDCT output planes (pitch pw[c])
    uint8_t* out;          // BGR24 / GRAY8 rows, stride ostride
    const DecTab* tab;
    int64_t nblocks;
    int32_t ntiles, nsub_max, nseg_max;
    int32_t w, h, ncomp, hs, vs, nby, nbmcu, mcux, mcuy, ri;
    int32_t pw[4], ph[4], cw[4], ch[4];
    int32_t fancy;         // chroma upsampled with the triangle filter (cw > 2)
    int32_t fuse420;       // s == 1, 4:2:0, fancy: luma IDCT fused into the colour pass (no luma plane)
    int32_t s, ow, oh, ostride;
    int32_t rgb;           // components are R, G, B (jdcolor.c null_convert), not YCbCr
    int32_t cmyk;          // 4 components: 1 CMYK, 2 YCCK (jdcolor.c ycck_cmyk_convert first)
    int32_t raw4;          // 4 components out as libjpeg's CMYK samples (debug), else BGR (k_dec_color)
    int32_t wmcu;          // blocks per MCU as the entropy walk sees them (dec_walk_mcu)
};

// Blocks per MCU for the entropy walks: a walk's block-in-MCU index only
// selects Huffman tables, so when every component of the scan uses the same
// DC and the same AC table (RGB files, for one) all indices are equivalent
// and the walks keep it at 0.  Otherwise two walks that differ only in it
// would never compare equal - the relaxation would carry that phantom
// difference through every subsequence (one launch each).  Block counts,
// ownership and the DC predictors use absolute block indices and are
// unaffected.
ICX_HD int dec_walk_mcu(int ncomp, int nbmcu, const int* td, const int* ta)
{
    if (ncomp != 3 && ncomp != 4) return nbmcu;
    for (int c = 1; c < ncomp; c++)
        if (td[c] != td[0] || ta[c] != ta[0]) return nbmcu;
    return 1;
}

// the IDCT kernels load a dequantisation row as one 16-byte load
static_assert(offsetof(DecTab, qt) % 16 == 0 && sizeof(DecTab) % 16 == 0, "DecTab.qt rows 16-byte aligned");

// k_dec_idct work items per image: tiles of 32 blocks (nblk_tiles),
// Bytes past each IDCT plane: k_dec_idct stores a dummy block's rows there
// (jdcoefct.c transforms no dummy block) so that every lane stores on every
// path.
constexpr int DEC_PLANE_SPARE = 64;
// DEC_IDCT_TILES consecutive tiles per workgroup.
#ifndef ICX_DEC_IDCT_TILES
#define ICX_DEC_IDCT_TILES 2  // with ICX_DEC_IDCT_PF: 1 / 2 / 4 tiles 3.86 / 3.40 / 3.62 ms per 1000 frames (ab_r5at_dec_idct_pipe.txt)
#endif
constexpr int DEC_IDCT_TILES = ICX_DEC_IDCT_TILES;  // 4: +20 % (r4e) - one tile per workgroup at 8 per CU overlaps
ICX_HD long long dec_idct_items(long long nblk_tiles)
{
    return (nblk_tiles + DEC_IDCT_TILES - 1) / DEC_IDCT_TILES;
}

// k_dec_luma_color_420 work items per image: tiles of one MCU row x 8 MCUs,
// DEC_LC_TILES consecutive tiles per workgroup.
#ifndef ICX_DEC_LC_TILES
#define ICX_DEC_LC_TILES 4
#endif
constexpr int DEC_LC_TILES = ICX_DEC_LC_TILES;
ICX_HD long long dec_lc_items(int mcux, int mcuy)
{
    return ((long long)mcuy * ((mcux + 7) / 8) + DEC_LC_TILES - 1) / DEC_LC_TILES;
}

// One k_stage copy: len bytes from src (any alignment, device memory) to dst
// (16-byte aligned), then zeros up to dst_len (a multiple of 16).  src may
// equal dst (in-place padding of an uploaded scan's last partial 16 bytes).
struct StageJob {
    const uint8_t* src;
    uint8_t* dst;
    int64_t len, dst_len;
};
constexpr int STAGE_TILE = 4096;  // bytes per k_stage workgroup

// Device-written per-image results.
struct DecState {
    int64_t end;           // stuffed offset of the terminating marker (or scan_len)
    uint32_t ent_len;      // unstuffed bytes incl. pads
    uint32_t nseg;         // intervals found (RSTn markers + 1)
    uint32_t nsub;         // subsequences in use
    uint32_t total_blocks; // blocks the entropy decode produced
    int32_t status;        // 0 ok, 6 corrupt
    int32_t pad;
};

ICX_HD uint64_t dec_pack(uint32_t pos, int b, int z) { return ((uint64_t)pos << 16) | ((uint64_t)b << 8) | (uint64_t)z; }
ICX_HD uint32_t dec_pos(uint64_t st) { return (uint32_t)(st >> 16); }

ICX_HD uint32_t dec_be32(uint32_t v)
{
#if defined(__HIP_DEVICE_COMPILE__) || defined(__GNUC__)
    return __builtin_bswap32(v);
#else
    return (v >> 24) | ((v >> 8) & 0xFF00u) | ((v << 8) & 0xFF0000u) | (v << 24);
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
#define ICX_GLOBAL __attribute__((address_space(1)))
#else
#define ICX_GLOBAL
#endif

// MSB-first bit reader over the unstuffed stream (big-endian 32-bit words).
// The next word q0 sits in a register; the words after it in a window of
// DEC_WIN words ("rows") read from the stream at once.  On the device the
// window is reloaded only at wave-uniform points (top_up() when low(), driven
// by the caller's loop) followed at once by an explicit vmcnt(0):
// vector-memory counters are in-order and count stores too, so a load
// consumed one symbol later would also wait for every block store issued in
// between.  A step consumes at most one window word and the device loops top
// up every lane once any holds <= 1 (<= 2 when they check every second step),
// so a device refill never finds the window empty; host loops (no top-ups)
// reload inside refill().  The stream buffer extends 64 + 4 DEC_WIN bytes past
// its padded end, so a window never reads outside it.
//
// Where the window lives (LDS_WIN): in registers a refill shifts the whole
// window by one word under the lane's "need" (one select per word, every
// step - the walks are instruction-issue bound); in LDS (rows [row][lane] of
// the wave, dec_win_lane) a refill advances a row pointer and reads the next
// q0 unconditionally (the LDS read returns before the next step's table
// look-up, which waits on LDS anyway).  The state-only walks keep it in LDS
// (9 KiB more per workgroup: 6 workgroups per CU instead of 8, still a gain;
// 6 / 12 words there: slower / +-0, ab_r5ai_dec_lds_win_size.txt); the write
// pass in registers (its workgroups fill LDS already).
#ifndef ICX_DEC_WIN
#define ICX_DEC_WIN 8
#endif
constexpr int DEC_WIN = ICX_DEC_WIN;
// The write pass's window (DecLeanWriter): each top-up waits for the
// coefficient stores the wave issued before it, so a longer window there
// means fewer such waits (the state-only walks issue no stores).
#ifndef ICX_DEC_WIN_WRITE
#define ICX_DEC_WIN_WRITE 9  // k_dec_write checks for top-ups every second step (ICX_DEC_WRITE_UNROLL2)
#endif
constexpr int DEC_WIN_WRITE = ICX_DEC_WIN_WRITE;
constexpr int DEC_WIN_MAX = DEC_WIN > DEC_WIN_WRITE ? DEC_WIN : DEC_WIN_WRITE;
// state-only walks (k_dec_init, k_dec_sync) / the write pass: window in LDS
#ifndef ICX_DEC_LDS_WIN
#define ICX_DEC_LDS_WIN 1  // -1.2 ms at 1000 frames (sync0 12.9 -> 12.1), +-0 at 200 (ab_r5ah_dec_lds_win.txt)
#endif
#ifndef ICX_DEC_LDS_WIN_WRITE
#define ICX_DEC_LDS_WIN_WRITE 0  // +4.6 ms: 10 KiB more LDS per workgroup leaves 3 workgroups per CU, not 4 (ab_r5ah)
#endif
// Workgroup size of the state-only walks (k_dec_init, k_dec_sync): their
// LDS is the image's tables (16 KiB, once per workgroup) plus the lanes'
// windows, so larger workgroups share the tables among more waves.
#ifndef ICX_DEC_SYNC_NT
#define ICX_DEC_SYNC_NT 256  // 512 (8 waves per SIMD): first sync walk 12.1 -> 12.85 ms per 1000 frames, slower at 64 frames (ab_r5ba_dec_sync_nt512.txt)
#endif
constexpr int DEC_SYNC_NT = ICX_DEC_SYNC_NT;
constexpr int DEC_WIN_NT = DEC_SYNC_NT;  // workgroup size of the kernels whose windows are in LDS

#if defined(__HIP_DEVICE_COMPILE__)
#define ICX_LDS __attribute__((address_space(3)))
// The lane's row 0 of the LDS window: rows of one wave are 64 words apart
// (a row read by the wave's lanes is bank-conflict free whatever row each
// lane is at), one spare row past the window (a refill reads the row after
// the last word before the caller tops up).
template <int WIN>
__device__ __forceinline__ ICX_LDS uint32_t* dec_win_lane()
{
    __shared__ uint32_t win[(WIN + 1) * DEC_WIN_NT];
    const int t = (int)threadIdx.x;
    return (ICX_LDS uint32_t*)(win + (t >> 6) * (WIN + 1) * 64 + (t & 63));
}
#endif

template <int WIN, bool LDS_WIN = false>
struct DecReaderT {
    static constexpr int DEC_WIN = WIN;  // (shadows the global inside the reader)
    static constexpr bool LDS = LDS_WIN;
    const ICX_GLOBAL uint32_t* w;
    uint64_t buf;
    int avail;
    uint32_t wi;    // stream word index of row 0 of the window
    uint32_t q0;    // the next word (row used())
    struct Regs {
        int nq;  // words left, q0 included (q[0] = q0)
        uint32_t q[WIN];
    };
#if defined(__HIP_DEVICE_COMPILE__)
    struct Lds {
        ICX_LDS uint32_t* lw;  // row 0
        ICX_LDS uint32_t* rp;  // q0's row
        ICX_HD int row() const { return (int)(rp - lw) >> 6; }
        ICX_HD void bind() { rp = lw = dec_win_lane<WIN>(); }
        ICX_HD void put(int j, uint32_t v) { lw[j * 64] = v; }
        ICX_HD uint32_t next(bool need)
        {
            rp += need ? 64 : 0;
            return *rp;
        }
    };
#else
    struct Lds {  // the host's stand-in (tests/dec_emu.cpp runs the same row logic)
        uint32_t rows[WIN + 1];
        int r;
        ICX_HD int row() const { return r; }
        ICX_HD void bind() { r = 0; }
        ICX_HD void put(int j, uint32_t v) { rows[j] = v; }
        ICX_HD uint32_t next(bool need)
        {
            r += need ? 1 : 0;
            return rows[r];
        }
    };
#endif
    typename std::conditional<LDS_WIN, Lds, Regs>::type m;

    ICX_HD int used() const
    {
        if constexpr (LDS) return m.row();
        else return WIN - m.nq;
    }
    ICX_HD int left() const { return WIN - used(); }
    ICX_HD void fetch(uint32_t at)
    {
        wi = at;
        const ICX_GLOBAL uint32_t* const wa = w + at;  // one address, the words at immediate offsets
        uint32_t t[WIN];
#pragma unroll
        for (int j = 0; j < WIN; j++) t[j] = wa[j];
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing later waits on the window
#endif
        if constexpr (LDS) {
            m.bind();
#pragma unroll
            for (int j = 0; j < WIN; j++) m.put(j, t[j]);  // row 0 too: a refill without need reads q0's row again
        } else {
#pragma unroll
            for (int j = 0; j < WIN; j++) m.q[j] = t[j];
            m.nq = WIN;
        }
        q0 = t[0];
    }
    // past q0 by `need` words (0 or 1): the next q0
    ICX_HD void advance(bool need)
    {
        if constexpr (LDS) {
            q0 = m.next(need);  // unconditional read: the same word again without need
        } else {
#pragma unroll
            for (int j = 0; j + 1 < WIN; j++) m.q[j] = need ? m.q[j + 1] : m.q[j];
            m.nq -= need ? 1 : 0;
            q0 = m.q[0];
        }
    }
    ICX_HD uint32_t pop()  // next window word, byte-swapped
    {
        const uint32_t v = q0;
        advance(true);
        return dec_be32(v);
    }
    ICX_HD void init(const uint32_t* words, uint32_t pos)
    {
        w = (const ICX_GLOBAL uint32_t*)words;
        fetch(pos >> 5);
        const uint64_t hi = pop();
        buf = ((hi << 32) | pop()) << (pos & 31);
        avail = 64 - (int)(pos & 31);
    }
    // a lane with no walk: reads no stream memory, never asks for a top-up
    ICX_HD void park()
    {
        buf = 0;
        avail = 64;
        wi = 0;
        q0 = 0;
        if constexpr (LDS) {
            m.bind();
        } else {
            m.nq = WIN;
            for (int j = 0; j < WIN; j++) m.q[j] = 0;
        }
    }
    ICX_HD bool low() const { return left() <= 1; }
#ifndef ICX_DEC_TOPUP_HALF
#define ICX_DEC_TOPUP_HALF 0
#endif
    ICX_HD bool wants() const { return !ICX_DEC_TOPUP_HALF || left() <= DEC_WIN / 2; }  // joins a top-up
    ICX_HD void top_up() { fetch(wi + (uint32_t)used()); }
    ICX_HD void refill()  // select-based: the common case takes no branch
    {
#if !defined(__HIP_DEVICE_COMPILE__)
        // host loops have no top-up points: top up where a device lane may be
        // (any left() <= 2), so refills right after a top-up run here too
        if (left() <= 2) top_up();
#endif
        const bool need = avail < 32;
        const uint32_t v = dec_be32(q0);
        buf |= need ? (uint64_t)v << (32 - avail) : 0ull;
        avail += need ? 32 : 0;
        advance(need);
    }
    ICX_HD uint32_t peek16() const { return (uint32_t)(buf >> 48); }
    ICX_HD void skip(int n)
    {
        buf <<= n;
        avail -= n;
    }
    ICX_HD int get(int n)  // 0 <= n <= 16
    {
        const int v = n ? (int)(buf >> (64 - n)) : 0;
        buf <<= n;
        avail -= n;
        return v;
    }
};
using DecReader = DecReaderT<DEC_WIN, ICX_DEC_LDS_WIN != 0>;

// The state-only walks' bit reader (ICX_DEC_FUNNEL): the next 32 stream bits
// are one funnel shift of two byte-swapped words, alignbit(w0, w1, s), with s
// in [0, 31] (s = 0: w1 itself), so a step costs a subtract, a mask, a compare
// and two word selects where DecReaderT's 64-bit buffer took a 64-bit shift,
// an OR-in under selects and its fill count.  Steps consume at most 31 bits
// (a code and its extra bits, or a symbol pair), so one word moves in per
// step at most; the next word (q0) comes from the window rows as in
// DecReaderT (LDS on the device, rows byte-swapped when the window is
// fetched), read unconditionally ahead of its use.  First sync walk per 1000
// frames 12.15 -> 11.48 ms, e2e decode 68.3 -> 67.45 ms
// (profiles/r6/ab/ab_r6_funnel_reader.txt).
#ifndef ICX_DEC_FUNNEL
#define ICX_DEC_FUNNEL 1
#endif
#ifndef ICX_DEC_FUNNEL_WRITE
#define ICX_DEC_FUNNEL_WRITE 1  // the write pass's walk too (register window): write pass 28.12 -> 27.66 ms per 1000 frames (ab_r6_funnel_write.txt)
#endif
// A window in registers (the write pass: its workgroups fill LDS already)
// shifts by one word under the lane's need, one select per word.
template <int WIN>
struct DecRegRows {
    uint32_t q[WIN + 1];  // [WIN]: the spare row (a refill may read past the last word before a top-up)
    int r;
    ICX_HD int row() const { return r; }
    ICX_HD void bind() { r = 0; }
    ICX_HD void put(int j, uint32_t v) { q[j] = v; }
    ICX_HD uint32_t next(bool need)
    {
#pragma unroll
        for (int j = 0; j < WIN; j++) q[j] = need ? q[j + 1] : q[j];
        r += need ? 1 : 0;
        return q[0];
    }
};
template <int WIN, bool LDS_WIN = true>
struct DecFunnelReader {
    using Base = DecReaderT<WIN, true>;
    static constexpr int DEC_WIN = WIN;
    const ICX_GLOBAL uint32_t* w;
    uint32_t w0, w1, q0;
    int s;
    uint32_t wi;  // stream word index of row 0 of the window
    typename std::conditional<LDS_WIN, typename Base::Lds, DecRegRows<WIN>>::type m;

    ICX_HD int used() const { return m.row(); }
    ICX_HD int left() const { return WIN - used(); }
    ICX_HD bool low() const { return left() <= 1; }
    ICX_HD bool wants() const { return true; }
    ICX_HD void fetch(uint32_t at)
    {
        wi = at;
        const ICX_GLOBAL uint32_t* const wa = w + at;
        uint32_t t[WIN];
#pragma unroll
        for (int j = 0; j < WIN; j++) t[j] = wa[j];
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
        m.bind();
#pragma unroll
        for (int j = 0; j < WIN; j++) m.put(j, dec_be32(t[j]));
        if constexpr (!LDS_WIN) m.put(WIN, 0u);
        q0 = dec_be32(t[0]);
    }
    ICX_HD void advance(bool need) { q0 = m.next(need); }
    ICX_HD void top_up() { fetch(wi + (uint32_t)used()); }
    ICX_HD void init(const uint32_t* words, uint32_t pos)
    {
        w = (const ICX_GLOBAL uint32_t*)words;
        fetch(pos >> 5);
        const uint32_t off = pos & 31;
        const uint32_t a = q0;
        advance(true);
        if (off) {
            w0 = a;
            w1 = q0;
            advance(true);
            s = 32 - (int)off;
        } else {
            w0 = 0;
            w1 = a;
            s = 0;
        }
    }
    ICX_HD void park()
    {
        w0 = w1 = q0 = 0;
        s = 0;
        wi = 0;
        m.bind();
        if constexpr (!LDS_WIN)
            for (int j = 0; j <= WIN; j++) m.put(j, 0u);
    }
    ICX_HD uint32_t peek32() const
    {
#if defined(__HIP_DEVICE_COMPILE__)
        return __builtin_amdgcn_alignbit(w0, w1, (uint32_t)s);
#else
        return s ? (w0 << (32 - s)) | (w1 >> s) : w1;
#endif
    }
    ICX_HD uint32_t peek16() const { return peek32() >> 16; }
    ICX_HD void refill()
    {
#if !defined(__HIP_DEVICE_COMPILE__)
        if (left() <= 2) top_up();  // host loops have no top-up points (as DecReaderT)
#endif
    }
    ICX_HD void skip(int c)  // 0 <= c <= 31
    {
        const int s2 = s - c;
        const bool need = s2 < 0;
        s = s2 & 31;
        w0 = need ? w1 : w0;
        w1 = need ? q0 : w1;
        advance(need);
    }
};
using DecLeanReader = typename std::conditional<ICX_DEC_FUNNEL && ICX_DEC_LDS_WIN, DecFunnelReader<DEC_WIN>, DecReader>::type;

#ifndef ICX_DEC_WALK_UNROLL2
#define ICX_DEC_WALK_UNROLL2 1  // state-only walks: two steps per top-up check (-2.6 %, profiles/r4/ab_r4ze_dec_walk_unroll.txt)
#endif
// (an unpredicated loop while every lane of a wave walks, ahead of this one:
// +30 % sync0, profiles/r5/ab_r5ag_walk_all.txt)
#ifndef ICX_DEC_PEND32
#define ICX_DEC_PEND32 1  // write walk: pending block as a 32-bit count from the piece's first block (-0.2 % / -1 % at 200 frames, ab_r4zc_dec_pend32.txt)
#endif
#ifndef ICX_DEC_EXT_BF
#define ICX_DEC_EXT_BF 1  // write walk: branch-free value extension (-0.9 %, profiles/r4/ab_r4zb_dec_write.txt)
#endif
// HUFF_EXTEND (jdhuff.c)
ICX_HD int dec_extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// Decode one symbol: (length << 8) | symbol, 0 if no valid code.  e = the
// first-level entry of pk (dec_symbol looks it up itself).
template <class HuffPtr>
ICX_HD uint32_t dec_symbol_from(HuffPtr t, const ICX_GLOBAL DecSlow* slow, uint32_t pk, uint32_t e)
{
    if (e & DEC_SUB) e = t->lut2[e & (DEC_NSUB - 1)][pk & ((1u << (16 - DEC_LUT_BITS)) - 1)];
    if (e & DEC_SLOW) {
        e = 0;
        for (int l = DEC_LUT_BITS + 1; l <= 16; l++) {
            const int code = (int)(pk >> (16 - l));
            if (code <= slow->maxcode[l]) {
                e = ((uint32_t)l << 8) | slow->vals[(slow->valoff[l] + code) & 255];
                break;
            }
        }
    }
    return e;
}

template <class HuffPtr>
ICX_HD uint32_t dec_symbol(HuffPtr t, const ICX_GLOBAL DecSlow* slow, uint32_t pk)
{
    return dec_symbol_from(t, slow, pk, t->lut[pk >> (16 - DEC_LUT_BITS)]);
}

// Huffman tables with the first level in one place (LDS) and the whole table
// (second level, slow path) in global memory: k_dec_write keeps only the
// 10-bit first levels in LDS to leave room for its block slots.
struct SplitHuff {
    const uint16_t (*lut)[1 << DEC_LUT_BITS];
    const ICX_GLOBAL DecHuff* full;
};

template <class HuffPtr>
ICX_HD uint32_t dec_lookup(HuffPtr H, int ti, const ICX_GLOBAL DecSlow* slow, uint32_t pk)
{
    return dec_symbol(&H[ti], &slow[ti], pk);
}

ICX_HD uint32_t dec_lookup(const SplitHuff& H, int ti, const ICX_GLOBAL DecSlow* slow, uint32_t pk)
{
    const uint32_t e = H.lut[ti][pk >> (16 - DEC_LUT_BITS)];
    return (e & (DEC_SUB | DEC_SLOW)) ? dec_symbol_from(&H.full[ti], &slow[ti], pk, e) : e;
}

// zig-zag index -> natural index with jpeg_natural_order's tail (k > 63 -> 63)
ICX_HD int dec_nat(int z)
{
    constexpr uint8_t N[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                               12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                               35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
    return N[z > 63 ? 63 : z];
}

// First interval start strictly after byte `byte` (DEC_END if none); *k = its index.
ICX_HD uint32_t dec_next_seg(const ICX_GLOBAL uint32_t* seg, uint32_t nseg, uint32_t byte, uint32_t* k)
{
    uint32_t lo = 0, hi = nseg;  // find first k with seg[k] > byte
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg[mid] > byte) hi = mid; else lo = mid + 1;
    }
    *k = lo;
    return lo < nseg ? seg[lo] : DEC_END;
}

// natural index -> zig-zag index (inverse of dec_nat on 0..63)
ICX_HD int dec_zz(int n)
{
    constexpr uint8_t Z[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                               3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                               10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                               21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
    return Z[n];
}

// Decode from state st until the first symbol boundary at or beyond `stop`
// (jdhuff.c decode_mcu, symbol by symbol).  Returns the exit state; nblk =
// blocks completed on the way.
//
// OWNED (the write pass): a block belongs to the subsequence in which its DC
// symbol starts, so every block is written whole by exactly one thread.  The
// walk skips the stores of a block it enters mid-way (its owner is the
// previous subsequence), and after `stop` it keeps decoding until the block in
// progress is complete.  An owned block's DC difference goes to sink.put(0, v),
// its AC coefficients to sink.put(zig-zag index, v) (indices past 63 clamp to
// 63, as jpeg_natural_order's tail), the finished block to sink.flush_if.
// Table index of (component, DC or AC) from the packed selector (dec_selector).
ICX_HD int dec_sel(uint32_t selp, int comp, int ac) { return (int)((selp >> (4 * (2 * comp + ac))) & 3); }
#ifndef ICX_DEC_BSEL
#define ICX_DEC_BSEL 1  // decode -0.4 % (profiles/r4/ab_r4x_dec_bsel.txt)
#endif
// The same per block of the walk's MCU: 4 bits per block-in-MCU bb (DC table
// index, then AC table index), so the lean walks pick the next table with one
// shift instead of the component arithmetic (nbmcu <= 10: 40 bits).
ICX_HD uint64_t dec_block_sel(uint32_t selp, int nby, int nbmcu)
{
    uint64_t r = 0;
    for (int bb = 0; bb < nbmcu && bb < 16; bb++) {
        const int comp = bb < nby ? 0 : bb - nby + 1;
        r |= (uint64_t)dec_sel(selp, comp, 0) << (4 * bb) | (uint64_t)dec_sel(selp, comp, 1) << (4 * bb + 2);
    }
    return r;
}
ICX_HD int dec_block_table(uint64_t bsel, int bb, int zz) { return (int)((bsel >> (4 * bb + (zz != 0 ? 2 : 0))) & 3); }
// The map in 32 bits (ICX_DEC_BSEL32): a walk's MCU has at most 8 blocks (the
// walk state packs the block-in-MCU index in 3 bits; the layouts parse_jpeg
// accepts have <= 6), so a table index is one bit-field extract, and after a
// step the next symbol's table is the next block's DC table at a block end,
// else block b's AC table - no compare of z (2 VALU less per step).
#ifndef ICX_DEC_BSEL32
#define ICX_DEC_BSEL32 1
#endif
ICX_HD uint32_t dec_bsel_bits(uint32_t bsel, uint32_t off)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ubfe(bsel, off, 2u);
#else
    return (bsel >> off) & 3u;
#endif
}
// The map is the same for every lane of a workgroup (one image): kept in
// scalar registers on the device.
ICX_HD uint64_t dec_uniform(uint64_t v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
#else
    return v;
#endif
}

// Sink of an owned walk: put(zig-zag index, value) per symbol (index 0 = the
// DC difference), flush_if(block complete and owned, index).  Every symbol
// stores exactly one value at an index below 64: a ZRL or EOB stores 0 at the
// current index (still zero in the block being assembled), and the symbols of
// the partial block a walk starts in (owned by the previous subsequence) store
// at index 0, which the walk's first owned block overwrites with its DC.
struct NoSink {
    ICX_HD void put(int, int) {}
    ICX_HD void put2(int, int) {}
    ICX_HD void flush_if(bool, int64_t) {}
};
// DecLeanWriter's puts (ICX_DEC_PUT2): put2(2 * index, value) - the byte
// offset of an int16 slot entry, so the device sink's address is one XOR with
// its (128-B aligned) slot base and swizzle; `own` is kept doubled too.
#ifndef ICX_DEC_PUT2
#define ICX_DEC_PUT2 1
#endif

// The walk as a state object, one symbol per step() (the device write pass
// drives it from a wave-uniform loop so finished blocks can be flushed by the
// whole wave between steps).
template <bool OWNED, class HuffPtr>
struct DecWalker {
    HuffPtr H;
    const ICX_GLOBAL DecSlow* slow;
    uint32_t selp;
    const uint32_t* words;
    const ICX_GLOBAL uint32_t* seg;
    uint32_t nseg, ent_bits;
    int nby, nbmcu;    // descriptor fields the walk uses, held in registers
    int ri, nbm;       // restart interval (MCUs) and blocks per MCU: the interval-end check
    int64_t nblocks;
    uint32_t pos, n;
    int b, z, comp;
    bool own;
    bool bad;  // met an invalid code mid-interval (corrupt data if this is the true path)
    int64_t blk_base;
    DecReader R;

    ICX_HD void start(uint64_t st)
    {
        pos = dec_pos(st);
        b = (int)((st >> 8) & 7);
        z = (int)(st & 63);
        n = 0;
        own = z == 0;
        bad = false;
        comp = b < nby ? 0 : b - nby + 1;
        R.init(words, pos);
    }
    ICX_HD bool running(uint32_t stop) const { return pos < stop || (OWNED && z != 0); }
    ICX_HD uint64_t state() const { return dec_pack(pos, b, z); }

    // Decode one symbol (or take one invalid-code transition).  Straight-line
    // apart from the rare paths (second-level / slow code tables, invalid
    // code): DC and AC symbols, runs, ZRL / EOB and the block end are all
    // selects, and every symbol makes exactly one sink.put (index 64 = nothing
    // to store), so a wave pays no branch bookkeeping on the common path.
    template <class Sink>
    ICX_HD void step(Sink& sink)
    {
        R.refill();
        const bool ac = z != 0;
        const int ti = dec_sel(selp, comp, ac ? 1 : 0);
        const uint32_t e = dec_lookup(H, ti, slow, R.peek16());
        const int len = (int)(e >> 8), sym = (int)(e & 255);
        if (len == 0 || (!ac && sym > 11)) {  // no valid code here
            invalid();
            return;
        }
        const int sz = ac ? (sym & 15) : sym;   // extra bits
        const int run = ac ? (sym >> 4) : 0;
        R.skip(len);
        const int v = R.get(sz);
        pos += (uint32_t)(len + sz);
        const int x = sz ? dec_extend(v, sz) : 0;
        const int zc = z + run;                 // zig-zag index of an AC coefficient
        if (OWNED) sink.put(!own ? 0 : !ac ? 0 : sz ? (zc > 63 ? 63 : zc) : z, x);
        z = !ac ? 1 : sz ? zc + 1 : (run == 15 ? z + 16 : 64);
        const bool end = z >= 64;
        if (OWNED) {
            const int64_t bi = blk_base + n;
            sink.flush_if(end && own && bi < nblocks, bi);
        }
        own = own || end;
        n += end ? 1u : 0u;
        const int bn = b + 1 == nbmcu ? 0 : b + 1;
        b = end ? bn : b;
        z = end ? 0 : z;
        comp = b < nby ? 0 : b - nby + 1;
    }

    // An invalid code: on a wrong-start path resume one bit later (flagged),
    // in an interval's padding move to the next interval or the end.
    ICX_HD void invalid()
    {
        uint32_t k;
        const uint32_t nx = dec_next_seg(seg, nseg, pos >> 3, &k);
        const uint32_t bound = nx == DEC_END ? ent_bits : (nx - DEC_PAD) * 8;  // end of interval data
        const bool partial = z != 0;  // a block in progress: extra data in the interval (below)
        b = 0;
        z = 0;
        comp = 0;
        own = true;
        if (pos + 8 < bound) {  // mid-interval: only a wrong-start path gets here; resume a bit later
            bad = true;
            pos++;
            R.init(words, pos);
            return;
        }
        // the interval's 1-bit padding (< 8 bits) or its pad bytes: next interval.
        // A symbol that reached past the interval's data read pad bits (ones)
        // where libjpeg reads zeros after setting insufficient_data: not the
        // clean case either (seq_decode's)
        if (OWNED && pos > bound) bad = true;
        // a block left half-decoded: the interval held more data than its MCUs
        // (libjpeg skips it at the restart); its symbols sit in the assembly
        // slot the next block would inherit
        if (OWNED && partial) bad = true;
        if (nx == DEC_END) {
            pos = DEC_END;
            return;
        }
        // the true walk leaves interval k-1 after exactly its ri MCUs; an RSTn
        // anywhere else (a stray or missing marker) is damaged data, on which
        // libjpeg's resynchronisation and zero fill give other pixels
        if (OWNED && ri > 0 && blk_base + (int64_t)n != (int64_t)k * ri * nbm) bad = true;
        pos = nx * 8;
        R.init(words, pos);
    }
};

template <bool OWNED, class HuffPtr>
ICX_HD DecWalker<OWNED, HuffPtr> dec_walker(const DecDesc& d, HuffPtr H, const DecSlow* slow, uint32_t selp,
                                            const uint32_t* words, const uint32_t* seg, uint32_t nseg,
                                            uint32_t ent_bits, int64_t blk_base)
{
    DecWalker<OWNED, HuffPtr> w;
    w.H = H;
    w.slow = (const ICX_GLOBAL DecSlow*)slow;
    w.selp = selp;
    w.words = words;
    w.seg = (const ICX_GLOBAL uint32_t*)seg;
    w.nseg = nseg;
    w.ent_bits = ent_bits;
    w.nby = d.nby;
    w.nbmcu = d.wmcu;
    w.ri = d.ri;
    w.nbm = d.nbmcu;
    w.nblocks = d.nblocks;
    w.blk_base = blk_base;
    return w;
}

// The walk of one thread (active == false: this lane only keeps the wave's
// uniform loop company).  On the device the loop is wave-uniform so the
// window top-ups happen together (DecReader).
template <bool OWNED, class HuffPtr, class Sink>
ICX_HD uint64_t dec_walk(const DecDesc& d, HuffPtr H, const DecSlow* slow, uint32_t selp, const uint32_t* words,
                         const uint32_t* seg, uint32_t nseg, uint32_t ent_bits, uint64_t st, uint32_t stop,
                         uint32_t& nblk, int64_t blk_base, Sink& sink, bool active = true)
{
    nblk = 0;
    DecWalker<OWNED, HuffPtr> w = dec_walker<OWNED>(d, H, slow, selp, words, seg, nseg, ent_bits, blk_base);
    const bool started = active && !(dec_pos(st) >= stop && (!OWNED || (st & 63) == 0));
    bool run = false;
    if (started) {
        w.start(st);
        run = w.running(stop);
    }
#if defined(__HIP_DEVICE_COMPILE__)
    while (__any(run)) {
        if (run) {
            w.step(sink);
            run = w.running(stop);
        }
        if (__any(run && w.R.low()) && run && w.R.wants()) w.R.top_up();
    }
#else
    while (run) {
        w.step(sink);
        run = w.running(stop);
    }
#endif
    if (!started) return st;
    nblk = w.n;
    return w.state();
}

// ---------------------------------------------------------------------------
// The state-only walk (k_dec_init warm-ups, k_dec_sync): DecWalker<false>'s
// transitions over DecLean entries.  Per symbol: refill, one look-up, skip
// the consumed bits, add to the zig-zag index, next block at >= 64 - the
// symbol itself (run, size, extra bits, value) is never decoded.  Every
// transition equals DecWalker<false>::step's (tests/dec_emu.cpp
// dec_emu_lean_check walks both from the same states), so the states the
// relaxation settles on are the ones the write pass's DecWalker<true> walks.
template <class LeanPtr>
ICX_HD uint32_t dec_lean_symbol(LeanPtr t, const ICX_GLOBAL DecSlow* slow, uint32_t pk, bool ac)
{
    const uint32_t e = t->lut[pk >> (16 - DEC_LUT_BITS)];
    // codes of at most DEC_LUT_BITS bits (or none): one bit test on the common
    // path - DEC_LEAN_LONG is a zig-zag advance of 32, which no symbol has
    if (!(e & DEC_LEAN_LONG)) return e;
    if (!(e & DEC_LEAN_SLOW)) return t->lut2[(e >> 5) & (DEC_NSUB - 1)][pk & ((1u << (16 - DEC_LUT_BITS)) - 1)];
    for (int l = DEC_LUT_BITS + 1; l <= 16; l++) {
        const int code = (int)(pk >> (16 - l));
        if (code <= slow->maxcode[l]) return dec_lean_entry(l, slow->vals[(slow->valoff[l] + code) & 255], ac);
    }
    return 0;
}

// First levels in one place (LDS) and the whole tables in global memory
// (k_dec_write keeps only the 10-bit first levels in LDS).
struct SplitLean {
    const uint32_t (*lut)[1 << DEC_LUT_BITS];
    const ICX_GLOBAL DecLean* full;
};
template <class LeanPtr>
ICX_HD uint32_t dec_lean_lookup(LeanPtr H, int ti, const ICX_GLOBAL DecSlow* slow, uint32_t pk, bool ac)
{
    return dec_lean_symbol(&H[ti], &slow[ti], pk, ac);
}
// Write-pass second levels: through the scalar cache (SCALAR2) and the rare
// vector fallback waited for inside its branch (LOCAL_WAIT).  Before, the
// compiler waited vmcnt(0) after the look-up on every symbol step, i.e. for
// every coefficient store the wave had in flight: decode 90.4 -> 88.5 ms per
// 1000-frame call (profiles/r4/ab_r4n_dec_wait.txt).
#ifndef ICX_DEC_SCALAR2
#define ICX_DEC_SCALAR2 1
#endif
#ifndef ICX_DEC_LOCAL_WAIT
#define ICX_DEC_LOCAL_WAIT 1
#endif
ICX_HD uint32_t dec_lean_lookup(const SplitLean& H, int ti, const ICX_GLOBAL DecSlow* slow, uint32_t pk, bool ac)
{
    uint32_t e = H.lut[ti][pk >> (16 - DEC_LUT_BITS)];
#if defined(__HIP_DEVICE_COMPILE__) && ICX_DEC_SCALAR2
    // Second levels (codes longer than DEC_LUT_BITS, ~0.3 % of q95 symbols but
    // a lane of the wave in ~15 % of steps) through the scalar cache, one lane
    // at a time: a vector load here would be waited for with vmcnt, i.e.
    // behind every coefficient store the wave still has in flight.
    uint64_t m = __ballot((e & (DEC_LEAN_LONG | DEC_LEAN_SLOW)) == DEC_LEAN_LONG);
    if (m) {
        const uint32_t off = (uint32_t)(ti * sizeof(DecLean) + offsetof(DecLean, lut2)) +
                             ((((e >> 5) & (DEC_NSUB - 1)) << (16 - DEC_LUT_BITS)) | (pk & ((1u << (16 - DEC_LUT_BITS)) - 1))) * 2;
        const uint64_t base = (uint64_t)(uintptr_t)H.full;
        const int lane = (int)__lane_id();
        do {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t o = __builtin_amdgcn_readlane(off, l);
            const uint32_t w = *(const __attribute__((address_space(4))) uint32_t*)(uintptr_t)(base + (o & ~3u));
            if (lane == l) e = (w >> ((o & 2u) * 8)) & 0xFFFFu;
        } while (m);
    }
#endif
#if defined(__HIP_DEVICE_COMPILE__) && ICX_DEC_LOCAL_WAIT
    // A long code's second level is a vector load.  Consumed inside the rare
    // branch (the v_mov), it is also waited for there; consumed after the
    // join, the compiler waited vmcnt(0) at the join on every step - behind
    // every coefficient store the wave still had in flight.
    if (e & DEC_LEAN_LONG) {
        const uint32_t e2 = dec_lean_symbol(&H.full[ti], &slow[ti], pk, ac);
        asm volatile("v_mov_b32 %0, %1" : "=v"(e) : "v"(e2));
    }
    return e;
#else
    return !(e & DEC_LEAN_LONG) ? e : dec_lean_symbol(&H.full[ti], &slow[ti], pk, ac);
#endif
}

template <class P>
struct dec_is_lean {
    static constexpr bool value = false;
};
template <>
struct dec_is_lean<DecLean*> {
    static constexpr bool value = true;
};
template <>
struct dec_is_lean<const DecLean*> {
    static constexpr bool value = true;
};
template <>
struct dec_is_lean<SplitLean> {
    static constexpr bool value = true;
};

template <class LeanPtr>
struct DecLeanWalker {
    static_assert(dec_is_lean<LeanPtr>::value, "state-only walks read DecLean tables");
    LeanPtr H;
    const ICX_GLOBAL DecSlow* slow;
    uint32_t selp;
    const ICX_GLOBAL uint32_t* seg;
    uint32_t nseg, ent_bits;
    int nby, nbmcu;
#if ICX_DEC_BSEL32
    uint32_t bsel;  // dec_block_sel (<= 8 blocks)
#else
    uint64_t bsel;  // dec_block_sel
#endif
    uint32_t pos, n;
    int b, z, ti;  // ti: table of the next symbol (component of block b, DC at z == 0)
    bool two;      // the last step was a symbol pair (tests compare against DecWalker's single steps)
    DecLeanReader R;
    const uint32_t* words;

#if ICX_DEC_BSEL && ICX_DEC_BSEL32
    ICX_HD int table(int bb, int zz) const { return (int)dec_bsel_bits(bsel, 4u * (uint32_t)bb + (zz != 0 ? 2u : 0u)); }
    // after a step (z >= 1 unless the block ended): the next symbol's table
    ICX_HD int table_after(bool end) const { return (int)dec_bsel_bits(bsel, ((uint32_t)b << 2) | (end ? 0u : 2u)); }
#elif ICX_DEC_BSEL
    ICX_HD int table(int bb, int zz) const { return dec_block_table(bsel, bb, zz); }
    ICX_HD int table_after(bool) const { return table(b, z); }
#else
    ICX_HD int table(int bb, int zz) const { return dec_sel(selp, bb < nby ? 0 : bb - nby + 1, zz != 0 ? 1 : 0); }
    ICX_HD int table_after(bool) const { return table(b, z); }
#endif
    ICX_HD void start(uint64_t st)
    {
        pos = dec_pos(st);
        b = (int)((st >> 8) & 7);
        z = (int)(st & 63);
        n = 0;
        ti = table(b, z);
        R.init(words, pos);
    }
    ICX_HD bool running(uint32_t stop) const { return pos < stop; }
    ICX_HD uint64_t state() const { return dec_pack(pos, b, z); }
    // a lane with no walk (it only keeps the wave's loop company, step(false)):
    // a state that reads no memory
    ICX_HD void park()
    {
        pos = DEC_END;
        b = z = ti = 0;
        n = 0;
        R.park();
    }
    // act == false: a lane whose walk has ended keeps the wave's loop company
    // without changing its state (no exec-masked region around the step: the
    // loop state then needs no merge copies at the loop head)
    ICX_HD void step(bool act = true)
    {
        R.refill();
        // a lane without a walk steps on entry 0, which changes nothing
        const uint32_t e = act ? dec_lean_lookup(H, ti, slow, R.peek16(), z != 0) : 0u;
        const int c1 = (int)(e & 31);
        // straight-line transition (an invalid entry, 0, leaves the state as
        // it is), then the rare invalid-code path overrides it
        const int z1 = z + (int)((e >> 5) & 127);
        // the pair's second symbol, unless the first ended the block
        const int c2 = (int)((e >> DEC_PAIR_SHIFT) & 31);
        two = c2 != 0 && z1 < 64;
        const int c = c1 + (two ? c2 : 0);
        R.skip(c);
        pos += (uint32_t)c;
        z = z1 + (two ? (int)(e >> 25) : 0);
        const bool end = z >= 64;
        n += end ? 1u : 0u;
        const int bn = b + 1 == nbmcu ? 0 : b + 1;
        b = end ? bn : b;
        z = end ? 0 : z;
        ti = table_after(end);  // (a lane without a walk never looks up again)
        if (act && c == 0) invalid();  // no valid code here
    }
    // DecWalker<false>::invalid: resume a bit later mid-interval, else the
    // next interval (or the end)
    ICX_HD void invalid()
    {
        uint32_t k;
        const uint32_t nx = dec_next_seg(seg, nseg, pos >> 3, &k);
        const uint32_t bound = nx == DEC_END ? ent_bits : (nx - DEC_PAD) * 8;
        b = 0;
        z = 0;
        ti = table(0, 0);
        if (pos + 8 < bound) {
            pos++;
            R.init(words, pos);
            return;
        }
        if (nx == DEC_END) {
            pos = DEC_END;
            return;
        }
        pos = nx * 8;
        R.init(words, pos);
    }
};

template <class LeanPtr>
ICX_HD DecLeanWalker<LeanPtr> dec_lean_walker(const DecDesc& d, LeanPtr H, const DecSlow* slow, uint32_t selp,
                                              const uint32_t* words, const uint32_t* seg, uint32_t nseg,
                                              uint32_t ent_bits)
{
    DecLeanWalker<LeanPtr> w;
    w.H = H;
    w.slow = (const ICX_GLOBAL DecSlow*)slow;
    w.selp = selp;
    w.words = words;
    w.seg = (const ICX_GLOBAL uint32_t*)seg;
    w.nseg = nseg;
    w.ent_bits = ent_bits;
    w.nby = d.nby;
    w.nbmcu = d.wmcu;
    w.bsel = (decltype(w.bsel))dec_uniform(dec_block_sel(selp, d.nby, d.wmcu));
    return w;
}

// dec_walk<false> over the lean tables (k_dec_init's warm-up walk).
template <class LeanPtr>
ICX_HD uint64_t dec_lean_walk(const DecDesc& d, LeanPtr H, const DecSlow* slow, uint32_t selp, const uint32_t* words,
                              const uint32_t* seg, uint32_t nseg, uint32_t ent_bits, uint64_t st, uint32_t stop,
                              uint32_t& nblk, bool active = true)
{
    nblk = 0;
    DecLeanWalker<LeanPtr> w = dec_lean_walker(d, H, slow, selp, words, seg, nseg, ent_bits);
    const bool started = active && dec_pos(st) < stop;
    bool run = false;
    if (started) {
        w.start(st);
        run = w.running(stop);
    } else {
        w.park();
    }
#if defined(__HIP_DEVICE_COMPILE__) && ICX_DEC_WALK_UNROLL2
    while (__any(run)) {  // two steps per top-up check (a step consumes <= 1 window word)
        w.step(run);
        run = run && w.running(stop);
        w.step(run);
        run = run && w.running(stop);
        if (__any(run && w.R.left() <= 2) && run) w.R.top_up();
    }
#elif defined(__HIP_DEVICE_COMPILE__)
    while (__any(run)) {
        w.step(run);  // predicated: lanes that are done keep their state
        run = run && w.running(stop);
        if (__any(run && w.R.low()) && run && w.R.wants()) w.R.top_up();
    }
#else
    while (run) {
        w.step();
        run = w.running(stop);
    }
#endif
    if (!started) return st;
    nblk = w.n;
    return w.state();
}

// The last sz of the first c bits of an MSB-first bit buffer (c <= 32: the
// field lies in its high word), a symbol's value bits: one bit-field extract
// on the device instead of a 64-bit shift and a mask.
#ifndef ICX_DEC_VALUE_BFE
#define ICX_DEC_VALUE_BFE 1  // +-0 alone (ab_r5aq_dec_write_lim.txt)
#endif
ICX_HD uint32_t dec_value_bits(uint64_t buf, int c, int sz)
{
#if defined(__HIP_DEVICE_COMPILE__) && ICX_DEC_VALUE_BFE
    return __builtin_amdgcn_ubfe((uint32_t)(buf >> 32), (uint32_t)(32 - c), (uint32_t)sz);
#else
    return (uint32_t)(buf >> (64 - c)) & ((1u << sz) - 1u);
#endif
}

// The write pass's walk (k_dec_write): DecWalker<true>'s transitions and
// sink calls over DecLean entries - the coefficient's value is the last
// `extra bits` of the bits the entry consumes, its zig-zag index z + zadd - 1.
// tests/dec_emu.cpp dec_emu_lean_check records both walkers' sink calls from
// random states and entry points and compares them.
template <class LeanPtr>
struct DecLeanWriter {
    static_assert(dec_is_lean<LeanPtr>::value, "the write walk reads DecLean tables");
    LeanPtr H;
    const ICX_GLOBAL DecSlow* slow;
    uint32_t selp;
    const ICX_GLOBAL uint32_t* seg;
    uint32_t nseg, ent_bits;
    int nby, nbmcu;
    int ri, nbm;
    int64_t nblocks;
#if ICX_DEC_BSEL32
    uint32_t bsel;  // dec_block_sel (<= 8 blocks)
#else
    uint64_t bsel;  // dec_block_sel
#endif
    uint32_t pos, n;
    int b, z, ti;
    // 63 once the walk owns its block, 0 before (the partial block it starts
    // in belongs to the previous piece): a put goes to min(index, own), so a
    // put before the first owned block lands on index 0, which that block's
    // DC overwrites - one v_min per put instead of a clamp and a select
    int own;
    static constexpr int OWN_SCALE = ICX_DEC_PUT2 ? 2 : 1;  // own in put2's units
    bool bad;
    bool two;  // the last step was a symbol pair
    int64_t blk_base;
    uint32_t nlim;  // blocks from blk_base to the image's end (clamped to 32 bits)
#if ICX_DEC_FUNNEL_WRITE
    DecFunnelReader<DEC_WIN_WRITE, ICX_DEC_LDS_WIN_WRITE != 0> R;
#else
    DecReaderT<DEC_WIN_WRITE, ICX_DEC_LDS_WIN_WRITE != 0> R;
#endif
    const uint32_t* words;

#if ICX_DEC_BSEL && ICX_DEC_BSEL32
    ICX_HD int table(int bb, int zz) const { return (int)dec_bsel_bits(bsel, 4u * (uint32_t)bb + (zz != 0 ? 2u : 0u)); }
    // after a step (z >= 1 unless the block ended): the next symbol's table
    ICX_HD int table_after(bool end) const { return (int)dec_bsel_bits(bsel, ((uint32_t)b << 2) | (end ? 0u : 2u)); }
#elif ICX_DEC_BSEL
    ICX_HD int table(int bb, int zz) const { return dec_block_table(bsel, bb, zz); }
    ICX_HD int table_after(bool) const { return table(b, z); }
#else
    ICX_HD int table(int bb, int zz) const { return dec_sel(selp, bb < nby ? 0 : bb - nby + 1, zz != 0 ? 1 : 0); }
    ICX_HD int table_after(bool) const { return table(b, z); }
#endif
    ICX_HD void start(uint64_t st)
    {
        pos = dec_pos(st);
        b = (int)((st >> 8) & 7);
        z = (int)(st & 63);
        n = 0;
        own = z == 0 ? 63 * OWN_SCALE : 0;
        bad = false;
        ti = table(b, z);
        R.init(words, pos);
    }
    ICX_HD bool running(uint32_t stop) const { return pos < stop || z != 0; }
    ICX_HD uint64_t state() const { return dec_pack(pos, b, z); }
    ICX_HD static int dec_extend_bf(uint32_t v, int sz)
    {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t m = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0u, (uint32_t)sz);  // one v_bfe_u32 (sz = 0: 0)
#else
        const uint32_t m = (1u << sz) - 1u;
#endif
        return (int)(v <= (m >> 1) ? v - m : v);
    }
#if ICX_DEC_FUNNEL_WRITE
    // value bits of a symbol whose code and value end `end` bits into the
    // step's 32-bit look-ahead (end <= 31: a code and its extra bits, or a pair)
    ICX_HD static uint32_t value_at(uint32_t x, int end, int sz)
    {
#if defined(__HIP_DEVICE_COMPILE__)
        return __builtin_amdgcn_ubfe(x, (uint32_t)(32 - end), (uint32_t)sz);
#else
        return (x >> (32 - end)) & ((1u << sz) - 1u);
#endif
    }
#endif
    template <class Sink>
    ICX_HD void step(Sink& sink)
    {
        R.refill();
#if ICX_DEC_FUNNEL_WRITE
        const uint32_t X = R.peek32();
        const uint32_t e = dec_lean_lookup(H, ti, slow, X >> 16, z != 0);
#else
        const uint32_t e = dec_lean_lookup(H, ti, slow, R.peek16(), z != 0);
#endif
        const int c = (int)(e & 31);
        two = false;
        if (c == 0) {  // no valid code here
            invalid();
            return;
        }
        const int sz = (int)((e >> 12) & 15), zadd = (int)((e >> 5) & 127);
#if ICX_DEC_FUNNEL_WRITE
        const uint32_t v = value_at(X, c, sz);
#else
        const uint32_t v = dec_value_bits(R.buf, c, sz);
        R.skip(c);
        pos += (uint32_t)c;
#endif
#if ICX_DEC_EXT_BF
        // HUFF_EXTEND without the sz == 0 branch (v = 0 and m = 0 then): v
        // below half = (m + 1) / 2 is v <= m / 2 - mask, shift, compare,
        // select, subtract
        const int x = dec_extend_bf(v, sz);
#else
        const int x = sz ? dec_extend((int)v, sz) : 0;
#endif
        // zig-zag index of a coefficient (DC: 0).  A size-0 symbol (EOB, ZRL,
        // a zero DC difference) puts its 0 at z + advance - 1 (clamped), a
        // position its zero run covers and nothing wrote yet in the zeroed
        // slot - no select for it
#if ICX_DEC_PUT2
        z += zadd;
        {
            const int zc2 = (z << 1) - 2;
            sink.put2(zc2 < own ? zc2 : own, x);
        }
#else
        const int zc = z + zadd - 1;
        sink.put(zc < own ? zc : own, x);
        z += zadd;
#endif
        // the pair's second symbol (an AC code inside the same look-ahead),
        // unless the first ended the block: its value bits follow its code
        const int c2 = (int)((e >> DEC_PAIR_SHIFT) & 31);
        two = c2 != 0 && z < 64;
#if ICX_DEC_FUNNEL_WRITE
        {  // one skip for the step (a pair's bits are inside the look-ahead)
            const int ct = c + (two ? c2 : 0);
            R.skip(ct);
            pos += (uint32_t)ct;
        }
#endif
        if (two) {
            const int sz2 = (int)((e >> 21) & 15), zadd2 = (int)(e >> 25);
#if ICX_DEC_FUNNEL_WRITE
            const uint32_t v2 = value_at(X, c + c2, sz2);
#else
            const uint32_t v2 = dec_value_bits(R.buf, c2, sz2);
            R.skip(c2);
            pos += (uint32_t)c2;
#endif
            const int x2 = dec_extend_bf(v2, sz2);
#if ICX_DEC_PUT2
            z += zadd2;
            const int zc2 = (z << 1) - 2;
            sink.put2(zc2 < own ? zc2 : own, x2);
#else
            const int zc2 = z + zadd2 - 1;
            sink.put(zc2 < own ? zc2 : own, x2);
            z += zadd2;
#endif
        }
        const bool end = z >= 64;
#if ICX_DEC_PEND32
        sink.flush_if(end && own != 0 && n < nlim, blk_base + n);  // 32-bit bound: nlim = nblocks - blk_base
#else
        const int64_t bi = blk_base + n;
        sink.flush_if(end && own != 0 && bi < nblocks, bi);
#endif
        own = end ? 63 * OWN_SCALE : own;
        n += end ? 1u : 0u;
        const int bn = b + 1 == nbmcu ? 0 : b + 1;
        b = end ? bn : b;
        z = end ? 0 : z;
        ti = table_after(end);
    }
    // DecWalker<true>::invalid
    ICX_HD void invalid()
    {
        uint32_t k;
        const uint32_t nx = dec_next_seg(seg, nseg, pos >> 3, &k);
        const uint32_t bound = nx == DEC_END ? ent_bits : (nx - DEC_PAD) * 8;
        const bool partial = z != 0;  // DecWalker<true>::invalid
        b = 0;
        z = 0;
        ti = table(0, 0);
        own = 63 * OWN_SCALE;
        if (pos + 8 < bound) {
            bad = true;
            pos++;
            R.init(words, pos);
            return;
        }
        if (pos > bound || partial) bad = true;  // read pad bits, extra data (DecWalker<true>::invalid)
        if (nx == DEC_END) {
            pos = DEC_END;
            return;
        }
        if (ri > 0 && blk_base + (int64_t)n != (int64_t)k * ri * nbm) bad = true;
        pos = nx * 8;
        R.init(words, pos);
    }
    // After the walk: it stopped (at its exit mark) past the data of the
    // interval its last symbol came from, i.e. that symbol read pad bits, and
    // no invalid code followed to flag it.  A position exactly at an interval
    // start is a jump (invalid() above), not a symbol's end: a symbol can
    // reach at most 31 bits into the DEC_PAD bytes of all-ones.
    ICX_HD bool overran() const
    {
        if (pos == DEC_END || pos == 0) return false;
        uint32_t k;
        const uint32_t nx = dec_next_seg(seg, nseg, (pos - 1) >> 3, &k);
        const uint32_t bound = nx == DEC_END ? ent_bits : (nx - DEC_PAD) * 8;
        return pos > bound && (nx == DEC_END || pos != nx * 8);
    }
};

template <class LeanPtr>
ICX_HD DecLeanWriter<LeanPtr> dec_lean_writer(const DecDesc& d, LeanPtr H, const DecSlow* slow, uint32_t selp,
                                              const uint32_t* words, const uint32_t* seg, uint32_t nseg,
                                              uint32_t ent_bits, int64_t blk_base)
{
    DecLeanWriter<LeanPtr> w;
    w.H = H;
    w.slow = (const ICX_GLOBAL DecSlow*)slow;
    w.selp = selp;
    w.words = words;
    w.seg = (const ICX_GLOBAL uint32_t*)seg;
    w.nseg = nseg;
    w.ent_bits = ent_bits;
    w.nby = d.nby;
    w.nbmcu = d.wmcu;
    w.ri = d.ri;
    w.nbm = d.nbmcu;
    w.nblocks = d.nblocks;
    w.blk_base = blk_base;
    const int64_t lim = d.nblocks - blk_base;
    w.nlim = lim <= 0 ? 0u : lim >= (int64_t)0xFFFFFFFF ? 0xFFFFFFFFu : (uint32_t)lim;
    w.bsel = (decltype(w.bsel))dec_uniform(dec_block_sel(selp, d.nby, d.wmcu));
    return w;
}

// ---------------------------------------------------------------------------
// Sync-walk checkpoints.  A walk records its state at the first symbol boundary
// at or beyond each interior mark base + (k + 1) * dec_ck_bits of its
// subsequence, with the blocks completed before it in bits 48..63.  The state
// (pos, block in MCU, zig-zag index) determines the rest of the walk, so a
// later walk of the same subsequence that reaches a recorded state can stop
// there: its exit is the recorded walk's exit, and its block count that walk's
// count plus the difference at the checkpoint.  A re-walk from a corrected
// entry state typically resynchronises within a few hundred bits, so relaunch
// walks cost about one checkpoint interval instead of a whole subsequence.
//
// Checkpoint intervals (= write-pass pieces) per subsequence: 8 (intervals of
// at least 2048 bits) below 65536-bit subsequences, DEC_CK_DIV from there.
// 16 at 65536 bits (4096-bit intervals): 1000 frames 75.1 vs 75.7-76.6 ms per
// call (write pass -0.7 ms: shorter pieces even out its lanes); at 200 frames
// (32768 bits) 16 intervals of 2048 bits cost +0.3 ms, so the shorter
// subsequences keep 8 (profiles/r5/ab_r5w_dec_ck.txt).
#ifndef ICX_DEC_CK_DIV
#define ICX_DEC_CK_DIV 16  // 8 / 32: +0.7 / +1.6 ms per 1000 frames (ab_r5x_dec_ck16.txt, ab_r5ay_dec_ck32.txt)
#endif
constexpr int DEC_CK_DIV = ICX_DEC_CK_DIV;
static_assert(DEC_CK_DIV >= 8, "shorter subsequences use 8 intervals");
constexpr int DEC_CK_MAX = DEC_CK_DIV - 1;
#ifndef ICX_DEC_CK_SMALL_DIV
#define ICX_DEC_CK_SMALL_DIV 8  // intervals below 65536-bit subsequences (at least 2048 bits each); 16: +0.3 ms at 200 frames, +-0 at 64 (ab_r5av_dec_ck_small16.txt)
#endif
static_assert(ICX_DEC_CK_SMALL_DIV <= DEC_CK_DIV, "checkpoint slots");
constexpr uint64_t DEC_CK_NONE = ~0ull;
constexpr uint64_t DEC_CK_STATE = (1ull << 48) - 1;
ICX_HD uint32_t dec_ck_bits(uint32_t sub_bits)
{
    if (sub_bits >= 65536) return sub_bits / DEC_CK_DIV;
    return sub_bits / ICX_DEC_CK_SMALL_DIV > 2048 ? sub_bits / ICX_DEC_CK_SMALL_DIV : 2048;
}
ICX_HD int dec_ck_slots(uint32_t sub_bits)
{
    const uint32_t c = dec_ck_bits(sub_bits);
    return sub_bits > c ? (int)(sub_bits / c) - 1 : 0;
}

// Checkpoint store of a subsequence's first walk: records, never matches.
template <class P>
struct CkRecord {
    P ck;  // DEC_CK_MAX slots
    int nck;
    ICX_HD bool visit(int k, uint64_t s, uint32_t&) { ck[k] = s; return false; }
    ICX_HD void finish(int k, bool)
    {
        for (; k < nck; k++) ck[k] = DEC_CK_NONE;
    }
};

// Checkpoints of a re-walk, compared in place: the previous walk's checkpoint
// k is read into a register one mark ahead, before this walk overwrites it,
// and on a match the later ones - not yet overwritten - are spliced with the
// block-count difference.  No private copy of the previous walk's checkpoints
// (k_dec_sync's relaunches kept one in LDS until round 4: 14 KiB a workgroup,
// five workgroups per CU instead of eight).  o = ck[0] on entry.
template <class P>
struct CkInPlace {
    P ck;
    int nck;
    uint32_t total;
    uint64_t o;
    ICX_HD bool visit(int k, uint64_t s, uint32_t& nblk)
    {
        const uint64_t ok = o;
        if (ok != DEC_CK_NONE && ((ok ^ s) & DEC_CK_STATE) == 0) {
            const int32_t delta = (int32_t)(s >> 48) - (int32_t)(ok >> 48);
            for (int q = k + 1; q < nck; q++) {
                const uint64_t v = ck[q];
                if (v != DEC_CK_NONE) ck[q] = v + ((uint64_t)(int64_t)delta << 48);
            }
            ck[k] = s;
            nblk = total + (uint32_t)delta;
            return true;
        }
        o = k + 1 < nck ? ck[k + 1] : DEC_CK_NONE;
        ck[k] = s;
        return false;
    }
    ICX_HD void finish(int k, bool early)
    {
        if (!early)
            for (; k < nck; k++) ck[k] = DEC_CK_NONE;
    }
};

// One sync walk of subsequence [base, base + sub_bits) from entry state st
// (H: the image's DecLean tables), with checkpoints (policy ck).  Returns the exit state, or st with early ==
// true when the walk met the previous walk (exit unchanged); nblk = blocks
// completed inside the subsequence either way.
template <class HuffPtr, class Ck>
ICX_HD uint64_t dec_sync_walk(const DecDesc& d, HuffPtr H, const DecSlow* slow, uint32_t selp,
                              const uint32_t* words, const uint32_t* seg, uint32_t nseg, uint32_t ent_bits,
                              uint64_t st, uint32_t base, uint32_t sub_bits, uint32_t& nblk, bool& early, Ck& ck,
                              bool active = true)
{
    const uint32_t stop = base + sub_bits, ckb = dec_ck_bits(sub_bits);
    const int nck = dec_ck_slots(sub_bits);
    nblk = 0;
    early = false;
    DecLeanWalker<HuffPtr> w = dec_lean_walker(d, H, slow, selp, words, seg, nseg, ent_bits);
    const bool started = active && dec_pos(st) < stop;
    bool run = false;
    if (started) {
        w.start(st);
        run = w.running(stop);
    } else {
        w.park();
    }
    int k = 0;
    uint32_t ckpos = base + ckb;
    auto one = [&]() {
        w.step(run);  // predicated: lanes that are done keep their state
        while (run && k < nck && w.pos >= ckpos) {  // a jump (END, next interval) may pass several marks
            if (ck.visit(k, w.state() | ((uint64_t)w.n << 48), nblk)) {
                early = true;
                break;
            }
            k++;
            ckpos += ckb;
        }
        run = run && !early && w.running(stop);
    };
#if defined(__HIP_DEVICE_COMPILE__) && ICX_DEC_WALK_UNROLL2
    while (__any(run)) {  // two steps per top-up check (a step consumes <= 1 window word)
        one();
        one();
        if (__any(run && w.R.left() <= 2) && run) w.R.top_up();
    }
#elif defined(__HIP_DEVICE_COMPILE__)
    while (__any(run)) {
        one();
        if (__any(run && w.R.low()) && run && w.R.wants()) w.R.top_up();
    }
#else
    while (run) one();
#endif
    if (active) ck.finish(k, early);
    if (!started || early) return st;
    nblk = w.n;
    return w.state();
}

// Write-pass pieces.  After the sync has settled, the checkpoints of
// subsequence j are states of its true walk (the last walk of j started from
// the final E[j]; a re-walk that met its previous walk spliced the rest with
// the block-count difference), so the write pass splits every subsequence
// at them: piece p of j starts at E[j] (p = 0) or at checkpoint p - 1, with
// the blocks completed before it (boff[j] + the checkpoint's count), and
// stops at the first symbol boundary at or beyond the next mark (the end of
// the subsequence for the last piece).  Ownership is as for subsequences: a
// block belongs to the piece where its DC symbol starts.  A piece whose
// checkpoint was never reached (the walk ended first) has nothing to do.
struct DecPiece {
    uint64_t e;     // entry state
    int64_t blk;    // blocks completed before it
    uint32_t stop;  // exit mark
    bool have;
};
ICX_HD int dec_pieces(uint32_t sub_bits) { return dec_ck_slots(sub_bits) + 1; }

template <class P64, class P32>
ICX_HD DecPiece dec_piece(P64 est, P64 ck, P32 boff, uint32_t j, int p, uint32_t sub_bits)
{
    const int np = dec_pieces(sub_bits);
    const uint32_t base = j * sub_bits;
    DecPiece r;
    r.stop = p + 1 < np ? base + (uint32_t)(p + 1) * dec_ck_bits(sub_bits) : base + sub_bits;
    r.have = true;
    if (p == 0) {
        r.e = est[j];
        r.blk = (int64_t)boff[j];
        return r;
    }
    const uint64_t c = ck[(int64_t)j * DEC_CK_MAX + p - 1];
    r.have = c != DEC_CK_NONE;
    r.e = c & DEC_CK_STATE;
    r.blk = (int64_t)boff[j] + (int64_t)(c >> 48);
    return r;
}

// Unstuffing rule for stuffed byte i (jdhuff.c fill_bit_buffer / jdmarker.c):
// returns output bytes it contributes (0, 1, or DEC_PAD for an RSTn code byte);
// *rst = 1 for an RSTn code byte.
ICX_HD int dec_unstuff_rule(int prev, int cur, int next, int* rst)
{
    *rst = 0;
    if (prev == 0xFF && cur == 0x00) return 0;                 // stuffed zero
    if (cur == 0xFF) return next == 0x00 ? 1 : 0;              // data 0xFF / marker prefix / fill
    if (prev == 0xFF && cur >= 0xD0 && cur <= 0xD7) {          // RSTn code
        *rst = 1;
        return DEC_PAD;
    }
    return 1;
}

}  // namespace icx
