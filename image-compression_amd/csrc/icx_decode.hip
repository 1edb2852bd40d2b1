// icx_decode.hip — CDNA4 (gfx950) kernels of the device JPEG decoder (row A11:
// the JDK JPEGImageReader decode behind ImageCompression.decodeImageWithSubsampling,
// core/ImageCompression.java:107-165; IJG 6b arithmetic, see
// oracle/icx_oracle_decode.c for the CPU statement of the same algorithm).
//
// Kernel map (per sub-batch of images, all launched on the context's stream):
//   k_unstuff_count    per 4 KiB tile: unstuffed bytes (RSTn -> DEC_PAD bytes),
//                      and the first terminating marker of each entropy segment
//   k_unstuff_scan     per image: tile offsets (the marker's tile recounted),
//                      stream length, tail pad
//   k_unstuff_scatter  compact the stream, record restart-interval starts
//   k_dec_init         guessed entry state of every subsequence
//   k_dec_sync         one relaxation step of E[j+1] = walk(E[j]) (icx_decode.h)
//   k_dec_offsets      per image: blocks before each subsequence, block count check
//   k_dec_write        decode again from the settled states, store coefficients
//   k_dec_dc           per image: DC prediction (segmented per restart interval)
//   k_dec_idct         jpeg_idct_islow of every real block into component planes
//                      (chroma blocks only when k_dec_luma_color_420 runs)
//   k_dec_luma_color_420  s == 1 4:2:0 fancy: luma IDCT + h2v2 fancy upsampling
//                      + ycc_rgb_convert, one MCU row x 8 MCUs per workgroup
//   k_dec_color        fancy upsampling + ycc_rgb_convert + source subsampling
// Byte/bit-serial integer work; no MFMA.  The entropy stages are bound by the
// dependent table look-ups of the bit-serial walk, the pixel stages by HBM.
#include <hip/hip_runtime.h>

#include "icx_decode.h"
#include "icx_decode_kernels.h"

namespace icx {

namespace {

__device__ __forceinline__ int slot_of(const int64_t* prefix, int m, int64_t item)
{
    int lo = 0, hi = m;  // prefix[lo] <= item < prefix[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (prefix[mid] <= item) lo = mid; else hi = mid;
    }
    return lo;
}

// Slot and item of this workgroup: 2-D launches (Plan.width > 0: x = item,
// y = slot) need no search and drop the items past a slot's count; 1-D
// launches search the prefix array.
__device__ __forceinline__ bool plan_slot(const Plan& p, int& slot, int64_t& item)
{
    if (gridDim.y > 1) {
        slot = (int)blockIdx.y;
        item = blockIdx.x;
        return item < p.prefix[slot + 1] - p.prefix[slot];
    }
    slot = slot_of(p.prefix, p.m, blockIdx.x);
    item = blockIdx.x - p.prefix[slot];
    return true;
}

// Block-wide exclusive scan of one uint32 per thread (blockDim.x == NT).
template <int NT>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* sh, uint32_t& total)
{
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < NT / 64; i++) {
            const uint32_t s = sh[i];
            sh[i] = acc;
            acc += s;
        }
        sh[NT / 64] = acc;
    }
    __syncthreads();
    total = sh[NT / 64];
    const uint32_t r = x - v + sh[w];
    __syncthreads();
    return r;
}

// 16 stuffed bytes at scan offset `base` (< scan_len) as four dwords, with
// the byte after them; bytes at or past scan_len read as zero.  The scan may
// start at any byte address - a device-resident file is read where it lies,
// no staging copy: the two aligned 16-B chunks covering the bytes are loaded
// (the second only when it holds a scan byte, so no load leaves the file's
// pages) and the misalignment, uniform over the image, is shifted out.
struct Scan16 {
    uint4 v;
    int next;
};
__device__ __forceinline__ Scan16 scan16(const uint8_t* scan, int64_t scan_len, int64_t base)
{
    const uintptr_t p = (uintptr_t)(scan + base), a = p & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(p & 15), q = sh >> 2, b = sh & 3;
    const bool more = a + 16 < (uintptr_t)(scan + scan_len);
    // global (not flat) loads: they wait on vmcnt alone, not on the LDS counter too
    const uint4 c0 = *(const ICX_GLOBAL uint4*)a;
    uint4 c1 = *(const ICX_GLOBAL uint4*)(more ? a + 16 : a);  // unconditional: no branch and wait around the load
    if (!more) c1 = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t x[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    uint32_t y[5];
#pragma unroll
    for (int k = 0; k < 5; k++) y[k] = q == 0 ? x[k] : q == 1 ? x[k + 1] : q == 2 ? x[k + 2] : x[k + 3];
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = __builtin_amdgcn_alignbyte(y[k + 1], y[k], b);
    Scan16 r;
    r.next = (int)((y[4] >> (8 * b)) & 255u);
    const int64_t rem = scan_len - base;
    if (rem <= 16) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t nb = rem - 4 * k;  // scan bytes in dword k
            if (nb < 4) w[k] = nb <= 0 ? 0u : w[k] & ((1u << (8 * nb)) - 1);
        }
        r.next = 0;
    }
    r.v = make_uint4(w[0], w[1], w[2], w[3]);
    return r;
}

}  // namespace

// -------------------------------------------------------------------- stage
// Gathers file bytes into aligned, zero-padded device buffers for a whole
// sub-batch in one launch (headers for the host parser, entropy segments for
// k_unstuff_*): 16 bytes per thread from five aligned dwords and a byte
// funnel shift; a dword is read only if it holds a byte of the source.
__global__ void __launch_bounds__(256) k_stage(const StageJob* J, Plan p)
{
    int slot;
    int64_t item;
    if (!plan_slot(p, slot, item)) return;
    const StageJob j = J[slot];
    const int64_t o = item * (int64_t)STAGE_TILE + threadIdx.x * 16;
    if (o >= j.dst_len) return;
    uint32_t w[4] = {0, 0, 0, 0};
    if (o < j.len) {
        const uintptr_t s = (uintptr_t)(j.src + o), end = (uintptr_t)(j.src + j.len);
        const uintptr_t a = s & ~(uintptr_t)3;
        const uint32_t sh = (uint32_t)(s & 3);
        uint32_t x[5];
#pragma unroll
        for (int k = 0; k < 5; k++) x[k] = a + 4 * k < end ? *(const uint32_t*)(a + 4 * k) : 0u;
        const int64_t rem = j.len - o;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
            const int64_t nb = rem - 4 * k;  // valid bytes in this dword
            if (nb < 4) v = nb <= 0 ? 0u : v & ((1u << (8 * nb)) - 1);
            w[k] = v;
        }
    }
    *(uint4*)(j.dst + o) = make_uint4(w[0], w[1], w[2], w[3]);
}

// ------------------------------------------------------------------ unstuff
// True when one of the 16 bytes or the byte before them is 0xFF: only then can
// a byte of this thread be a stuffed zero, a marker or an RSTn code.
__device__ __forceinline__ bool any_ff(const uint4& v, int prev)
{
    uint32_t m = 0;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t x = ~w[k];  // 0xFF bytes -> zero bytes
        m |= (x - 0x01010101u) & ~x & 0x80808080u;
    }
    return m != 0 || prev == 0xFF;
}

// Byte classes of 16 stuffed bytes as 16-bit masks (bit k = byte k), SWAR on
// the four dwords: 0xFF bytes, 0x00 bytes, RSTn codes (0xD0..0xD7).
__device__ __forceinline__ uint32_t zero_bytes4(uint32_t x)  // bit j: byte j of x is 0
{
    const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // exact per byte
    uint32_t m = (~nz & 0x80808080u) >> 7;  // bits 0, 8, 16, 24
    m |= m >> 7;
    m |= m >> 14;
    return m & 0xFu;
}
struct ByteClass {
    uint32_t ff, z, r;
};
__device__ __forceinline__ ByteClass classify16(const uint4& v)
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    ByteClass c{0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        c.ff |= zero_bytes4(~w[k]) << (4 * k);
        c.z |= zero_bytes4(w[k]) << (4 * k);
        c.r |= zero_bytes4((w[k] ^ 0xD0D0D0D0u) & 0xF8F8F8F8u) << (4 * k);
    }
    return c;
}

// The unstuffing rule (dec_unstuff_rule) over 16 bytes at once, given the byte
// before them (prev) and after them (next): keep = bytes contributing one
// output byte, rst = RSTn codes (DEC_PAD bytes each), mark = 0xFF bytes that
// start a terminating marker (followed by neither 0x00, 0xFF nor an RSTn code).
struct Unstuff16 {
    uint32_t keep, rst, mark;
};
__device__ __forceinline__ Unstuff16 unstuff16(const ByteClass& c, int prev, int next)
{
    const uint32_t pff = ((c.ff << 1) | (prev == 0xFF ? 1u : 0u)) & 0xFFFFu;  // byte k follows a 0xFF
    const uint32_t nz = (c.z >> 1) | (next == 0x00 ? 0x8000u : 0u);           // byte k precedes a 0x00
    const uint32_t nff = (c.ff >> 1) | (next == 0xFF ? 0x8000u : 0u);
    const uint32_t nr = (c.r >> 1) | (next >= 0xD0 && next <= 0xD7 ? 0x8000u : 0u);
    const uint32_t stuffed = pff & c.z, rst = pff & c.r & ~c.ff;
    Unstuff16 u;
    u.keep = (~c.ff & ~stuffed & ~rst & 0xFFFFu) | (c.ff & nz);
    u.rst = rst;
    u.mark = c.ff & ~nz & ~nff & ~nr;
    return u;
}

// Per 4 KiB tile: output bytes and RSTn markers of its bytes below scan_len,
// and (atomicMin into S.end) the first terminating marker - a 0xFF followed by
// neither 0x00, 0xFF nor an RSTn code.  Bytes from that marker on are dropped
// by k_unstuff_scan (it recounts the marker's tile and zeroes the tiles after
// it), so one pass over the stuffed stream finds both.  A thread whose bytes
// hold no 0xFF (nor follow one) counts them without the per-byte rule.  A
// workgroup counts DEC_UNSTUFF_TILES consecutive tiles, all their loads
// issued first (one 4 KiB tile per workgroup left each workgroup a single
// 16-byte load per thread in flight).
#ifndef ICX_UNSTUFF_COMPACT
#define ICX_UNSTUFF_COMPACT 1  // unstuffing 7.93 -> 7.14 ms at 1000 frames (ab_r5aj_dec_unstuff_compact.txt)
#endif
__global__ void __launch_bounds__(256) k_unstuff_count(const DecDesc* D, DecState* S, Plan p)
{
    constexpr int U = DEC_UNSTUFF_TILES;
    __shared__ uint32_t sh[U][4];
    int slot;
    int64_t item;
    if (!plan_slot(p, slot, item)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    const int64_t len = d.scan_len;
    const int64_t tile0 = item * U;
    Scan16 q[U];
    int prev[U];
#pragma unroll
    for (int u = 0; u < U; u++) {  // bases past the scan load its last chunk and count nothing
        const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
        const int64_t bc = base < len ? base : len - 1;
        q[u] = scan16(d.scan, len, bc);
        prev[u] = ((const ICX_GLOBAL uint8_t*)d.scan)[bc > 0 ? bc - 1 : 0];
    }
    uint32_t cnt[U];  // output bytes (bits 0..19) + RSTn markers << 20 of this thread's 16 bytes
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#if ICX_UNSTUFF_COMPACT
    // Chunks with a 0xFF byte (or one before them) are ~6 % of the stream,
    // but nearly every wave holds one, so a per-lane branch ran the masks of
    // classify16 / unstuff16 (~140 VALU) for every chunk of every wave.  Here
    // the wave counts its plain chunks directly and moves the others into
    // LDS (compacted: wave-uniform rounds of 64), so the masks run once per
    // 64 such chunks, on full lanes.
    __shared__ uint4 cv[4][64];
    __shared__ uint32_t cm[4][64];  // prev | next << 8 | u << 16 | thread << 20
    bool spc[U];
    uint32_t nsp = 0;  // special chunks of the wave so far
    uint32_t ord[U];   // this lane's index among them, per tile
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
        const int pv = base > 0 ? prev[u] : 0;
        spc[u] = base < len && any_ff(q[u].v, pv);
        cnt[u] = base < len && !spc[u] ? (uint32_t)min((int64_t)16, len - base) : 0u;
        const uint64_t m = __ballot(spc[u]);
        ord[u] = nsp + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        nsp += (uint32_t)__popcll(m);
    }
    for (uint32_t r0 = 0; r0 < nsp; r0 += 64) {  // wave-uniform
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (spc[u] && ord[u] >= r0 && ord[u] < r0 + 64) {
                const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
                const uint32_t pv = base > 0 ? (uint32_t)prev[u] : 0u;
                cv[w][ord[u] - r0] = q[u].v;
                cm[w][ord[u] - r0] = pv | (uint32_t)q[u].next << 8 | (uint32_t)u << 16 | threadIdx.x << 20;
            }
        }
        __builtin_amdgcn_wave_barrier();  // (a wave's LDS accesses complete in order)
        if (r0 + lane < nsp) {
            const uint4 v = cv[w][lane];
            const uint32_t mt = cm[w][lane];
            const int su = (int)((mt >> 16) & 15);
            const int64_t base = (tile0 + su) * DEC_TILE + (int64_t)(mt >> 20) * 16;
            const Unstuff16 x = unstuff16(classify16(v), (int)(mt & 255), (int)((mt >> 8) & 255));
            const int64_t rem = len - base;  // bytes of that chunk below scan_len
            const uint32_t valid = rem >= 16 ? 0xFFFFu : (1u << rem) - 1;
            const uint32_t nr = (uint32_t)__popc(x.rst & valid);
            const uint32_t c = (uint32_t)__popc(x.keep & valid) + DEC_PAD * nr + (nr << 20);
#pragma unroll
            for (int u = 0; u < U; u++) cnt[u] += su == u ? c : 0u;
            // a marker needs its next byte below scan_len
            const uint32_t mk = x.mark & (rem - 1 >= 16 ? 0xFFFFu : (1u << (rem - 1)) - 1);
            if (mk) atomicMin((unsigned long long*)&S[img].end, (unsigned long long)(base + __builtin_ctz(mk)));
        }
        __builtin_amdgcn_wave_barrier();  // the reads before the next round's writes
    }
#else
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
        const int pv = base > 0 ? prev[u] : 0;
        uint32_t c = 0;
        if (base < len) {
            if (!any_ff(q[u].v, pv)) {
                c = (uint32_t)min((int64_t)16, len - base);
            } else {  // branch-free rule over the 16 bytes (SWAR masks)
                const Unstuff16 x = unstuff16(classify16(q[u].v), pv, q[u].next);
                const int64_t rem = len - base;  // bytes of this thread below scan_len
                const uint32_t valid = rem >= 16 ? 0xFFFFu : (1u << rem) - 1;
                const uint32_t nr = (uint32_t)__popc(x.rst & valid);
                c = (uint32_t)__popc(x.keep & valid) + DEC_PAD * nr + (nr << 20);
                // a marker needs its next byte below scan_len
                const uint32_t mk = x.mark & (rem - 1 >= 16 ? 0xFFFFu : (1u << (rem - 1)) - 1);
                if (mk) atomicMin((unsigned long long*)&S[img].end, (unsigned long long)(base + __builtin_ctz(mk)));
            }
        }
        cnt[u] = c;
    }
#endif
    // workgroup sums: wave reductions, then the four wave totals (a tile's
    // bytes < 2^20, its markers < 2^12)
#pragma unroll
    for (int u = 0; u < U; u++) {
        uint32_t c = cnt[u];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) sh[u][w] = c;
    }
    __syncthreads();
    if (threadIdx.x < U) {
        const int u = threadIdx.x;
        const int64_t tile = tile0 + u;
        if (tile < d.ntiles) {
            const uint32_t c = sh[u][0] + sh[u][1] + sh[u][2] + sh[u][3];
            ((ICX_GLOBAL uint32_t*)d.tile_cnt)[tile] = c & 0xFFFFFu;
            ((ICX_GLOBAL uint32_t*)d.tile_rst)[tile] = c >> 20;
        }
    }
}

// One workgroup per image: tile offsets, stream length, subsequence count, tail pad.
__global__ void __launch_bounds__(1024) k_unstuff_scan(const DecDesc* D, DecState* S, const int32_t* ids,
                                                       uint32_t sub_bits)
{
    __shared__ uint32_t sh[24];
    __shared__ uint32_t te_cnt[2];
    __shared__ int64_t s_end;
    __shared__ int s_fake;
    const int img = ids[blockIdx.x];
    const DecDesc& d = D[img];
    DecState& st = S[img];
    // A file that ends in 0xFF bytes inside the scan (cut after an FF of an
    // FF 00 pair, or in fill bytes): the JDK's source manager appends a fake
    // EOI, so those FFs start a marker and are no data - k_unstuff_count,
    // which needs a marker's next byte, kept the last one.  The terminating
    // marker moves to the start of that FF run.
    if (threadIdx.x == 0) {
        int64_t e = st.end;
        int fake = 0;
        if (e >= d.scan_len && d.scan_len > 0 && d.scan[d.scan_len - 1] == 0xFF) {
            e = d.scan_len - 1;
            while (e > 0 && d.scan[e - 1] == 0xFF) e--;
            st.end = e;
            fake = 1;
        }
        s_end = e;
        s_fake = fake;
    }
    __syncthreads();
    // k_unstuff_count counted every tile up to scan_len: the tile holding the
    // terminating marker is recounted below it (4 bytes per thread), the
    // tiles after it count nothing
    const int64_t end = s_end;
    const int64_t te = end / DEC_TILE;
    if (te < d.ntiles) {
        uint32_t nb = 0, nr = 0;
#pragma unroll
        for (int k = 0; k < DEC_TILE / 1024; k++) {
            const int64_t i = te * DEC_TILE + threadIdx.x * (DEC_TILE / 1024) + k;
            if (i < end) {
                int rst;
                nb += (uint32_t)dec_unstuff_rule(i > 0 ? d.scan[i - 1] : 0, d.scan[i],
                                                 i + 1 < d.scan_len ? d.scan[i + 1] : 0, &rst);
                nr += (uint32_t)rst;
            }
        }
        uint32_t tb, tr;
        block_exscan<1024>(nb, sh, tb);
        block_exscan<1024>(nr, sh, tr);
        if (threadIdx.x == 0) {
            te_cnt[0] = tb;
            te_cnt[1] = tr;
        }
        __syncthreads();
    }
    uint32_t carry_b = 0, carry_r = 0;
    for (int t0 = 0; t0 < d.ntiles; t0 += 1024) {
        const int t = t0 + threadIdx.x;
        uint32_t b = t < d.ntiles ? d.tile_cnt[t] : 0, r = t < d.ntiles ? d.tile_rst[t] : 0;
        if (t == te) {
            b = te_cnt[0];
            r = te_cnt[1];
        } else if (t > te) {
            b = r = 0;
        }
        uint32_t sb, sr;
        const uint32_t eb = block_exscan<1024>(b, sh, sb);
        const uint32_t er = block_exscan<1024>(r, sh, sr);
        if (t < d.ntiles) {
            d.tile_cnt[t] = carry_b + eb;
            d.tile_rst[t] = carry_r + er;
        }
        carry_b += sb;
        carry_r += sr;
    }
    const uint32_t len = carry_b;
    const bool fits = (int64_t)len + DEC_TAIL + 8 <= d.ent_cap;  // more RSTn markers than intervals: corrupt
    if (fits)
        for (int k = threadIdx.x; k < DEC_TAIL + 8; k += blockDim.x) d.ent[len + k] = 0xFF;
    if (threadIdx.x == 0) {
        if (!fits) st.status = 6;
        // the scan ends at a marker other than EOI: jpeg_finish_decompress
        // reads the markers after it (the JDK reader throws on a bad one), a
        // walk icx_seqdecode.cpp's route does - never the clean case's
        if (!s_fake && end + 1 < d.scan_len && d.scan[end + 1] != 0xD9) st.status = 6;
        st.ent_len = len;
        st.nseg = carry_r + 1 <= (uint32_t)d.nseg_max ? carry_r + 1 : (uint32_t)d.nseg_max;
        if (carry_r + 1 > (uint32_t)d.nseg_max) st.status = 6;
        uint32_t nsub = (uint32_t)(((uint64_t)len * 8 + sub_bits - 1) / sub_bits);
        if (nsub > (uint32_t)d.nsub_max) {
            nsub = d.nsub_max;
            st.status = 6;
        }
        st.nsub = nsub;
        d.seg[0] = 0;
    }
}

// Compact DEC_SCATTER_TILES consecutive tiles (all their loads issued
// first), one after the other: each thread applies the unstuffing rule to its
// 16 bytes (fully unrolled, no dynamic register indexing) and places its
// output bytes at its workgroup-local offset in a zeroed LDS copy of the
// tile's output - a thread without 0xFF bytes as four shifted dwords (the two
// partial ones ORed in), the others byte by byte - and the workgroup then
// stores the tile's output as aligned dwords (funnel-shifted out of LDS), the
// unaligned head and tail bytes by single lanes.
#ifndef ICX_SCATTER_SCAN1
#define ICX_SCATTER_SCAN1 1  // unstuffing 6.38 -> 6.23 ms per 1000 frames (ab_r5au_dec_scatter_scan1.txt)
#endif
#ifndef ICX_SCATTER_COMPACT
#define ICX_SCATTER_COMPACT 1  // with 4 tiles per workgroup: unstuffing 7.1 -> 6.35 ms per 1000 frames
#endif
__global__ void __launch_bounds__(256) k_unstuff_scatter(const DecDesc* D, const DecState* S, Plan p)
{
    constexpr int U = DEC_SCATTER_TILES;
    __shared__ uint32_t sh[8];
    __shared__ __attribute__((aligned(16))) uint32_t bufw[(DEC_TILE / 2 * DEC_PAD + 64) / 4];  // worst case: an RSTn marker every 2 bytes
    uint8_t* const buf = (uint8_t*)bufw;
    int slot;
    int64_t item;
    if (!plan_slot(p, slot, item)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    const int64_t end = S[img].end, len = d.scan_len;
    const int64_t tile0 = item * U;
    if (tile0 * DEC_TILE >= end) return;  // workgroup-uniform: nothing of these tiles is data
    Scan16 q[U];
    int prev[U];
#pragma unroll
    for (int u = 0; u < U; u++) {  // bases past the scan load its last chunk and place nothing
        const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
        const int64_t bc = base < len ? base : len - 1;
        q[u] = scan16(d.scan, len, bc);
        prev[u] = ((const ICX_GLOBAL uint8_t*)d.scan)[bc > 0 ? bc - 1 : 0];
    }
#if ICX_SCATTER_COMPACT
    // the byte-class masks of the chunks that need them (a 0xFF among or
    // before their bytes, or `end` inside them), compacted into full lanes as
    // in k_unstuff_count - over the dead tile buffer (the first barrier of
    // the first tile's scan orders these accesses before its zeroing); the
    // masks go back to their chunks' lanes through the same LDS
    bool pln[U];
    uint32_t km[U];  // keep | rst << 16 of a chunk that is not plain
    {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint4* const cv = (uint4*)bufw + w * 64;
        uint32_t* const cm = bufw + 4 * 256 + w * 64;
        static_assert(sizeof(bufw) >= 5 * 256 * 4, "staging fits the tile buffer");
        bool spc[U];
        uint32_t nsp = 0, ord[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
            pln[u] = base + 16 <= end && !any_ff(q[u].v, base > 0 ? prev[u] : 0);
            spc[u] = base < end && !pln[u];
            km[u] = 0;
            const uint64_t m = __ballot(spc[u]);
            ord[u] = nsp + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            nsp += (uint32_t)__popcll(m);
        }
        for (uint32_t r0 = 0; r0 < nsp; r0 += 64) {  // wave-uniform
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (spc[u] && ord[u] >= r0 && ord[u] < r0 + 64) {
                    const int64_t base = (tile0 + u) * DEC_TILE + threadIdx.x * 16;
                    const uint32_t pv = base > 0 ? (uint32_t)prev[u] : 0u;
                    cv[ord[u] - r0] = q[u].v;
                    cm[ord[u] - r0] = pv | (uint32_t)q[u].next << 8 | (uint32_t)u << 16 | threadIdx.x << 20;
                }
            }
            __builtin_amdgcn_wave_barrier();  // (a wave's LDS accesses complete in order)
            if (r0 + lane < nsp) {
                const uint4 v = cv[lane];
                const uint32_t mt = cm[lane];
                const int64_t base = (tile0 + ((mt >> 16) & 15)) * DEC_TILE + (int64_t)(mt >> 20) * 16;
                const Unstuff16 x = unstuff16(classify16(v), (int)(mt & 255), (int)((mt >> 8) & 255));
                const int64_t rem = end - base;  // bytes from `end` on drop out
                const uint32_t valid = rem >= 16 ? 0xFFFFu : (1u << rem) - 1;
                cm[lane] = (x.keep & valid) | (x.rst & valid) << 16;
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int u = 0; u < U; u++)
                if (spc[u] && ord[u] >= r0 && ord[u] < r0 + 64) km[u] = cm[ord[u] - r0];
            __builtin_amdgcn_wave_barrier();  // the reads before the next round's writes
        }
    }
#endif
#if ICX_SCATTER_SCAN1
    // The byte and marker offsets of all U tiles in one workgroup scan (one
    // barrier for the U wave totals instead of three per tile), and the tiles'
    // global offsets loaded up front rather than after each tile's scan.
    __shared__ uint32_t shu[U][4];
    uint32_t exu[U], totu[U], toffu[U], trstu[U];
    {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t xin[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t tile = tile0 + u;
            const int64_t tl = tile < d.ntiles ? tile : d.ntiles - 1;
            toffu[u] = d.tile_cnt[tl];
            trstu[u] = d.tile_rst[tl];
            const int64_t base = tile * DEC_TILE + threadIdx.x * 16;
            uint32_t nb = 0, nr = 0;
            if (base < end) {
#if ICX_SCATTER_COMPACT
                nr = (uint32_t)__popc(km[u] >> 16);
                nb = pln[u] ? 16u : (uint32_t)__popc(km[u] & 0xFFFFu) + DEC_PAD * nr;
#endif
            }
            xv[u] = nb | (nr << 20);
            uint32_t x = xv[u];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            xin[u] = x;
            if (lane == 63) shu[u][w] = x;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t before = 0, all = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t s4 = shu[u][k];
                before += k < w ? s4 : 0u;
                all += s4;
            }
            exu[u] = xin[u] - xv[u] + before;
            totu[u] = all;
        }
    }
    static_assert(ICX_SCATTER_COMPACT, "the one-pass scan takes the compacted masks");
#endif
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t tile = tile0 + u;
        // workgroup-uniform; the scan's first barrier also orders the previous
        // tile's buffer reads before this tile's zeroing
        if (tile * DEC_TILE >= end) break;
        const int64_t base = tile * DEC_TILE + threadIdx.x * 16;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        bool plain = false;  // 16 data bytes, no 0xFF among them or before them
        uint32_t keep = 0, rstm = 0;
        if (base < end) {
            v = q[u].v;
#if ICX_SCATTER_COMPACT
            plain = pln[u];
            keep = km[u] & 0xFFFFu;
            rstm = km[u] >> 16;
#else
            const int prev_b = base > 0 ? prev[u] : 0;
            plain = base + 16 <= end && !any_ff(v, prev_b);
            if (!plain) {  // the rule over the 16 bytes as masks (bytes from `end` on drop out)
                const Unstuff16 x = unstuff16(classify16(v), prev_b, q[u].next);
                const int64_t rem = end - base;
                const uint32_t valid = rem >= 16 ? 0xFFFFu : (1u << rem) - 1;
                keep = x.keep & valid;
                rstm = x.rst & valid;
            }
#endif
        }
        const uint32_t nr = (uint32_t)__popc(rstm);
        const uint32_t nb = plain ? 16u : (uint32_t)__popc(keep) + DEC_PAD * nr;
#if ICX_SCATTER_SCAN1
        const uint32_t tot = totu[u], ex = exu[u];
        if (u > 0) __syncthreads();  // the previous tile's buffer reads before this tile's zeroing
        const uint32_t tb = tot & 0xFFFFFu;
        uint32_t ob = ex & 0xFFFFFu;
        uint32_t orr = (ex >> 20) + trstu[u];
        const uint32_t tile_off = toffu[u];
#else
        uint32_t tot;  // one scan of bytes (bits 0..19) and RSTn markers (<< 20)
        const uint32_t ex = block_exscan<256>(nb | (nr << 20), sh, tot);
        const uint32_t tb = tot & 0xFFFFFu;
        uint32_t ob = ex & 0xFFFFFu;
        uint32_t orr = (ex >> 20) + d.tile_rst[tile];
        const uint32_t tile_off = d.tile_cnt[tile];
#endif
        for (uint32_t k = threadIdx.x; k < (tb + 7) / 4; k += 256) bufw[k] = 0;
        __syncthreads();
        if (plain) {
            const uint32_t s8 = (ob & 3) * 8;
            uint32_t* wp = bufw + (ob >> 2);
            if (s8 == 0) {
                wp[0] = v.x; wp[1] = v.y; wp[2] = v.z; wp[3] = v.w;
            } else {
                atomicOr(wp, v.x << s8);
                wp[1] = (v.x >> (32 - s8)) | (v.y << s8);
                wp[2] = (v.y >> (32 - s8)) | (v.z << s8);
                wp[3] = (v.z >> (32 - s8)) | (v.w << s8);
                atomicOr(wp + 4, v.w >> (32 - s8));
            }
        } else if (nr == 0 && nb > 0) {
            // drop the bytes outside `keep` (highest first, so lower positions stay
            // put: usually one stuffed zero), then OR the nb bytes in at ob
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
            uint32_t drop = ~keep & 0xFFFFu;
            while (drop) {
                const int k = 31 - __builtin_clz(drop);
                drop &= ~(1u << k);
                const int q = k >> 2;
                const uint32_t low = (1u << (8 * (k & 3))) - 1u;  // bytes of dword q below k
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t up = j < 3 ? w[j + 1] << 24 : 0u;
                    if (j > q) w[j] = (w[j] >> 8) | up;
                    else if (j == q) w[j] = (w[j] & low) | ((w[j] >> 8) & ~low) | up;
                }
            }
            const uint32_t s8 = (ob & 3) * 8;
            uint32_t* wp = bufw + (ob >> 2);
            atomicOr(wp, w[0] << s8);
#pragma unroll
            for (int j = 1; j < 4; j++) atomicOr(wp + j, (w[j] << s8) | (s8 ? w[j - 1] >> (32 - s8) : 0u));
            if (s8) atomicOr(wp + 4, w[3] >> (32 - s8));
        } else if (nr > 0) {  // RSTn codes (restart intervals): byte by byte
            const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                if ((rstm >> k) & 1) {
                    // marker orr must be RST(orr mod 8): another number makes
                    // jdmarker.c resynchronise (jpeg_resync_to_restart), which
                    // the walks do not restate - the host route does
                    if (((vw[k >> 2] >> (8 * (k & 3))) & 7) != (orr & 7))
                        atomicOr(&((DecState*)S)[img].status, 6);
                    for (int q = 0; q < DEC_PAD; q++) buf[ob + q] = 0xFF;
                    ob += DEC_PAD;
                    if (orr + 1 < (uint32_t)d.nseg_max) ((ICX_GLOBAL uint32_t*)d.seg)[orr + 1] = tile_off + ob;
                    orr++;
                } else if ((keep >> k) & 1) {
                    buf[ob++] = (uint8_t)(vw[k >> 2] >> (8 * (k & 3)));
                }
            }
        }
        __syncthreads();
        // tile output = global bytes [tile_off, tile_off + tb)
        const uint32_t head = min((4u - (tile_off & 3u)) & 3u, tb);
        ICX_GLOBAL uint8_t* const ent = (ICX_GLOBAL uint8_t*)d.ent;
        if (threadIdx.x < head && (int64_t)(tile_off + threadIdx.x) < d.ent_cap)
            ent[tile_off + threadIdx.x] = buf[threadIdx.x];
        const uint32_t nw = (tb - head) >> 2;         // whole aligned dwords
        const uint32_t sh8 = head;                    // local byte of the first dword: head + 4k
        ICX_GLOBAL uint32_t* const dstw = (ICX_GLOBAL uint32_t*)(ent + tile_off + head);  // 4-byte aligned
        const int64_t cap_w = (d.ent_cap - (int64_t)(tile_off + head)) >> 2;
        for (uint32_t k = threadIdx.x; k < nw; k += 256) {
            const uint32_t lb = head + 4 * k;
            const uint32_t val = __builtin_amdgcn_alignbyte(bufw[(lb >> 2) + 1], bufw[lb >> 2], sh8);
            if ((int64_t)k < cap_w) dstw[k] = val;
        }
        const uint32_t t0 = head + 4 * nw;
        if (threadIdx.x < tb - t0 && (int64_t)(tile_off + t0 + threadIdx.x) < d.ent_cap)
            ent[tile_off + t0 + threadIdx.x] = buf[t0 + threadIdx.x];
    }
}

// ------------------------------------------------------------ entropy decode
// Initial entry-state estimates: subsequence j starts decoding `warm` bits
// before its first bit from a guessed state (block 0, DC next) and takes the
// state at which that walk reaches j * sub_bits.  A Huffman decoder
// resynchronises within a few hundred bits on typical content, so most
// estimates are already the fixed point and the first sync launch confirms
// them; the rest are repaired by the relaxation like any other guess.
__device__ __forceinline__ void load_tables(const DecTab* T, DecLean* L);
__device__ __forceinline__ void load_first_levels(const DecTab* T, uint32_t (*L1)[1 << DEC_LUT_BITS]);
__device__ __forceinline__ uint32_t selector(const DecTab* T);

// The state-only walks (k_dec_init, k_dec_sync) keep both levels of the
// image's tables in LDS (16 KiB at 9 bits with 8 second-level tables);
// ICX_DEC_SYNC_SPLIT=1: only the first levels there, the second levels of the
// long codes through the scalar cache as in the write pass (SplitLean) - 1-3 %
// slower (ab_r5d_dec_lut.txt).
#ifndef ICX_DEC_SYNC_SPLIT
#define ICX_DEC_SYNC_SPLIT 0
#endif
#if ICX_DEC_SYNC_SPLIT
#define DEC_WALK_TABLES                                                                   \
    __shared__ __attribute__((aligned(16))) uint32_t L1[4][1 << DEC_LUT_BITS];
#define DEC_WALK_LOAD(T) load_first_levels(T, L1)
#define DEC_WALK_H(T) SplitLean{(const uint32_t (*)[1 << DEC_LUT_BITS])L1, (const ICX_GLOBAL DecLean*)(T)->lean}
#else
#define DEC_WALK_TABLES __shared__ __attribute__((aligned(16))) DecLean L[4];
#define DEC_WALK_LOAD(T) load_tables(T, L)
#define DEC_WALK_H(T) ((const DecLean*)L)
#endif

__global__ void __launch_bounds__(DEC_SYNC_NT) k_dec_init(const DecDesc* D, const DecState* S, Plan p, uint32_t sub_bits,
                                                  uint32_t warm)
{
    DEC_WALK_TABLES
    int slot;
    int64_t wg;
    if (!plan_slot(p, slot, wg)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    const DecState& st = S[img];
    const int64_t j = wg * DEC_SYNC_NT + threadIdx.x;
    const bool live = st.status == 0 && wg * DEC_SYNC_NT < (int64_t)st.nsub;
    if (live) DEC_WALK_LOAD(d.tab);
    if (j > d.nsub_max) return;
    const uint32_t start = (uint32_t)j * sub_bits;
    uint64_t e = dec_pack(start, 0, 0);
    if (live && j > 0 && j < st.nsub && warm > 0) {
        const uint32_t from = start > warm ? start - warm : 0;
        uint32_t n;
        e = dec_lean_walk(d, DEC_WALK_H(d.tab), d.tab->slow, selector(d.tab), (const uint32_t*)d.ent, d.seg,
                          st.nseg, st.ent_len * 8, dec_pack(from, 0, 0), start, n);
    }
    d.est[j] = e;
}

// Stage the image's distinct Huffman tables, as state transitions (DecLean),
// in LDS (all threads participate).
__device__ __forceinline__ void load_tables(const DecTab* T, DecLean* L)
{
    const uint4* src = (const uint4*)T->lean;
    uint4* dst = (uint4*)L;
    const int n = (int)(sizeof(DecLean) * T->ntab / 16);
    for (int k = threadIdx.x; k < n; k += blockDim.x) dst[k] = src[k];
    __syncthreads();
}

// The first levels (10-bit look-ups) of the image's distinct tables, in LDS.
__device__ __forceinline__ void load_first_levels(const DecTab* T, uint32_t (*L1)[1 << DEC_LUT_BITS])
{
    constexpr int per = (int)(sizeof(L1[0]) / 16);
    const int n = (int)T->ntab * per;
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
        const int t = k / per, o = k % per;
        ((uint4*)L1[t])[o] = ((const uint4*)T->lean[t].lut)[o];
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t selector(const DecTab* T)
{
    uint32_t s = 0;
    for (int k = 0; k < 8; k++) s |= (uint32_t)(T->sel[k] & 3) << (4 * k);
    return s;
}

// One relaxation launch.  Launch 0 walks every subsequence; launch r > 0 walks
// the worklist launch r-1 built (entry k of workgroup w: wl[r & 1][DEC_SYNC_NT w + k]),
// so the few subsequences still moving fill whole waves.  A thread whose exit
// differs from the stored next entry stores it and appends j + 1 to the next
// worklist (only thread j writes E[j+1], so entries are unique per launch).
// Launch 0 records each walk's checkpoints; a re-walk compares against them
// in place (CkInPlace) and stops where it meets its previous walk (dec_sync_walk).
#ifndef ICX_DEC_AGG
#define ICX_DEC_AGG 0  // k_dec_sync: wave-aggregated worklist / change-count atomics (+-0: few lanes change)
#endif
// Issue priority of the relaxation's later launches: their few long re-walks
// share SIMDs with the settled images' write and colour passes (aux streams),
// and a re-walk is a serial chain of table look-ups, so its wave goes first
// when both are ready (s_setprio; 2: the first launch too).  Decode per call,
// two interleaved rounds (profiles/r6/ab/ab_r6_sync_prio.txt): 200 frames
// 17.10 -> 16.80 ms (2: 16.84), 64 and 1000 frames +-0.
#ifndef ICX_DEC_SYNC_PRIO
#define ICX_DEC_SYNC_PRIO 1
#endif
template <bool FIRST>
__global__ void __launch_bounds__(DEC_SYNC_NT) k_dec_sync(const DecDesc* D, const DecState* S, Plan p, uint32_t sub_bits,
                                                  int iter, int nimg, uint32_t* changed)
{
    DEC_WALK_TABLES
    if (ICX_DEC_SYNC_PRIO > (FIRST ? 1 : 0)) __builtin_amdgcn_s_setprio(3);
    int slot;
    int64_t wg;
    if (!plan_slot(p, slot, wg)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    const DecState& st = S[img];
    if (st.status) return;
    const int64_t k = wg * DEC_SYNC_NT + threadIdx.x;
    const uint32_t n = FIRST ? st.nsub : d.wl_cnt[(int64_t)(iter - 1) * nimg + img];
    if (wg * DEC_SYNC_NT >= (int64_t)n) return;
    DEC_WALK_LOAD(d.tab);
    if (k >= n) return;
    const uint32_t j = FIRST ? (uint32_t)k : d.wl[iter & 1][k];
    if (j >= st.nsub) return;
    const uint64_t e = __hip_atomic_load(&d.est[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int nck = dec_ck_slots(sub_bits);
    ICX_GLOBAL uint64_t* ckg = (ICX_GLOBAL uint64_t*)d.ck + (int64_t)j * DEC_CK_MAX;
    uint32_t nb;
    bool early;
    uint64_t x;
    if (FIRST) {
        CkRecord<ICX_GLOBAL uint64_t*> ck{ckg, nck};
        x = dec_sync_walk(d, DEC_WALK_H(d.tab), d.tab->slow, selector(d.tab), (const uint32_t*)d.ent, d.seg, st.nseg,
                          st.ent_len * 8, e, j * sub_bits, sub_bits, nb, early, ck);
    } else {
        CkInPlace<ICX_GLOBAL uint64_t*> ck{ckg, nck, d.ncnt[j], nck > 0 ? ckg[0] : DEC_CK_NONE};
        x = dec_sync_walk(d, DEC_WALK_H(d.tab), d.tab->slow, selector(d.tab), (const uint32_t*)d.ent, d.seg, st.nseg,
                          st.ent_len * 8, e, j * sub_bits, sub_bits, nb, early, ck);
    }
    d.ncnt[j] = nb;
    if (early) return;  // met the previous walk: same exit as before
    const uint64_t old = __hip_atomic_load(&d.est[j + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (x != old) {
        __hip_atomic_store(&d.est[j + 1], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if ICX_DEC_AGG
        // one device-scope atomic per wave for each counter (the lanes of a
        // workgroup share the image): a worklist slot per changed lane from
        // the wave's base by its rank among the changed lanes - device
        // atomics are slow memory operations the wave's next loads queue
        // behind (the FDCT's per-wave atomics cost 5.7 %, profiles/NOTES.md §9)
        const uint64_t act = __ballot(1);
        const uint64_t mw = __ballot(j + 1 < st.nsub);
        const int lane = threadIdx.x & 63, leader = __ffsll((unsigned long long)act) - 1;
        uint32_t base = 0;
        if (lane == leader) {
            if (mw) base = atomicAdd(&d.wl_cnt[(int64_t)iter * nimg + img], (uint32_t)__popcll(mw));
            atomicAdd(changed, (uint32_t)__popcll(act));
        }
        base = (uint32_t)__shfl((int)base, leader);
        if (j + 1 < st.nsub) d.wl[(iter + 1) & 1][base + (uint32_t)__popcll(mw & ((1ull << lane) - 1))] = j + 1;
#else
        if (j + 1 < st.nsub) {
            const uint32_t pos = atomicAdd(&d.wl_cnt[(int64_t)iter * nimg + img], 1u);
            d.wl[(iter + 1) & 1][pos] = j + 1;
        }
        atomicAdd(changed, 1u);
#endif
    }
}

// One workgroup per image: exclusive scan of blocks per subsequence.
__global__ void __launch_bounds__(1024) k_dec_offsets(const DecDesc* D, DecState* S, const int32_t* ids)
{
    __shared__ uint32_t sh[24];
    const int img = ids[blockIdx.x];
    const DecDesc& d = D[img];
    DecState& st = S[img];
    const int n = (int)st.nsub;
    uint32_t carry = 0;
    for (int t0 = 0; t0 < n; t0 += 1024) {
        const int t = t0 + threadIdx.x;
        uint32_t tot;
        const uint32_t e = block_exscan<1024>(t < n ? d.ncnt[t] : 0u, sh, tot);
        if (t < n) d.boff[t] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        st.total_blocks = carry;
        if ((int64_t)carry != d.nblocks) st.status = 6;
    }
}

// Per-thread block assembly slot in LDS: 64 int16 (32 dwords) in zig-zag
// order, the DC difference at [0].  Int16 z of lane l's slot sits at
// (z ^ (l & 62)): lanes storing the same zig-zag position (they walk in near
// lockstep) and the 32 lanes copying one slot hit 64 (32) distinct banks
// without a pad dword, so 256 slots take 32 KiB and, with the 8 KiB of
// first-level Huffman tables, a workgroup 40 KiB: four per CU.
constexpr int SLOT_DW = 32;
#ifndef ICX_DEC_WRITE_UNROLL2
#define ICX_DEC_WRITE_UNROLL2 1  // with a 9-word write window: -2.1 % (profiles/r4/ab_r4zd_dec_unroll.txt)
#endif
#ifndef ICX_DEC_FLUSH2
#define ICX_DEC_FLUSH2 0
#endif
#ifndef ICX_DEC_DC_LANE
#define ICX_DEC_DC_LANE 1  // 87.8 vs 88.3 ms per 1000-frame decode (profiles/r4/ab_r4o_dec_win.txt)
#endif
// Flush addressing in scalar registers (round 6): the finished block's index
// is one readlane (a 32-bit block index), its store a global_store with the
// block's 64-bit address in SGPRs and a 32-bit lane offset (lane 32's: d.dc's
// entry, which follows the coefficients in the same allocation), the slot
// reads one v_xad each.  The write pass is VALU-issue-bound at four waves per
// SIMD (five: no faster, three: +18 %, profiles/r6/ab/ab_r6_write_occupancy.txt),
// and the flush cost ~18 VALU per finished block.
#ifndef ICX_DEC_FLUSH_SADDR
#define ICX_DEC_FLUSH_SADDR 1
#endif

// A lane that finishes an owned block only records its index, and the wave
// then copies every finished slot together (below), permuting to natural
// order on the way.
struct PendSink {
    uint8_t* slot;  // this lane's slot
    uint32_t sw;    // lane & 62
#if ICX_DEC_PEND32
    int64_t base;   // the piece's first block
    int32_t pend;   // block waiting for the wave flush, from base; -1 = none
    __device__ __forceinline__ void flush_if(bool c, int64_t bi) { pend = c ? (int32_t)(bi - base) : pend; }
    __device__ __forceinline__ int64_t block_of(int l) const
    {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)base, l);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)base >> 32), l);
        return (int64_t)(((uint64_t)hi << 32) | lo) + (int64_t)__builtin_amdgcn_readlane((uint32_t)pend, l);
    }
#else
    int64_t pend;   // block waiting for the wave flush, -1 = none
    __device__ __forceinline__ void flush_if(bool c, int64_t bi) { pend = c ? bi : pend; }
    __device__ __forceinline__ int64_t block_of(int l) const
    {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)pend, l);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)pend >> 32), l);
        return (int64_t)(((uint64_t)hi << 32) | lo);
    }
#endif
    __device__ __forceinline__ void put(int z, int v) { *(int16_t*)(slot + ((z ^ sw) << 1)) = (int16_t)v; }
    // z2 = 2 z (ICX_DEC_PUT2): the entry's LDS byte address is sa ^ z2, sa =
    // the slot's LDS address | 2 sw (the slot is 128-B aligned)
    uint32_t sa;
    __device__ __forceinline__ void put2(int z2, int v)
    {
        *(__attribute__((address_space(3))) int16_t*)(size_t)(sa ^ (uint32_t)z2) = (int16_t)v;
    }
};

// Write pass.  The walk runs in a wave-uniform loop, one symbol per lane per
// iteration; after each step the wave tops up the bit windows if any lane runs
// low (DecReader), then ballots the lanes that finished a block and copies
// each of those 128-byte slots with 32 lanes (one coalesced dword store each,
// natural order: coefficient pair 2l, 2l+1 read from its zig-zag positions),
// zeroing it behind (lane 32 also stores the DC difference into d.dc; with
// ICX_DEC_FLUSH_SADDR the addresses are scalar and a block costs 5 VALU).  The
// block stores are the only vector-memory traffic between top-ups, so no
// symbol waits for them.  A per-lane flush costs every lane of the wave its
// copy whenever any lane finishes a block, which on q95 content is most
// iterations (measured: write pass +28 %, profiles/r6/ab/ab_r6_flush_lane.txt).  Only the first levels of the
// Huffman tables are in LDS (SplitHuff): the second levels of the few codes
// longer than 10 bits are read from the image's tables in global memory.
__global__ void __launch_bounds__(DEC_WRITE_NT) k_dec_write(const DecDesc* D, DecState* S, Plan p, uint32_t sub_bits)
{
    __shared__ __attribute__((aligned(16))) uint32_t L1[4][1 << DEC_LUT_BITS];
    __shared__ __attribute__((aligned(128))) uint32_t slots[DEC_WRITE_NT * SLOT_DW];  // 128-B slots on 128-B boundaries (the flush ORs offsets in)
    int slot;
    int64_t wg;
    if (!plan_slot(p, slot, wg)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    const DecState& st = S[img];
    if (st.status) return;
    // thread = one piece of a subsequence (dec_piece): the pieces of one
    // subsequence sit in neighbouring lanes, so a wave reads a contiguous
    // stretch of the stream
    const int np = dec_pieces(sub_bits);
    const int64_t t = wg * DEC_WRITE_NT + threadIdx.x;
    if (wg * DEC_WRITE_NT >= (int64_t)st.nsub * np) return;
    const int64_t j = t / np;
    const int lane = threadIdx.x & 63;
    uint32_t* wave_slots = slots + (threadIdx.x - lane) * SLOT_DW;
    uint32_t* mys = slots + threadIdx.x * SLOT_DW;
    for (int k = 0; k < 32; k++) mys[k] = 0;
    {  // first levels of the image's distinct tables
        const int n = (int)(d.tab->ntab * sizeof(L1[0]) / 16);
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const int t = k / (int)(sizeof(L1[0]) / 16), o = k % (int)(sizeof(L1[0]) / 16);
            ((uint4*)L1[t])[o] = ((const uint4*)d.tab->lean[t].lut)[o];
        }
        __syncthreads();
    }
    DecPiece pc{0, 0, 0, false};
    if (j < st.nsub)
        pc = dec_piece((const ICX_GLOBAL uint64_t*)d.est, (const ICX_GLOBAL uint64_t*)d.ck,
                       (const ICX_GLOBAL uint32_t*)d.boff, (uint32_t)j, (int)(t - j * np), sub_bits);
    const uint32_t stop = pc.stop;
    const SplitLean H{(const uint32_t (*)[1 << DEC_LUT_BITS])L1, (const ICX_GLOBAL DecLean*)d.tab->lean};
    DecLeanWriter<SplitLean> w = dec_lean_writer(d, H, d.tab->slow, selector(d.tab), (const uint32_t*)d.ent, d.seg,
                                                 st.nseg, st.ent_len * 8, pc.blk);
    bool run = false, started = false;
    if (pc.have) {
        run = !(dec_pos(pc.e) >= stop && (pc.e & 63) == 0);
        if (run) {
            w.start(pc.e);
            started = true;
            run = w.running(stop);
        }
    }
#if ICX_DEC_PEND32
    PendSink sk{(uint8_t*)mys, (uint32_t)(lane & 62), pc.blk, -1};
#else
    PendSink sk{(uint8_t*)mys, (uint32_t)(lane & 62), -1};
#endif
    sk.sa = (uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t*)mys | ((uint32_t)(lane & 62) << 1);
    ICX_GLOBAL uint32_t* coefs32 = (ICX_GLOBAL uint32_t*)d.coefs;  // global_store: vmcnt only, not lgkmcnt
    ICX_GLOBAL int32_t* dcs = (ICX_GLOBAL int32_t*)d.dc;
    const int zl = dec_zz((2 * lane) & 63), zh = dec_zz((2 * lane + 1) & 63);  // this lane's flush pair (lane % 32)
#if ICX_DEC_FLUSH_SADDR
    // d.dc relative to d.coefs: lane 32's store offset is rel - 124 bi (>= 0
    // while rel >= 128 nblocks; < 2^32 while rel is); otherwise the general path
    const uint64_t coefs_s = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)(uintptr_t)coefs32 >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)coefs32);  // (int: no sign extension)
    const uint64_t rel = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)(uintptr_t)dcs >> 32)) << 32 |
                          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dcs)) -
                         coefs_s;
    const bool saddr = __builtin_amdgcn_readfirstlane(rel >= (uint64_t)d.nblocks * 128u && rel < (1ull << 32));  // wave-uniform
    const uint32_t zl2 = (uint32_t)zl << 1, zh2 = (uint32_t)zh << 1, lane4 = (uint32_t)(lane & 31) << 2;
    // wave-uniform, in SGPRs: the wave's first slot (LDS byte address) and the
    // coefficient array
    typedef __attribute__((address_space(3))) uint16_t lds16_t;
    typedef uint16_t us2_t __attribute__((ext_vector_type(2)));
    uint32_t offv = lane4;  // store offset: lanes 0..31 their pair, lane 32 (set per block) the DC entry
    typedef __attribute__((address_space(3))) uint32_t lds32_t;
    const uint32_t ws_lds = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds32_t*)wave_slots);

#if ICX_DEC_PEND32
    const uint32_t blk32 = (uint32_t)pc.blk;  // block indices fit 32 bits (nblocks < 2^31)
#endif
#endif
    // copy the wave's finished blocks out of their slots (after every step: a
    // lane's next block reuses its slot)
    auto flush = [&]() {
    uint64_t m = __ballot(sk.pend >= 0);
#if ICX_DEC_FLUSH_SADDR
    if (saddr) {
        // every lane's block index, computed before the lane mask below (the
        // readlane takes it from lanes past 32 too)
#if ICX_DEC_PEND32
        uint32_t mine = blk32 + (uint32_t)sk.pend;
#else
        uint32_t mine = (uint32_t)sk.pend;
#endif
        asm volatile("" : "+v"(mine));  // pinned here, with every lane active (not sunk under the mask)
        if (m && lane <= 32) {
            do {
                const int l = __builtin_ctzll(m);
                m &= ~(1ull << l);  // s_bitset0
                const uint32_t bi = (uint32_t)__builtin_amdgcn_readlane(mine, l);
                // lane l's slot (LDS byte address) and its swizzle, both wave-uniform
                // slot base + swizzle (a 128-B aligned base: + and ^ commute
                // with the 7-bit offsets), then one v_xor per read address
                const uint32_t sw = ws_lds + (uint32_t)l * (SLOT_DW * 4) + ((uint32_t)(l & 62) << 1);
                lds16_t* const pl = (lds16_t*)(size_t)(sw ^ zl2);
                lds16_t* const ph = (lds16_t*)(size_t)(sw ^ zh2);
                us2_t pr;
                pr.x = *pl;
                pr.y = *ph;
                const uint32_t v = __builtin_bit_cast(uint32_t, pr);
                // zeroed behind, at the addresses read (the wave's LDS
                // instructions complete in order: lane 0's zeroes follow lane
                // 32's reads of the same two positions)
                *pl = 0;
                *ph = 0;
                // lanes 0..31: the block's 32 coefficient pairs; lane 32: the pair
                // (DC difference, zig-zag 1) into d.dc - k_dec_dc takes the low half
                ICX_GLOBAL uint8_t* const base = (ICX_GLOBAL uint8_t*)(uintptr_t)(coefs_s + ((uint64_t)bi << 7));
                asm("v_writelane_b32 %0, %1, 32" : "+v"(offv) : "s"((uint32_t)rel - bi * 124u));  // lane 32's offset
                *(ICX_GLOBAL uint32_t*)(base + offv) = v;
            } while (m);
        }
        sk.pend = -1;
        return;
    }
#endif
#if ICX_DEC_FLUSH2
    // two finished blocks per round: lanes 0..31 copy the first, 32..63 the second
    while (m) {
        const int l0 = __builtin_ctzll(m);
        m &= m - 1;
        const int l1 = m ? __builtin_ctzll(m) : l0;
        const bool two = m != 0;
        m &= m - 1;
        const int64_t b0 = sk.block_of(l0), b1 = sk.block_of(l1);
        const bool upper = lane >= 32;
        const int l = upper ? l1 : l0;
        const int64_t bi = upper ? b1 : b0;
        uint32_t* src = wave_slots + l * SLOT_DW;
        if (!upper || two) {
            const int q = lane & 31;
            const uint16_t* s16 = (const uint16_t*)src;
            const int lsw = l & 62;
            const uint32_t v = s16[zl ^ lsw] | ((uint32_t)s16[zh ^ lsw] << 16);
            __builtin_amdgcn_wave_barrier();  // every lane's reads before the zeroing
            src[q] = 0;
            coefs32[bi * 32 + q] = v;
            if (q == 0) dcs[bi] = (int16_t)v;  // the DC difference, also for k_dec_dc's dense reads
        }
    }
#else
    while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const int64_t bi = sk.block_of(l);
        uint32_t* src = wave_slots + l * SLOT_DW;
#if ICX_DEC_DC_LANE
        // lanes 0..31 store the block's 32 coefficient pairs, lane 32 (whose
        // pair also starts at zig-zag 0) its DC difference into d.dc for
        // k_dec_dc's dense reads - one store instruction per block
        if (lane <= 32) {
            const uint16_t* s16 = (const uint16_t*)src;
            const int lsw = l & 62;
            const uint32_t v = s16[zl ^ lsw] | ((uint32_t)s16[zh ^ lsw] << 16);
            __builtin_amdgcn_wave_barrier();  // every lane's reads before the zeroing
            src[lane & 31] = 0;               // (lane 32 zeroes word 0 with lane 0)
            ICX_GLOBAL int32_t* dst = lane < 32 ? (ICX_GLOBAL int32_t*)coefs32 + bi * 32 + lane : dcs + bi;
            *dst = lane < 32 ? (int32_t)v : (int32_t)(int16_t)v;
        }
#else
        if (lane < 32) {
            const uint16_t* s16 = (const uint16_t*)src;
            const int lsw = l & 62;
            const uint32_t v = s16[zl ^ lsw] | ((uint32_t)s16[zh ^ lsw] << 16);
            __builtin_amdgcn_wave_barrier();  // every lane's reads before the zeroing
            src[lane] = 0;
            coefs32[bi * 32 + lane] = v;
            if (lane == 0) dcs[bi] = (int16_t)v;  // the DC difference, also for k_dec_dc's dense reads
        }
#endif
    }
#endif
    sk.pend = -1;
    };
#if ICX_DEC_WRITE_UNROLL2
    // two steps per top-up check: a step consumes at most one window word, so
    // a lane holding >= 1 word at every refill needs the top-up once any holds <= 2
    while (__any(run)) {
        if (run) {
            w.step(sk);
            run = w.running(stop);
        }
        flush();
        if (run) {
            w.step(sk);
            run = w.running(stop);
        }
        if (__any(run && w.R.left() <= 2) && run) w.R.top_up();
        flush();
    }
#else
    while (__any(run)) {
        if (run) {
            w.step(sk);
            run = w.running(stop);
        }
        if (__any(run && w.R.low()) && run && w.R.wants()) w.R.top_up();
        flush();
    }
#endif
    // The settled states are the true decode: an invalid code met on it
    // (outside an interval's padding), a symbol reaching into the padding or
    // an interval of the wrong length is damaged data (jdhuff.c warns,
    // zero-fills and resynchronises there): the caller re-decodes the file
    // with libjpeg's recovery (icx_seqdecode.cpp).
    if (started && (w.bad || w.overran())) atomicOr(&S[img].status, 6);
}

// One workgroup per image: DC values from the differences the write pass left
// in d.dc, in place, per component, the predictor reset at every restart
// interval (jdhuff.c process_restart; jdhuff.c keeps last_dc_val as an int
// and stores the int16 JCOEF).  The image's MCUs go by in tiles of 1024, one
// MCU per thread: its differences (one coalesced row of a tile), their sums
// per component, a segmented scan over the tile (flag = a restart interval
// starts at the MCU) carried from the previous tile, then the values.  (Round
// 4; it was a 32-MCU sequential run per thread in two passes: 8.7 ms per
// 1000 4K frames, profiles/NOTES.md §10.)
struct DcAgg {
    int32_t v[4];  // per component (CMYK / YCCK: four)
    int f;  // a restart interval starts inside the span: what came before does not count
};

__device__ __forceinline__ DcAgg dc_join(const DcAgg& a, const DcAgg& b)  // a before b
{
    DcAgg r;
#pragma unroll
    for (int c = 0; c < 4; c++) r.v[c] = b.f ? b.v[c] : a.v[c] + b.v[c];
    r.f = a.f | b.f;
    return r;
}

template <int NB>
__device__ __forceinline__ void dc_tile(ICX_GLOBAL int32_t* dc, int nb, int ny, int64_t m, bool in, int ri,
                                        DcAgg& carry, DcAgg (*s_w)[16], int t)
{
    const int n = NB > 0 ? NB : nb;
    int32_t d[NB > 0 ? NB : 10];  // T.81: at most 10 blocks per MCU
    DcAgg a{{0, 0, 0, 0}, 0};
    if (in) {
#pragma unroll
        for (int k = 0; k < (NB > 0 ? NB : 10); k++)
            if (k < n) d[k] = (int16_t)dc[m * n + k];  // the write pass may leave zig-zag 1 in the high half
#pragma unroll
        for (int k = 0; k < (NB > 0 ? NB : 10); k++)
            if (k < n) a.v[k < ny ? 0 : k - ny + 1] += d[k];
        a.f = ri > 0 && m % ri == 0;
    }
    // inclusive segmented scan over the wave, then over the 16 waves
    DcAgg x = a;
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        DcAgg y;
#pragma unroll
        for (int c = 0; c < 4; c++) y.v[c] = __shfl_up(x.v[c], o, 64);
        y.f = __shfl_up(x.f, o, 64);
        if (lane >= o) x = dc_join(y, x);
    }
    if (lane == 63) (*s_w)[wv] = x;
    __syncthreads();
    DcAgg pre = carry;  // everything before this wave: the carry, then the earlier waves
    for (int k = 0; k < wv; k++) pre = dc_join(pre, (*s_w)[k]);
    DcAgg total = carry;
    for (int k = 0; k < 16; k++) total = dc_join(total, (*s_w)[k]);
    // this MCU's predictor: everything before it (the carry, the earlier
    // waves, the earlier lanes: the inclusive scan one lane up), or 0 where an
    // interval starts at it
    DcAgg prev;
#pragma unroll
    for (int c = 0; c < 4; c++) prev.v[c] = __shfl_up(x.v[c], 1, 64);
    prev.f = __shfl_up(x.f, 1, 64);
    if (lane == 0) prev = DcAgg{{0, 0, 0, 0}, 0};
    const DcAgg excl = dc_join(pre, prev);
    if (in) {
        int32_t acc[4] = {a.f ? 0 : excl.v[0], a.f ? 0 : excl.v[1], a.f ? 0 : excl.v[2], a.f ? 0 : excl.v[3]};
#pragma unroll
        for (int k = 0; k < (NB > 0 ? NB : 10); k++)
            if (k < n) {
                const int c = k < ny ? 0 : k - ny + 1;
                acc[c] += d[k];
                dc[m * n + k] = (int32_t)(int16_t)acc[c];
            }
    }
    __syncthreads();  // s_w is rewritten by the next tile
    carry = total;
}

template <int NB>
__device__ __forceinline__ void dc_image(const DecDesc& d, DcAgg (*s_w)[16])
{
    const int64_t nmcu = (int64_t)d.mcux * d.mcuy;
    ICX_GLOBAL int32_t* dc = (ICX_GLOBAL int32_t*)d.dc;
    const int nb = d.nbmcu, ri = d.ri, ny = d.nby;
    const int t = threadIdx.x;
    DcAgg carry{{0, 0, 0, 0}, 0};
    for (int64_t m0 = 0; m0 < nmcu; m0 += 1024) {
        const int64_t m = m0 + t;
        dc_tile<NB>(dc, nb, ny, m, m < nmcu, ri, carry, s_w, t);
    }
}

__global__ void __launch_bounds__(1024) k_dec_dc(const DecDesc* D, const DecState* S, const int32_t* ids)
{
    __shared__ DcAgg s_w[16];
    const int img = ids[blockIdx.x];
    const DecDesc& d = D[img];
    if (S[img].status) return;
    switch (d.nbmcu) {  // 4:2:0, 4:2:2, 4:4:4, grey; anything else at run time
        case 6: dc_image<6>(d, &s_w); break;
        case 4: dc_image<4>(d, &s_w); break;
        case 3: dc_image<3>(d, &s_w); break;
        case 1: dc_image<1>(d, &s_w); break;
        default: dc_image<0>(d, &s_w); break;
    }
}

// ------------------------------------------------------------------- IDCT
// Two signed values shifted right by sh and saturated to 0..255, as bytes 0
// and 1 (gfx950 v_ashr_pk_u8_i32: the shift, both clamps and the packing in
// one instruction).
__device__ __forceinline__ uint32_t ashr_pk_u8(int a, int b, int sh)
{
    uint32_t r;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(sh));
    return r;
}
// bytes 0, 1 of lo and of hi as one dword
__device__ __forceinline__ uint32_t pk16(uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); }

#define CONST_BITS 13
#define PASS1_BITS 2
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

// Products of the IDCT: v_mul_i32_i24 (full rate) when the data operand is
// known to fit 24 signed bits - then its low 32 bits equal the 32-bit
// product's - else v_mul_lo_u32 (a quarter-rate instruction).
template <bool M24>
__device__ __forceinline__ int32_t imul(int32_t a, int32_t c)
{
    return M24 ? __mul24(a, c) : a * c;
}

// One 1-D pass of jpeg_idct_islow (jidctint.c, IJG 6b); d[0..7] in place.
// M24: every data operand of a product is a sum of at most four inputs, so
// inputs below 2^21 in magnitude keep them inside 24 bits.
template <int SH, bool M24>
__device__ __forceinline__ void idct8(int32_t* v)
{
    int32_t z2 = v[2], z3 = v[6];
    int32_t z1 = imul<M24>(z2 + z3, 4433);                   // FIX_0_541196100
    const int32_t t2 = z1 + imul<M24>(z3, -15137);           // FIX_1_847759065
    const int32_t t3 = z1 + imul<M24>(z2, 6270);             // FIX_0_765366865
    const int32_t t0 = (v[0] + v[4]) << CONST_BITS;
    const int32_t t1 = (v[0] - v[4]) << CONST_BITS;
    const int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    int32_t o0 = v[7], o1 = v[5], o2 = v[3], o3 = v[1];
    int32_t q1 = o0 + o3, q2 = o1 + o2, q3 = o0 + o2, q4 = o1 + o3;
    const int32_t z5 = imul<M24>(q3 + q4, 9633);             // FIX_1_175875602
    o0 = imul<M24>(o0, 2446); o1 = imul<M24>(o1, 16819); o2 = imul<M24>(o2, 25172); o3 = imul<M24>(o3, 12299);
    q1 = imul<M24>(q1, -7373); q2 = imul<M24>(q2, -20995); q3 = imul<M24>(q3, -16069); q4 = imul<M24>(q4, -3196);
    q3 += z5; q4 += z5;
    o0 += q1 + q3; o1 += q2 + q4; o2 += q2 + q3; o3 += q1 + q4;
    v[0] = DESCALE(t10 + o3, SH);
    v[7] = DESCALE(t10 - o3, SH);
    v[1] = DESCALE(t11 + o2, SH);
    v[6] = DESCALE(t11 - o2, SH);
    v[2] = DESCALE(t12 + o1, SH);
    v[5] = DESCALE(t12 - o1, SH);
    v[3] = DESCALE(t13 + o0, SH);
    v[4] = DESCALE(t13 - o0, SH);
}

// IDCT_range_limit(cinfo)[x & RANGE_MASK] (jdmaster.c prepare_range_limit_table):
// the table maps the low 10 bits, read as a signed value s, to clamp(s + 128)
__device__ __forceinline__ uint32_t idct_limit(int32_t v)
{
    const int s = (int)((uint32_t)v << 22) >> 22;
    const int x = s + 128;
    return (uint32_t)(x < 0 ? 0 : x > 255 ? 255 : x);
}

// jpeg_idct_islow of one block by 8 threads (thread r owns coefficient row r,
// then column r, then output row r); ws = this block's 8 x 9 LDS workspace.
// q = the block's quantised coefficient row r (natural order), dc = its DC
// value, qt = dequantisation row r.  Returns output row r as 8 range-limited
// samples packed in two dwords.  The caller's 8 threads must all reach the
// barriers (real == false: no work).
__device__ __forceinline__ uint2 idct_row_of(const uint4& q, int32_t dc, const uint4& qt, int r, bool real,
                                             int32_t* ws)
{
    int32_t v[8];
    if (real) {
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
        const uint32_t t[4] = {qt.x, qt.y, qt.z, qt.w};
#pragma unroll
        for (int c = 0; c < 8; c++)
            v[c] = (int32_t)(int16_t)(w[c >> 1] >> (16 * (c & 1))) * (int32_t)((t[c >> 1] >> (16 * (c & 1))) & 0xFFFFu);
        if (r == 0) v[0] = dc * (int32_t)(qt.x & 0xFFFFu);
#pragma unroll
        for (int c = 0; c < 8; c++) ws[r * 9 + c] = v[c];
    }
    // pass 1 runs on 24-bit products when every dequantised value of the
    // wave's blocks is below 2^21 in magnitude (a block's 8 threads are lanes
    // of one wave; any real image's are below 2^14); pass 2 always can: its
    // inputs are 32-bit values shifted right by 11, below 2^20
    uint32_t acc = 0;
    if (real) {
#pragma unroll
        for (int c = 0; c < 8; c++) acc |= (uint32_t)(v[c] + (1 << 21));
    }
    const bool m24 = __all(acc < (1u << 22));
    __syncthreads();
    if (real) {  // pass 1: column r
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = ws[k * 9 + r];
        if (m24)
            idct8<CONST_BITS - PASS1_BITS, true>(v);
        else
            idct8<CONST_BITS - PASS1_BITS, false>(v);
#pragma unroll
        for (int k = 0; k < 8; k++) ws[k * 9 + r] = v[k];
    }
    __syncthreads();
    uint32_t lo = 0, hi = 0;
    if (real) {  // pass 2: row r
#pragma unroll
        for (int c = 0; c < 8; c++) v[c] = ws[r * 9 + c];
        idct8<CONST_BITS + PASS1_BITS + 3, true>(v);
        // idct_limit: clamp(sext10(v) + 128), two samples per ashr_pk
        int x[8];
#pragma unroll
        for (int c = 0; c < 8; c++) x[c] = ((int)((uint32_t)v[c] << 22) >> 22) + 128;
        lo = pk16(ashr_pk_u8(x[0], x[1], 0), ashr_pk_u8(x[2], x[3], 0));
        hi = pk16(ashr_pk_u8(x[4], x[5], 0), ashr_pk_u8(x[6], x[7], 0));
    }
    return make_uint2(lo, hi);
}

__device__ __forceinline__ uint2 idct_block_row(const DecDesc& d, int64_t b, int comp, int r, bool real,
                                                int32_t* ws)
{
    uint4 q = make_uint4(0u, 0u, 0u, 0u), qt = q;
    int32_t dc = 0;
    if (real) {
        q = *(const uint4*)(d.coefs + b * 64 + r * 8);
        qt = *(const uint4*)(d.tab->qt[comp] + r * 8);
        dc = d.dc[b];
    }
    return idct_row_of(q, dc, qt, r, real, ws);
}

// 8 threads per block, 32 blocks per tile, DEC_IDCT_TILES consecutive tiles
// per workgroup (the next tile's coefficient row, DC value and dequantisation
// row in registers while the current one transforms), one image per
// workgroup, into the component planes.  fuse420 images: chroma blocks only
// (their luma IDCT runs inside k_dec_luma_color_420).
struct IdctBlk {
    int64_t b;
    int comp, bx, by;
    bool real;
};
__device__ __forceinline__ IdctBlk idct_blk(const DecDesc& d, int i)
{
    int m, k;
    if (d.fuse420) {
        m = i >> 1;
        k = d.nby + (i & 1);
    } else {
        m = i / d.nbmcu;
        k = i - m * d.nbmcu;
    }
    IdctBlk r{(int64_t)m * d.nbmcu + k, 0, 0, 0, false};
    const bool valid = r.b < d.nblocks;
    if (valid) {
        const int mx = m % d.mcux, my = m / d.mcux;
        if (k < d.nby) {
            r.bx = mx * d.hs + k % d.hs;
            r.by = my * d.vs + k / d.hs;
        } else {
            r.comp = k - d.nby + 1;
            r.bx = mx;
            r.by = my;
        }
    }
    r.real = valid && r.bx * 8 < d.pw[r.comp] && r.by * 8 < d.ph[r.comp];  // dummy blocks: no IDCT (jdcoefct.c)
    return r;
}

#ifndef ICX_DEC_IDCT_PF
#define ICX_DEC_IDCT_PF 1  // > 0: the pipelined tile loop below, loads this many tiles ahead (0: the loop before it)
#endif
__global__ void __launch_bounds__(256) k_dec_idct(const DecDesc* D, const DecState* S, Plan p)
{
    __shared__ int32_t ws[32][8 * 9];
    int slot;
    int64_t wg;
    if (!plan_slot(p, slot, wg)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    if (S[img].status) return;
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int ntile = (int)(d.fuse420 ? (2 * (int64_t)d.mcux * d.mcuy + 31) / 32 : (d.nblocks + 31) / 32);
    const ICX_GLOBAL int16_t* const coefs = (const ICX_GLOBAL int16_t*)d.coefs;
    const ICX_GLOBAL int32_t* const dcs = (const ICX_GLOBAL int32_t*)d.dc;
    const ICX_GLOBAL uint16_t* const qts = (const ICX_GLOBAL uint16_t*)d.tab->qt[0];
    ICX_GLOBAL uint8_t* const planes[4] = {(ICX_GLOBAL uint8_t*)d.plane[0], (ICX_GLOBAL uint8_t*)d.plane[1],
                                           (ICX_GLOBAL uint8_t*)d.plane[2], (ICX_GLOBAL uint8_t*)d.plane[3]};
    const int pw[4] = {d.pw[0], d.pw[1], d.pw[2], d.pw[3]};
    int tile = (int)wg * DEC_IDCT_TILES;
    if (tile >= ntile) return;
#if ICX_DEC_IDCT_PF
    // as k_dec_luma_color_420: the tile loop unrolled, each tile's loads in
    // registers of their own issued IDCT_PF tiles ahead (tile index clamped,
    // no branch around them), and one store per lane on every path (a dummy
    // block's rows go to the plane's spare bytes), so the compiler's wait for
    // a tile's loads does not wait for the previous tiles' stores
    constexpr int T = DEC_IDCT_TILES, PF = ICX_DEC_IDCT_PF;
    IdctBlk B[T];
    uint4 Q[T], QT[T];
    int32_t DCv[T];
    auto fetch = [&](int k, int tl) {
        B[k] = idct_blk(d, tl * 32 + lb);
        const int64_t bb = B[k].b < d.nblocks ? B[k].b : 0;
        Q[k] = *(const ICX_GLOBAL uint4*)(coefs + bb * 64 + r * 8);
        DCv[k] = dcs[bb];
        QT[k] = *(const ICX_GLOBAL uint4*)(qts + B[k].comp * 64 + r * 8);
    };
#pragma unroll
    for (int k = 0; k < PF && k < T; k++) fetch(k, min(tile + k, ntile - 1));
#pragma unroll
    for (int it = 0; it < T; it++, tile++) {
        if (tile >= ntile) break;  // workgroup-uniform
        if (it + PF < T) fetch(it + PF < T ? it + PF : 0, min(tile + PF, ntile - 1));
        const IdctBlk& cb = B[it];
        const uint2 row = idct_row_of(Q[it], DCv[it], QT[it], r, cb.real, ws[lb]);
        // a lane past the image's blocks has no component of its own: the
        // spare bytes of a plane this launch always has (fuse420: no luma plane)
        const int c = cb.real ? cb.comp : d.fuse420 ? 1 : 0;
        ICX_GLOBAL uint8_t* const dst = cb.real ? planes[c] + (int64_t)(cb.by * 8 + r) * pw[c] + cb.bx * 8
                                                : planes[c] + (int64_t)pw[c] * d.ph[c] + r * 8;
        *(ICX_GLOBAL uint2*)dst = row;
    }
    return;
#endif
    // i < 2^31: at most 65535^2 * 3 / 64 blocks
    IdctBlk cb = idct_blk(d, tile * 32 + lb);
    const int64_t b0 = cb.b < d.nblocks ? cb.b : 0;
    uint4 q = *(const ICX_GLOBAL uint4*)(coefs + b0 * 64 + r * 8);
    int32_t dc = dcs[b0];
    uint4 qt = *(const ICX_GLOBAL uint4*)(qts + cb.comp * 64 + r * 8);
    for (int it = 0; it < DEC_IDCT_TILES; it++, tile++) {
        if (tile >= ntile) break;  // workgroup-uniform
        IdctBlk nb = cb;
        uint4 nq = q, nqt = qt;
        int32_t ndc = dc;
        if (it + 1 < DEC_IDCT_TILES && tile + 1 < ntile) {
            nb = idct_blk(d, (tile + 1) * 32 + lb);
            const int64_t bb = nb.b < d.nblocks ? nb.b : 0;
            nq = *(const ICX_GLOBAL uint4*)(coefs + bb * 64 + r * 8);
            ndc = dcs[bb];
            nqt = *(const ICX_GLOBAL uint4*)(qts + nb.comp * 64 + r * 8);
        }
        const uint2 row = idct_row_of(q, dc, qt, r, cb.real, ws[lb]);
        // no barrier before the next tile: a thread's pass 2 reads only its own
        // workspace row, which only it rewrites, and pass 1 of the next tile
        // comes after idct_row_of's first barrier
        if (cb.real) *(ICX_GLOBAL uint2*)(planes[cb.comp] + (int64_t)(cb.by * 8 + r) * pw[cb.comp] + cb.bx * 8) = row;
        cb = nb;
        q = nq;
        qt = nqt;
        dc = ndc;
    }
}

// ----------------------------------------------------------- colour output
// Upsampled chroma sample of component plane P at full-resolution (X, Y)
// (jdsample.c: h2v2/h2v1 fancy when cw > 2, else replication - also
// int_upsample's for 1x2 (4:4:0) and 4x1 (4:1:1) luma; 1x1 direct).
__device__ __forceinline__ int chroma_at(const DecDesc& d, const uint8_t* P, int pitch, int cw, int ch, int X, int Y)
{
    if (d.hs == 1 && d.vs == 1) return P[(int64_t)Y * pitch + X];
    if (!d.fancy) return P[(int64_t)(Y / d.vs) * pitch + X / d.hs];
    const int i = X >> 1;
    if (d.vs == 1) {  // h2v1_fancy_upsample
        const uint8_t* in = P + (int64_t)Y * pitch;
        const int c = in[i];
        if (!(X & 1)) return i == 0 ? c : (c * 3 + in[i - 1] + 1) >> 2;
        return i == cw - 1 ? c : (c * 3 + in[i + 1] + 2) >> 2;
    }
    // h2v2_fancy_upsample: context row above (even Y) / below (odd Y), replicated at the edges
    const int r0 = Y >> 1;
    int rn = (Y & 1) ? r0 + 1 : r0 - 1;
    rn = rn < 0 ? 0 : rn > ch - 1 ? ch - 1 : rn;
    const uint8_t* a = P + (int64_t)r0 * pitch;
    const uint8_t* bb = P + (int64_t)rn * pitch;
    const int cs = a[i] * 3 + bb[i];
    if (!(X & 1)) return i == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + a[i - 1] * 3 + bb[i - 1] + 8) >> 4;
    return i == cw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + a[i + 1] * 3 + bb[i + 1] + 7) >> 4;
}

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

// a * k + c on v_mad_i32_i24 (full rate), a and k within 24 signed bits.
// Inline asm: with the operands' ranges known the compiler turns __mul24 back
// into v_mul_lo_u32 / v_mad_u64_u32, quarter-rate instructions.
__device__ __forceinline__ int mad24(int a, int k, int c)
{
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
    return r;
}

// ycc_rgb_convert (jdcolor.c, SCALEBITS 16) of one pixel, cb / cr already
// less 128: y + ((k * c + ONE_HALF) >> 16) computed as ((y << 16) + ONE_HALF
// + k * c) >> 16 (y << 16 is a multiple of 2^16; |c| <= 128, |k| < 2^17)
struct Bgr {
    uint32_t b, g, r;
};
__device__ __forceinline__ Bgr ycc_bgr(int yy, int cb, int cr)
{
    const int y16 = (yy << 16) + 32768;
    Bgr o;
    o.b = clamp255(mad24(cb, 116130, y16) >> 16);
    o.g = clamp255(mad24(cr, -46802, mad24(cb, -22554, y16)) >> 16);
    o.r = clamp255(mad24(cr, 91881, y16) >> 16);
    return o;
}

// Thread per 4 output pixels of one output row; one image per workgroup.
__global__ void __launch_bounds__(256) k_dec_color(const DecDesc* D, const DecState* S, Plan p)
{
    int slot;
    int64_t wg;
    if (!plan_slot(p, slot, wg)) return;
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    if (S[img].status) return;
    const int64_t item = wg * 256 + threadIdx.x;
    const int gpr = (d.ow + 3) >> 2;
    const int y = (int)(item / gpr), x0 = (int)(item % gpr) * 4;
    if (y >= d.oh) return;
    const int Y = y * d.s;
    uint8_t* orow = d.out + (int64_t)y * d.ostride;
    const uint8_t* yrow = d.plane[0] + (int64_t)Y * d.pw[0];
    if (d.ncomp == 1) {
        for (int k = 0; k < 4 && x0 + k < d.ow; k++) orow[x0 + k] = yrow[(x0 + k) * d.s];
        return;
    }
    if (d.ncomp == 4) {  // CMYK / YCCK: every component 1x1 (icx_jpeg_parse.cpp)
        const int64_t off = (int64_t)Y * d.pw[0];
        for (int k = 0; k < 4 && x0 + k < d.ow; k++) {
            const int X = (x0 + k) * d.s;
            int c0 = d.plane[0][off + X], c1 = d.plane[1][off + X], c2 = d.plane[2][off + X];
            const int kk = d.plane[3][off + X];
            if (d.cmyk == 2) {  // ycck_cmyk_convert (jdcolor.c): C, M, Y = 255 - R, G, B of ycc_rgb_convert
                const int cb = c1 - 128, cr = c2 - 128, yy = c0;
                c0 = 255 - clamp255(yy + ((91881 * cr + 32768) >> 16));
                c1 = 255 - clamp255(yy + ((-22554 * cb + 32768 - 46802 * cr) >> 16));
                c2 = 255 - clamp255(yy + ((116130 * cb + 32768) >> 16));
            }
            if (d.raw4) {  // libjpeg's CMYK samples (debug / parity)
                uint8_t* o = orow + (int64_t)(x0 + k) * 4;
                o[0] = (uint8_t)c0, o[1] = (uint8_t)c1, o[2] = (uint8_t)c2, o[3] = (uint8_t)kk;
                continue;
            }
            // to RGB as the host path did (Pillow: the samples read as Adobe-inverted
            // CMYK, then cmyk2rgb: nk - nk * c / 255 with nk = 255 - k); TwelveMonkeys'
            // ICC conversion is not restatable here (parity unpinned)
            const int nk = kk;  // 255 - (255 - raw k)
            uint8_t* o = orow + (int64_t)(x0 + k) * 3;
            const int cv[3] = {255 - c0, 255 - c1, 255 - c2};
            int rgb[3];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int t = cv[q] * nk + 128;
                rgb[q] = nk - (((t >> 8) + t) >> 8);
            }
            o[0] = clamp255(rgb[2]), o[1] = clamp255(rgb[1]), o[2] = clamp255(rgb[0]);  // BGR
        }
        return;
    }
    uint8_t px[12];
    const int n = d.ow - x0 < 4 ? d.ow - x0 : 4;
    for (int k = 0; k < n; k++) {
        const int X = (x0 + k) * d.s;
        const int yy = yrow[X];
        const int cb = chroma_at(d, d.plane[1], d.pw[1], d.cw[1], d.ch[1], X, Y) - 128;
        const int cr = chroma_at(d, d.plane[2], d.pw[2], d.cw[1], d.ch[1], X, Y) - 128;
        if (d.rgb) {  // null_convert (jdcolor.c): R, G, B as stored
            px[3 * k + 0] = (uint8_t)(cr + 128);
            px[3 * k + 1] = (uint8_t)(cb + 128);
            px[3 * k + 2] = (uint8_t)yy;
            continue;
        }
        const Bgr c = ycc_bgr(yy, cb, cr);
        px[3 * k + 0] = (uint8_t)c.b;
        px[3 * k + 1] = (uint8_t)c.g;
        px[3 * k + 2] = (uint8_t)c.r;
    }
    uint8_t* o = orow + x0 * 3;
    if (n == 4 && (((uintptr_t)o) & 3) == 0) {
        uint32_t w[3];
        for (int q = 0; q < 3; q++)
            w[q] = px[4 * q] | (px[4 * q + 1] << 8) | (px[4 * q + 2] << 16) | ((uint32_t)px[4 * q + 3] << 24);
        *(uint3*)o = make_uint3(w[0], w[1], w[2]);
    } else {
        for (int k = 0; k < 3 * n; k++) o[k] = px[k];
    }
}

// s == 1, 4:2:0 with fancy upsampling (the JDK decode of nearly every photo):
// a tile is one MCU row x LC_NM MCUs (16 x 128 output pixels).  The 32 luma
// blocks are inverse-transformed straight into an LDS tile (the luma plane
// never reaches HBM); chroma rows cy0-1 .. cy0+8 (edge-replicated, jdmainct.c
// context rows) and columns cx0-4 .. cx0+67 of both chroma planes (written by
// k_dec_idct) are staged as dwords; each thread then converts a 4 x 2 pixel
// tile from the 3 x 4 chroma neighbourhood it shares (h2v2_fancy_upsample +
// ycc_rgb_convert).  A workgroup runs LC_T consecutive tiles with the next
// tile's coefficient, DC and chroma loads in registers while it transforms
// and converts the current one, so the HBM reads of a CU's workgroups stay in
// flight through their barrier phases (one tile per workgroup left each
// workgroup's loads exposed, then a few microseconds of compute with none).
#ifndef ICX_DEC_LC_DWORD
#define ICX_DEC_LC_DWORD 0
#endif
#ifndef ICX_DEC_LC_WAVES
#define ICX_DEC_LC_WAVES 1
#endif
#ifndef ICX_DEC_LC_PF
#define ICX_DEC_LC_PF 3  // tiles whose loads are in flight ahead of the one being converted: 1 / 2 / 3 = 11.15 / 11.1 / 10.85 ms colour pass per 1000 frames (ab_r5an_dec_color_pipe.txt)
#endif
#ifndef ICX_DEC_LC_FULL
#define ICX_DEC_LC_FULL 1  // interior tiles: a fixed store sequence (below); without: 11.7 ms
#endif
constexpr int LC_NM = 8;  // dec_lc_items
constexpr int LC_W = 16 * LC_NM;      // output columns per tile
constexpr int LC_CD = LC_W / 8 + 2;   // chroma dwords per staged row
constexpr int LC_CE = 2 * 10 * LC_CD; // chroma dwords per tile (both planes)
constexpr int LC_T = DEC_LC_TILES;    // tiles per workgroup

struct LcLoad {
    uint4 q;         // coefficient row r of this thread's luma block
    int32_t dc;      // its DC value
    uint32_t c[2];   // chroma dwords e = t, t + 256 of the tile
};

// The image's fields the tile loop uses, read once into registers (the
// loop's byte stores may alias the descriptor as far as the compiler knows,
// and a reload after each store would wait for the prefetch in flight).
struct LcImg {
    const ICX_GLOBAL int16_t* coefs;  // global address space: loads that wait on vmcnt alone
    const ICX_GLOBAL int32_t* dc;
    const ICX_GLOBAL uint8_t* plane[2];
    int pitch[2];
    int nbmcu, mcux, ch, pwd, tpr;
};

__device__ __forceinline__ void lc_fetch(const LcImg& g, int item, int t, LcLoad& L)
{
    const int my = item / g.tpr, mx0 = (item - my * g.tpr) * LC_NM;
    const int lb = t >> 3, r = t & 7, k = lb & 3;
    int mx = mx0 + (lb >> 2);
    mx = mx < g.mcux ? mx : g.mcux - 1;  // blocks past the last MCU: any loadable block, not transformed
    const int64_t b = ((int64_t)my * g.mcux + mx) * g.nbmcu + k;
    L.q = *(const ICX_GLOBAL uint4*)(g.coefs + b * 64 + r * 8);
    L.dc = g.dc[b];
    const int cx0 = mx0 * 8, cy0 = my * 8;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        int e = t + 256 * h;
        e = e < LC_CE ? e : LC_CE - 1;
        const int comp = e / (10 * LC_CD), rem = e - comp * (10 * LC_CD);
        const int j = rem / LC_CD, q = rem - j * LC_CD;
        int rr = cy0 - 1 + j;
        rr = rr < 0 ? 0 : rr > g.ch - 1 ? g.ch - 1 : rr;
        int dw = (cx0 >> 2) - 1 + q;
        dw = dw < 0 ? 0 : dw > g.pwd - 1 ? g.pwd - 1 : dw;  // clamped dwords hold only unused columns
        const ICX_GLOBAL uint32_t* row = (const ICX_GLOBAL uint32_t*)(g.plane[comp] + (int64_t)rr * g.pitch[comp]);
        L.c[h] = row[dw];
    }
}

__global__ void __launch_bounds__(256, ICX_DEC_LC_WAVES) k_dec_luma_color_420(const DecDesc* D, const DecState* S, Plan p)
{
    __shared__ int32_t ws[32][8 * 9];
    // luma tile rows padded to 36 dwords: the IDCT's 8-byte row stores (lanes
    // r = 0..7 of a block, one row each) spread over the banks instead of
    // eight lanes on one bank pair at a 32-dword stride
    __shared__ __attribute__((aligned(16))) uint32_t ly[16][LC_W / 4 + 4];
    __shared__ uint32_t lcb[2][LC_CE];  // per tile parity: [cb|cr][chroma row cy0-1+j][dword]; byte q <-> column cx0-4+q
    int slot;
    int64_t wg;
    // the image's state and descriptor fields are read before the exits, so
    // their loads go out together with the plan's
    const bool in = plan_slot(p, slot, wg);
    const int img = p.ids[slot];
    const DecDesc& d = D[img];
    const int status = S[img].status, mcux = d.mcux, mcuy = d.mcuy, cw = d.cw[1];
    const int pw0 = d.pw[0], ph0 = d.ph[0], ow = d.ow, oh = d.oh, ostride = d.ostride;
    ICX_GLOBAL uint8_t* const out = (ICX_GLOBAL uint8_t*)d.out;
    const LcImg g{(const ICX_GLOBAL int16_t*)d.coefs, (const ICX_GLOBAL int32_t*)d.dc,
                  {(const ICX_GLOBAL uint8_t*)d.plane[1], (const ICX_GLOBAL uint8_t*)d.plane[2]}, {d.pw[1], d.pw[2]},
                  d.nbmcu, mcux, d.ch[1], d.pw[1] >> 2, (mcux + LC_NM - 1) / LC_NM};
    const ICX_GLOBAL uint16_t* const qtab = (const ICX_GLOBAL uint16_t*)d.tab->qt[0];
    if (!in || status) return;
    const int tpr = g.tpr, ntile = tpr * mcuy;
    const int t = threadIdx.x;
    int item = (int)wg * LC_T;
    if (item >= ntile) return;
    const uint4 qt = *(const ICX_GLOBAL uint4*)(qtab + (t & 7) * 8);
    // The tile loop unrolled, each tile's loads in registers of their own,
    // issued LC_PF tiles ahead: no register copies between tiles (a copy of
    // a load's destination waits for the load) and no branch around a load
    // (the tile index is clamped to the image's last tile instead), so the
    // compiler's counter waits see every load and store in flight.
    LcLoad L[LC_T];
    constexpr int PF = ICX_DEC_LC_PF;
#pragma unroll
    for (int k = 0; k < PF && k < LC_T; k++) lc_fetch(g, min(item + k, ntile - 1), t, L[k]);
#pragma unroll
    for (int it = 0; it < LC_T; it++, item++) {
        if (item >= ntile) break;  // workgroup-uniform
        if (it + PF < LC_T) lc_fetch(g, min(item + PF, ntile - 1), t, L[it + PF < LC_T ? it + PF : 0]);
        const LcLoad& cur = L[it];
        const int my = item / tpr, mx0 = (item - my * tpr) * LC_NM;
        uint32_t* lc = lcb[it & 1];  // the previous tile's colour pass may still read the other one
        lc[t] = cur.c[0];
        if (t + 256 < LC_CE) lc[t + 256] = cur.c[1];
        {  // luma: block lb = MCU lb / 4, block k = lb % 4 of it
            const int lb = t >> 3, r = t & 7, mx = mx0 + (lb >> 2), k = lb & 3;
            const int bx = mx * 2 + (k & 1), by = my * 2 + (k >> 1);
            const bool real = mx < mcux && bx * 8 < pw0 && by * 8 < ph0;
            const uint2 row = idct_row_of(cur.q, cur.dc, qt, r, real, ws[lb]);
            *(uint2*)&ly[(k >> 1) * 8 + r][(lb >> 2) * 4 + (k & 1) * 2] = row;
        }
        __syncthreads();
        {
            // the edge columns replicated (h2v2_fancy_upsample's first / last
            // column: c * 4 = c * 3 + the column itself), so the colour pass
            // below has no edge cases: column -1 := column 0 (local bytes 3 <-
            // 4), column cw := column cw - 1; tile-uniform, so the extra
            // barrier runs in edge tiles only
            const int cx0 = mx0 * 8, lr = cw - cx0 + 4;  // local byte of column cw
            const bool left = cx0 == 0, right = lr < 4 * LC_CD;
            if (left || right) {
                if (t < 20) {  // one staged row (2 planes x 10 rows) per thread
                    uint8_t* row = (uint8_t*)(lc + t * LC_CD);
                    if (left) row[3] = row[4];
                    if (right) row[lr] = row[lr - 1];
                }
                __syncthreads();
            }
        }
        const int rp = t >> 5, xt = 4 * (t & 31);  // chroma row cy0 + rp -> output rows 2rp, 2rp+1; columns xt..xt+3
        const int x0 = mx0 * 16;
        const int n = ow - x0 - xt;
        const int y0 = my * 16 + 2 * rp;
#if ICX_DEC_LC_FULL
        // A tile whose 128 x 16 output pixels are all inside the image, on a
        // 4-byte aligned output, stores two 12-byte groups per thread and
        // nothing else; edge tiles keep the per-pixel tests and byte stores
        // and then wait for their stores.  The loop's wait for the next
        // tile's loads (vector-memory counters count stores too, in order)
        // then leaves a full tile's two stores in flight instead of waiting
        // for every store the tile issued - the compiler only counts stores
        // it can see issued on every path.
        const bool full = x0 + LC_W <= ow && my * 16 + 16 <= oh && (((uintptr_t)out | (uintptr_t)ostride) & 3) == 0;
        auto convert = [&](auto full_c) {
        constexpr bool FULL = decltype(full_c)::value;
#else
        {
        constexpr bool FULL = false;
#endif
        if (FULL || (n > 0 && y0 < oh)) {
            const int li = (xt >> 1) + 4;        // local byte of i0
            int cv[2][2][4];                     // [comp][top|bottom row][column]: upsampled value - 128
#pragma unroll
            for (int comp = 0; comp < 2; comp++) {
                int cs_t[4], cs_b[4];  // column sums for i0-1 .. i0+2
#if ICX_DEC_LC_DWORD
                // the 4 bytes li-1 .. li+2 of rows cy0+rp-1 .. +1: two aligned
                // dword reads per row and a funnel shift, not four byte reads
                const uint32_t* r0 = lc + comp * 10 * LC_CD + rp * LC_CD + ((li - 1) >> 2);
                const uint32_t sh = (uint32_t)(li - 1) & 3u;
                const uint32_t v0 = __builtin_amdgcn_alignbyte(r0[1], r0[0], sh);
                const uint32_t v1 = __builtin_amdgcn_alignbyte(r0[LC_CD + 1], r0[LC_CD], sh);
                const uint32_t v2 = __builtin_amdgcn_alignbyte(r0[2 * LC_CD + 1], r0[2 * LC_CD], sh);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int a = (int)((v1 >> (8 * k)) & 255u) * 3;
                    cs_t[k] = a + (int)((v0 >> (8 * k)) & 255u);
                    cs_b[k] = a + (int)((v2 >> (8 * k)) & 255u);
                }
#else
                const uint8_t* c0 = (const uint8_t*)(lc + comp * 10 * LC_CD + rp * LC_CD);  // rows cy0+rp-1 .. +1
                const uint8_t* c1 = c0 + LC_CD * 4;
                const uint8_t* c2 = c1 + LC_CD * 4;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int a = c1[li - 1 + k] * 3;
                    cs_t[k] = a + c0[li - 1 + k];
                    cs_b[k] = a + c2[li - 1 + k];
                }
#endif
                // chroma column i0 + u -> output columns 2u (with column i0+u-1)
                // and 2u + 1 (with i0+u+1); the staged edge columns are
                // replicas, and (s + 8 - 2048) >> 4 = ((s + 8) >> 4) - 128
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int* cs = h ? cs_b : cs_t;
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const int a = cs[1 + u] * 3;
                        cv[comp][h][2 * u] = (a + cs[u] - 2040) >> 4;
                        cv[comp][h][2 * u + 1] = (a + cs[2 + u] - 2041) >> 4;
                    }
                }
            }
            const int m = FULL ? 4 : n < 4 ? n : 4;
            const int rows = FULL ? 2 : oh - y0 < 2 ? 1 : 2;
#pragma unroll
            for (int h = 0; h < 2; h++) {  // unrolled: cv stays in registers
                if (h >= rows) break;
                const uint32_t yq = ly[2 * rp + h][xt >> 2];
                int cb_[4], cg_[4], cr_[4];  // (y << 16) + ONE_HALF + products (ycc_bgr before the shift)
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    // (y << 16) + 32768 from byte k of yq in one v_perm_b32
                    const int y16 = (int)__builtin_amdgcn_perm(0x8000u, yq, 0x0C000504u | ((uint32_t)k << 16));
                    const int cb = cv[0][h][k], cr = cv[1][h][k];
                    cb_[k] = mad24(cb, 116130, y16);
                    cg_[k] = mad24(cr, -46802, mad24(cb, -22554, y16));
                    cr_[k] = mad24(cr, 91881, y16);
                }
                // B0 G0 R0 B1 | G1 R1 B2 G2 | R2 B3 G3 R3: >> 16, clamp, pack
                const uint32_t w[3] = {pk16(ashr_pk_u8(cb_[0], cg_[0], 16), ashr_pk_u8(cr_[0], cb_[1], 16)),
                                       pk16(ashr_pk_u8(cg_[1], cr_[1], 16), ashr_pk_u8(cb_[2], cg_[2], 16)),
                                       pk16(ashr_pk_u8(cr_[2], cb_[3], 16), ashr_pk_u8(cg_[3], cr_[3], 16))};
                ICX_GLOBAL uint8_t* o = out + (int64_t)(y0 + h) * ostride + (int64_t)(x0 + xt) * 3;
                if (FULL || (m == 4 && (((uintptr_t)o) & 3) == 0)) {
                    *(ICX_GLOBAL uint3*)o = make_uint3(w[0], w[1], w[2]);
                } else {
                    for (int k = 0; k < 3 * m; k++) o[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
                }
            }
        }
#if ICX_DEC_LC_FULL
        };
        if (full) {
            convert(std::true_type{});
        } else {
            convert(std::false_type{});
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this path's stores are all done here
        }
#else
        }
#endif
    }
}

// ---------------------------------------------------------------- launchers
// 2-D grid (x = item, y = slot) when the plan asks for one, else one row of nwg
static dim3 grid_of(const Plan& p, int64_t nwg)
{
    return p.width > 0 ? dim3((unsigned)p.width, (unsigned)p.m) : dim3((unsigned)nwg);
}

void launch_stage(const StageJob* jobs, const Plan& tiles, int64_t nwg, hipStream_t st)
{
    if (nwg > 0) hipLaunchKernelGGL(k_stage, grid_of(tiles, nwg), dim3(256), 0, st, jobs, tiles);
}

void launch_unstuff(const DecDesc* d, DecState* s, const Plan& cnt, int64_t ncnt, const Plan& tiles, int64_t ntiles,
                    const int32_t* ids, int m, uint32_t sub_bits, hipStream_t st)
{
    if (ntiles <= 0 || m <= 0) return;
    hipLaunchKernelGGL(k_unstuff_count, grid_of(cnt, ncnt), dim3(256), 0, st, d, s, cnt);
    hipLaunchKernelGGL(k_unstuff_scan, dim3((unsigned)m), dim3(1024), 0, st, d, s, ids, sub_bits);
    hipLaunchKernelGGL(k_unstuff_scatter, grid_of(tiles, ntiles), dim3(256), 0, st, d, s, tiles);
}

void launch_dec_init(const DecDesc* d, const DecState* s, const Plan& subs, int64_t nwg, uint32_t sub_bits,
                     uint32_t warm, hipStream_t st)
{
    if (nwg > 0) hipLaunchKernelGGL(k_dec_init, grid_of(subs, nwg), dim3(DEC_SYNC_NT), 0, st, d, s, subs, sub_bits, warm);
}

void launch_dec_sync(const DecDesc* d, const DecState* s, const Plan& subs, int64_t nwg, uint32_t sub_bits,
                     int iter, int nimg, uint32_t* changed, hipStream_t st)
{
    if (nwg > 0)
        hipLaunchKernelGGL(iter == 0 ? k_dec_sync<true> : k_dec_sync<false>, grid_of(subs, nwg), dim3(DEC_SYNC_NT), 0, st,
                           d, s, subs, sub_bits, iter, nimg, changed);
}

void launch_dec_offsets(const DecDesc* d, DecState* s, const int32_t* ids, int m, hipStream_t st)
{
    if (m > 0) hipLaunchKernelGGL(k_dec_offsets, dim3((unsigned)m), dim3(1024), 0, st, d, s, ids);
}

void launch_dec_write(const DecDesc* d, DecState* s, const Plan& subs, int64_t nwg, uint32_t sub_bits,
                      hipStream_t st)
{
    if (nwg > 0) hipLaunchKernelGGL(k_dec_write, grid_of(subs, nwg), dim3(DEC_WRITE_NT), 0, st, d, s, subs, sub_bits);
}

void launch_dec_dc(const DecDesc* d, const DecState* s, const int32_t* ids, int m, hipStream_t st)
{
    if (m > 0) hipLaunchKernelGGL(k_dec_dc, dim3((unsigned)m), dim3(1024), 0, st, d, s, ids);
}

void launch_dec_idct(const DecDesc* d, const DecState* s, const Plan& blocks, int64_t nwg, hipStream_t st)
{
    if (nwg > 0) hipLaunchKernelGGL(k_dec_idct, grid_of(blocks, nwg), dim3(256), 0, st, d, s, blocks);
}

void launch_dec_color(const DecDesc* d, const DecState* s, const Plan& px, int64_t nwg, hipStream_t st)
{
    if (nwg > 0) hipLaunchKernelGGL(k_dec_color, grid_of(px, nwg), dim3(256), 0, st, d, s, px);
}

void launch_dec_luma_color_420(const DecDesc* d, const DecState* s, const Plan& tiles, int64_t nwg, hipStream_t st)
{
    if (nwg > 0) hipLaunchKernelGGL(k_dec_luma_color_420, grid_of(tiles, nwg), dim3(256), 0, st, d, s, tiles);
}

}  // namespace icx
