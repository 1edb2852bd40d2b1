// icx_progressive.cpp — entropy decode of progressive JPEGs (SOF2) on the host.
//
// The JDK reader (ImageCompression.java:119-155 -> JPEGImageReader ->
// imageioJPEG.c) decodes a progressive file in buffered-image mode with IJG
// 6b: every scan is absorbed into the whole-image coefficient buffer by
// jdphuff.c, and the final output pass runs the ISLOW IDCT, upsampling and
// colour conversion over the completed coefficients.  The pixel half of that
// is the device decoder's (icx_decode.hip: k_dec_idct / k_dec_color /
// k_dec_luma_color_420); this file is the entropy half.  A progressive scan
// is not a candidate for the device's self-synchronising decode: its EOB
// runs span blocks and its refinement bits depend on which coefficients
// earlier scans left nonzero, so one scan is one sequential walk — the host
// walks one file per thread and hands the device the coefficient array in
// the layout k_dec_write produces (MCU order, natural order, DC in [0]).
//
// Scope (anything else returns ICX_E_CORRUPT / ICX_E_UNSUPPORTED and the
// caller falls back to the host reader):
//  * 8-bit, 1 or 3 components, the baseline decoder's sampling factors;
//  * clean streams: a bad Huffman code, a scan that runs out of data, a
//    missing restart marker or a bogus progression (each only a warning in
//    libjpeg, which then substitutes zeros) are reported as corrupt;
//  * no block smoothing: jdcoefct.c smoothing_ok() enables it only while a
//    component's AC coefficients 1..5 are not fully refined at the final
//    output pass; such files (truncated scan scripts) are ICX_E_UNSUPPORTED.
#include <string.h>

#include <vector>

#include "icx_jpeg_parse.h"

namespace icx {

namespace {

const uint8_t kNat[64 + 16] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
                               40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
                               29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
                               47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// Canonical Huffman table (jdhuff.c jpeg_make_d_derived_tbl): a LOOK-bit
// lookahead table, then maxcode / valoff per code length.
constexpr int LOOK = 11;
struct Huff {
    uint16_t look[1 << LOOK];  // (length << 8) | symbol, 0 = longer than LOOK bits
    int32_t maxcode[18];
    int32_t valoff[17];
    uint8_t vals[256];
    bool ok = false;
};

bool build_huff(const uint8_t* bits, const uint8_t* vals, int n, Huff& t)
{
    memset(t.look, 0, sizeof(t.look));
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        const int cnt = bits[l - 1];
        if (code + cnt >= (1 << l) || k + cnt > n) return false;
        t.valoff[l] = k - code;
        for (int i = 0; i < cnt; i++, code++, k++)
            if (l <= LOOK)
                for (int f = 0; f < (1 << (LOOK - l)); f++)
                    t.look[(code << (LOOK - l)) | f] = (uint16_t)((l << 8) | vals[k]);
        t.maxcode[l] = cnt ? code - 1 : -1;
        code <<= 1;
    }
    t.maxcode[17] = 0x7FFFFFFF;
    if (k != n) return false;
    memcpy(t.vals, vals, (size_t)n);
    t.ok = true;
    return true;
}

// Bit reader over the stuffed entropy segment (jdhuff.c fill_bit_buffer): FF
// 00 is a data FF, FF fill bytes before a marker are skipped, and at a marker
// the reader stops and supplies zero bits, counted so that consuming any of
// them is reported.
struct Bits {
    const uint8_t* p;
    size_t pos, end;
    uint64_t buf = 0;  // left-aligned
    int cnt = 0, zbits = 0;
    int marker = 0;    // unread marker code, 0 while in the data
    bool eof = false;  // the file ended inside the scan (marker = 0xD9 stands for it)
    bool over = false;  // a zero bit past the marker was consumed

    void fill()
    {
        // fast path: 4 plain bytes (no 0xFF among them) at once
        while (cnt <= 32 && !marker && pos + 4 <= end) {
            uint32_t v;
            memcpy(&v, p + pos, 4);
            const uint32_t x = ~v;  // a 0xFF byte of v is a zero byte of x
            if ((x - 0x01010101u) & ~x & 0x80808080u) break;
            buf |= (uint64_t)__builtin_bswap32(v) << (32 - cnt);
            cnt += 32;
            pos += 4;
        }
        while (cnt <= 56) {
            uint32_t b = 0;
            if (!marker) {
                if (pos >= end) {
                    marker = 0xD9;  // end of file: as libjpeg's inserted EOI
                    eof = true;
                    continue;
                }
                b = p[pos++];
                if (b == 0xFF) {
                    uint32_t c = 0xFF;
                    while (c == 0xFF && pos < end) c = p[pos++];
                    if (c == 0xFF) {  // the file ends in FF fill bytes
                        c = 0xD9;
                        eof = true;
                    }
                    if (c != 0) {
                        marker = (int)c;
                        continue;
                    }
                }
            } else {
                zbits += 8;
            }
            buf |= (uint64_t)b << (56 - cnt);
            cnt += 8;
        }
    }
    uint32_t peek(int n)
    {
        if (cnt < n) fill();
        return (uint32_t)(buf >> (64 - n));
    }
    void skip(int n)
    {
        buf <<= n;
        cnt -= n;
        if (cnt < zbits) over = true;
    }
    uint32_t get(int n)
    {
        if (n == 0) return 0;
        const uint32_t v = peek(n);
        skip(n);
        return v;
    }
    int decode(const Huff& t)
    {
        const uint32_t w = peek(16);
        const uint16_t e = t.look[w >> (16 - LOOK)];
        if (e) {
            skip(e >> 8);
            return e & 255;
        }
        for (int l = LOOK + 1; l <= 16; l++) {
            const int32_t code = (int32_t)(w >> (16 - l));
            if (code <= t.maxcode[l]) {
                skip(l);
                return t.vals[(t.valoff[l] + code) & 255];
            }
        }
        over = true;  // bad Huffman code
        return 0;
    }
    // Restart boundary (jdphuff.c process_restart + jdmarker.c read_restart_marker):
    // drop the buffered bits, then expect RSTn.
    bool restart(int want)
    {
        buf = 0;
        cnt = zbits = 0;
        if (!marker) {  // the reader stopped short of the marker: find it (next_marker)
            for (;;) {
                while (pos < end && p[pos] != 0xFF) pos++;
                while (pos < end && p[pos] == 0xFF) pos++;
                if (pos >= end) return false;
                const int c = p[pos++];
                if (c != 0) {
                    marker = c;
                    break;
                }
            }
        }
        if (marker != 0xD0 + want) return false;  // resync_to_restart territory: corrupt
        marker = 0;
        return true;
    }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

struct Comp {
    int id, hs, vs, tq, wb, hb;  // wb/hb: width_in_blocks / height_in_blocks
    bool latched;
    int coef_bits[64];
};

}  // namespace

icx_status prog_decode(const uint8_t* p, size_t len, const JpegHeader& J, int16_t* coefs, int32_t* dc,
                       uint16_t (*qt_out)[64])
{
    const int nc = J.ncomp;
    const int hmax = nc == 3 ? J.hs[0] : 1, vmax = nc == 3 ? J.vs[0] : 1;
    const int nby = hmax * vmax, nbmcu = nc == 3 ? nby + 2 : 1;
    const int mcux = (J.w + 8 * hmax - 1) / (8 * hmax), mcuy = (J.h + 8 * vmax - 1) / (8 * vmax);
    Comp C[3];
    for (int c = 0; c < nc; c++) {
        const int hc = nc == 3 ? J.hs[c] : 1, vc = nc == 3 ? J.vs[c] : 1;
        C[c] = Comp{J.id[c], hc, vc, J.tq[c], 0, 0, false, {}};
        // jdinput.c initial_setup: width_in_blocks = ceil(image_width * h / (max_h * 8))
        C[c].wb = (int)(((int64_t)J.w * hc + 8 * hmax - 1) / (8 * hmax));
        C[c].hb = (int)(((int64_t)J.h * vc + 8 * vmax - 1) / (8 * vmax));
        for (int k = 0; k < 64; k++) C[c].coef_bits[k] = -1;
    }
    // block index of component c's block (bx, by) in the device layout
    auto block_of = [&](int c, int bx, int by) -> int64_t {
        if (nc == 1) return (int64_t)by * mcux + bx;
        if (c == 0) return ((int64_t)(by / vmax) * mcux + bx / hmax) * nbmcu + (by % vmax) * hmax + bx % hmax;
        return ((int64_t)by * mcux + bx) * nbmcu + nby + c - 1;
    };
    uint16_t qt[4][64];
    bool qt_ok[4] = {};
    Huff H[2][4];
    int ri = 0;
    bool sof = false, any_scan = false;
    size_t i = 2;
    if (len < 4 || p[0] != 0xFF || p[1] != 0xD8) return ICX_E_CORRUPT;
    for (;;) {
        // jdmarker.c next_marker: skip anything up to FF, the FF fill bytes, and
        // FF 00 pairs (stuffed data the scan's reader did not need)
        int m = 0;
        while (m == 0) {
            while (i < len && p[i] != 0xFF) i++;
            while (i < len && p[i] == 0xFF) i++;
            if (i >= len) return ICX_E_CORRUPT;  // no EOI
            m = p[i++];
        }
        if (m == 0xD9) break;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (i + 2 > len) return ICX_E_CORRUPT;
        const size_t seg = ((size_t)p[i] << 8) | p[i + 1];
        if (seg < 2 || i + seg > len) return ICX_E_CORRUPT;
        const uint8_t* s = p + i + 2;
        const size_t n = seg - 2;
        i += seg;
        if (m == 0xDB) {  // DQT
            size_t o = 0;
            while (o < n) {
                const int pq = s[o] >> 4, tq = s[o] & 15;
                if (tq > 3 || pq > 1 || o + 1 + (pq ? 128 : 64) > n) return ICX_E_CORRUPT;
                for (int k = 0; k < 64; k++)
                    qt[tq][kNat[k]] = pq ? (uint16_t)((s[o + 1 + 2 * k] << 8) | s[o + 2 + 2 * k]) : s[o + 1 + k];
                qt_ok[tq] = true;
                o += 1 + (pq ? 128 : 64);
            }
        } else if (m == 0xC4) {  // DHT
            size_t o = 0;
            while (o < n) {
                if (o + 17 > n) return ICX_E_CORRUPT;
                const int tc = s[o] >> 4, th = s[o] & 15;
                int cnt = 0;
                for (int l = 0; l < 16; l++) cnt += s[o + 1 + l];
                if (tc > 1 || th > 3 || cnt > 256 || o + 17 + (size_t)cnt > n) return ICX_E_CORRUPT;
                if (!build_huff(s + o + 1, s + o + 17, cnt, H[tc][th])) return ICX_E_CORRUPT;
                o += 17 + (size_t)cnt;
            }
        } else if (m == 0xDD) {  // DRI
            if (n < 2) return ICX_E_CORRUPT;
            ri = (s[0] << 8) | s[1];
        } else if (m == 0xC2) {  // the frame parse_jpeg read
            if (sof || n < 6 || ((s[1] << 8) | s[2]) != J.h || ((s[3] << 8) | s[4]) != J.w || s[5] != nc)
                return ICX_E_CORRUPT;
            sof = true;
        } else if (m == 0xDA) {  // SOS: one scan
            if (!sof || n < 1) return ICX_E_CORRUPT;
            const int ns = s[0];
            if (ns < 1 || ns > nc || n < 4 + 2 * (size_t)ns) return ICX_E_CORRUPT;
            int sc[3], td[3], ta[3];
            for (int k = 0; k < ns; k++) {
                sc[k] = -1;
                for (int c = 0; c < nc; c++)
                    if (C[c].id == s[1 + 2 * k]) sc[k] = c;
                td[k] = s[2 + 2 * k] >> 4;
                ta[k] = s[2 + 2 * k] & 15;
                if (sc[k] < 0 || td[k] > 3 || ta[k] > 3) return ICX_E_CORRUPT;
                for (int q = 0; q < k; q++)
                    if (sc[q] == sc[k]) return ICX_E_CORRUPT;
            }
            const int Ss = s[1 + 2 * ns], Se = s[2 + 2 * ns], Ah = s[3 + 2 * ns] >> 4, Al = s[3 + 2 * ns] & 15;
            // jdphuff.c start_pass_phuff_decoder: parameter checks, then progression
            const bool dcband = Ss == 0;
            if (dcband ? Se != 0 : (Ss > Se || Se > 63 || ns != 1)) return ICX_E_CORRUPT;
            if ((Ah != 0 && Al != Ah - 1) || Al > 13) return ICX_E_CORRUPT;
            for (int k = 0; k < ns; k++) {
                int* cb = C[sc[k]].coef_bits;
                if (!dcband && cb[0] < 0) return ICX_E_CORRUPT;  // AC before any DC scan
                for (int q = Ss; q <= Se; q++) {
                    if (Ah != (cb[q] < 0 ? 0 : cb[q])) return ICX_E_CORRUPT;
                    cb[q] = Al;
                }
                Comp& cp = C[sc[k]];  // jdinput.c latch_quant_tables: first scan of the component
                if (!cp.latched) {
                    if (!qt_ok[cp.tq]) return ICX_E_CORRUPT;
                    memcpy(qt_out[sc[k]], qt[cp.tq], sizeof(qt[0]));
                    cp.latched = true;
                }
                // tables the scan uses must exist (jdhuff.c: only DC first scans read a DC table,
                // only AC scans an AC table)
                if (dcband && Ah == 0 && !H[0][td[k]].ok) return ICX_E_CORRUPT;
                if (!dcband && !H[1][ta[k]].ok) return ICX_E_CORRUPT;
            }
            any_scan = true;
            Bits B{p, i, len};
            int last_dc[3] = {0, 0, 0};
            uint32_t eobrun = 0;
            int rst_next = 0;
            const int64_t nunits = ns > 1 ? (int64_t)mcux * mcuy : (int64_t)C[sc[0]].wb * C[sc[0]].hb;
            int64_t togo = ri;
            const int p1 = 1 << Al, m1 = -1 << Al;
            for (int64_t u = 0; u < nunits; u++) {
                if (ri && togo == 0) {
                    if (!B.restart(rst_next)) return ICX_E_CORRUPT;
                    rst_next = (rst_next + 1) & 7;
                    togo = ri;
                    last_dc[0] = last_dc[1] = last_dc[2] = 0;
                    eobrun = 0;
                }
                togo--;
                if (dcband) {
                    // MCU: each scan component's blocks (interleaved), or one block
                    int64_t blk[6];
                    int bc[6], nb = 0;
                    if (ns == 1) {
                        const int c = sc[0];
                        const int bx = (int)(u % C[c].wb), by = (int)(u / C[c].wb);
                        blk[0] = block_of(c, bx, by);
                        bc[0] = 0;
                        nb = 1;
                    } else {
                        const int mx = (int)(u % mcux), my = (int)(u / mcux);
                        for (int k = 0; k < ns; k++) {
                            const int c = sc[k];
                            for (int v = 0; v < C[c].vs; v++)
                                for (int h = 0; h < C[c].hs; h++) {
                                    blk[nb] = block_of(c, mx * C[c].hs + h, my * C[c].vs + v);
                                    bc[nb++] = k;
                                }
                        }
                    }
                    for (int q = 0; q < nb; q++) {
                        int16_t* co = coefs + blk[q] * 64;
                        if (Ah == 0) {  // decode_mcu_DC_first
                            const int t = B.decode(H[0][td[bc[q]]]);
                            int d = 0;
                            if (t) {
                                if (t > 11) return ICX_E_CORRUPT;
                                d = extend((int)B.get(t), t);
                            }
                            last_dc[bc[q]] = (int)((unsigned)last_dc[bc[q]] + (unsigned)d);  // wraps, no UB
                            co[0] = (int16_t)(last_dc[bc[q]] * (1 << Al));
                        } else if (B.get(1)) {  // decode_mcu_DC_refine
                            co[0] = (int16_t)(co[0] | p1);
                        }
                    }
                } else {
                    const int c = sc[0];
                    const int bx = (int)(u % C[c].wb), by = (int)(u / C[c].wb);
                    int16_t* co = coefs + block_of(c, bx, by) * 64;
                    const Huff& T = H[1][ta[0]];
                    if (Ah == 0) {  // decode_mcu_AC_first
                        if (eobrun) {
                            eobrun--;
                        } else {
                            for (int k = Ss; k <= Se; k++) {
                                const int rs = B.decode(T);
                                int r = rs >> 4, t = rs & 15;
                                if (t) {
                                    k += r;
                                    if (k > Se) return ICX_E_CORRUPT;
                                    co[kNat[k]] = (int16_t)(extend((int)B.get(t), t) * (1 << Al));
                                } else if (r == 15) {
                                    k += 15;
                                } else {
                                    eobrun = 1u << r;
                                    if (r) eobrun += B.get(r);
                                    eobrun--;
                                    break;
                                }
                            }
                        }
                    } else {  // decode_mcu_AC_refine
                        int k = Ss;
                        if (eobrun == 0) {
                            for (; k <= Se; k++) {
                                const int rs = B.decode(T);
                                int r = rs >> 4, t = rs & 15, sv = 0;
                                if (t) {
                                    if (t != 1) return ICX_E_CORRUPT;
                                    sv = B.get(1) ? p1 : m1;
                                } else if (r != 15) {
                                    eobrun = 1u << r;
                                    if (r) eobrun += B.get(r);
                                    break;  // the rest of the band: the EOB pass below
                                }
                                // step over nonzero coefficients (a correction bit each) and r zero ones
                                do {
                                    int16_t& z = co[kNat[k]];
                                    if (z != 0) {
                                        if (B.get(1) && (z & p1) == 0) z = (int16_t)(z >= 0 ? z + p1 : z + m1);
                                    } else if (--r < 0) {
                                        break;
                                    }
                                    k++;
                                } while (k <= Se);
                                if (sv) {
                                    if (k > Se) return ICX_E_CORRUPT;
                                    co[kNat[k]] = (int16_t)sv;
                                }
                            }
                        }
                        if (eobrun > 0) {
                            for (; k <= Se; k++) {
                                int16_t& z = co[kNat[k]];
                                if (z != 0 && B.get(1) && (z & p1) == 0) z = (int16_t)(z >= 0 ? z + p1 : z + m1);
                            }
                            eobrun--;
                        }
                    }
                }
                if (B.over) return ICX_E_CORRUPT;
            }
            // continue the marker walk at the marker that ended the scan (bytes the
            // reader fetched past the last needed bit are padding)
            if (B.eof) return ICX_E_CORRUPT;  // the file ends inside a scan
            i = B.pos;
            if (B.marker) {  // back to the marker's FF
                while (i > 0 && p[i - 1] != 0xFF) i--;
                if (i > 0) i--;
            }
        } else if ((m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) || m == 0xDC) {
            return ICX_E_CORRUPT;  // a second frame / DNL: not a single progressive frame
        }
        // APPn, COM: skipped
    }
    if (!sof || !any_scan) return ICX_E_CORRUPT;
    // Deliberately more conservative than jdcoefct.c smoothing_ok(): the device
    // path takes a file only when every component's DC is known and AC 1..5
    // are final (then no block smoothing happens); everything else goes to the
    // host reader, including cases smoothing_ok() would also leave unsmoothed
    // (a component without any DC scan, a zero Q00..Q20 quantiser entry)
    for (int c = 0; c < nc; c++) {
        if (C[c].coef_bits[0] < 0) return ICX_E_UNSUPPORTED;
        for (int k = 1; k <= 5; k++)
            if (C[c].coef_bits[k] != 0) return ICX_E_UNSUPPORTED;
        if (!C[c].latched) return ICX_E_CORRUPT;
    }
    const int64_t nblocks = (int64_t)mcux * mcuy * nbmcu;
    for (int64_t b = 0; b < nblocks; b++) dc[b] = coefs[b * 64];
    return ICX_OK;
}

}  // namespace icx

extern "C" icx_status icx_debug_progressive_coefs(const uint8_t* data, size_t len, int16_t* coefs, size_t ncoefs)
{
    using namespace icx;
    if (!data || !coefs) return ICX_E_NULL;
    JpegHeader J;
    icx_status s = parse_jpeg(data, len, len, J);
    if (s != ICX_OK) return s;
    if (!J.progressive) return ICX_E_INVALID;
    const int hs = J.ncomp == 3 ? J.hs[0] : 1, vs = J.ncomp == 3 ? J.vs[0] : 1;
    const size_t nb = (size_t)((J.w + 8 * hs - 1) / (8 * hs)) * ((J.h + 8 * vs - 1) / (8 * vs)) *
                      (J.ncomp == 3 ? hs * vs + 2 : 1);
    if (nb * 64 > ncoefs) return ICX_E_BUFFER;
    memset(coefs, 0, nb * 128);
    std::vector<int32_t> dc(nb);
    uint16_t qt[3][64];
    return prog_decode(data, len, J, coefs, dc.data(), qt);
}
