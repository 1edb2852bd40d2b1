// icx_jpeg_parse.cpp — see icx_jpeg_parse.h.
#include "icx_jpeg_parse.h"

#include <stdlib.h>
#include <string.h>

namespace icx {

namespace {
const uint8_t kNat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
}

// Colour space of a 3-component file as the JDK reader settles it: libjpeg's
// guess (jdapimin.c default_decompress_parms: JFIF -> YCbCr; an Adobe marker's
// transform 0 -> RGB, else YCbCr; no marker: ids 1,2,3 -> YCbCr, 'R','G','B'
// -> RGB, else YCbCr), then OpenJDK imageioJPEG.c's override of a YCbCr
// guess: an Adobe marker with a transform other than 1 -> unknown (-1: left to
// the host reader), also next to a JFIF marker; no JFIF and no EXIF marker
// (IS_EXIF: the first saved COM/APPn marker is an APP1), ids other than 1,2,3
// and every component sampled alike -> RGB.  0 YCbCr, 1 RGB.
int colour_space(const JpegHeader& J, bool jfif, bool exif, bool adobe, int transform)
{
    /* libjpeg's guess */
    int ycc;
    if (jfif) ycc = 1;
    else if (adobe) ycc = transform != 0;
    else ycc = !(J.id[0] == 'R' && J.id[1] == 'G' && J.id[2] == 'B');
    if (!ycc) return 1;
    /* imageioJPEG.c's override of a YCbCr guess: an Adobe marker whose
     * transform is not 1 -> unknown, even next to a JFIF marker; else, with
     * neither JFIF nor EXIF, ids 1,2,3 keep YCbCr and equal sampling -> RGB */
    if (adobe) return transform == 1 ? 0 : -1;
    if (jfif || exif) return 0;
    if (J.id[0] == 1 && J.id[1] == 2 && J.id[2] == 3) return 0;
    return J.hs[1] == J.hs[0] && J.hs[2] == J.hs[0] && J.vs[1] == J.vs[0] && J.vs[2] == J.vs[0];
}

icx_status parse_jpeg(const uint8_t* p, size_t avail, size_t total, JpegHeader& J)
{
    J = JpegHeader{};
    if (total < 4) return ICX_E_CORRUPT;
    if (avail < 4) return ICX_E_BUFFER;
    if (p[0] != 0xFF || p[1] != 0xD8) return ICX_E_CORRUPT;
    size_t i = 2;
    bool sof = false, unsupported = false, refused = false, adobe = false, jfif = false, exif = false,
         saved_any = false;
    int transform = 0;
    for (;;) {
        // next marker: skip non-0xFF garbage, then fill bytes (jdmarker.c next_marker)
        while (i < avail && p[i] != 0xFF) i++;
        while (i < avail && p[i] == 0xFF) i++;
        if (i >= avail) return avail < total ? ICX_E_BUFFER : ICX_E_CORRUPT;
        const int m = p[i++];
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) return ICX_E_CORRUPT;
        if (i + 2 > avail) return avail < total ? ICX_E_BUFFER : ICX_E_CORRUPT;
        const size_t seg = ((size_t)p[i] << 8) | p[i + 1];
        if (seg < 2) return ICX_E_CORRUPT;
        if (i + seg > avail) return avail < total ? ICX_E_BUFFER : ICX_E_CORRUPT;
        const uint8_t* s = p + i + 2;
        const size_t n = seg - 2;
        i += seg;
        // imageioJPEG.c IS_EXIF: the first marker the reader saves (COM, APP0..15)
        // is an APP1, whatever it holds
        if (!saved_any && (m == 0xFE || (m >= 0xE0 && m <= 0xEF))) {
            saved_any = true;
            exif = m == 0xE1;
        }
        switch (m) {
        case 0xDB: {  // DQT
            size_t o = 0;
            while (o < n) {
                const int pq = s[o] >> 4, tq = s[o] & 15;
                if (tq > 3 || pq > 1) return ICX_E_CORRUPT;
                const size_t need = 1 + (pq ? 128 : 64);
                if (o + need > n) return ICX_E_CORRUPT;
                for (int k = 0; k < 64; k++)
                    J.qt[tq][kNat[k]] = pq ? (uint16_t)((s[o + 1 + 2 * k] << 8) | s[o + 2 + 2 * k]) : s[o + 1 + k];
                J.qt_ok[tq] = true;
                o += need;
            }
            break;
        }
        case 0xC4: {  // DHT
            size_t o = 0;
            while (o < n) {
                if (o + 17 > n) return ICX_E_CORRUPT;
                const int tc = s[o] >> 4, th = s[o] & 15;
                if (tc > 1 || th > 3) return ICX_E_CORRUPT;
                int cnt = 0;
                for (int l = 0; l < 16; l++) cnt += s[o + 1 + l];
                if (cnt > 256 || o + 17 + (size_t)cnt > n) return ICX_E_CORRUPT;
                memcpy(J.hbits[tc][th], s + o + 1, 16);
                memcpy(J.hvals[tc][th], s + o + 17, (size_t)cnt);
                J.hn[tc][th] = cnt;
                J.h_ok[tc][th] = true;
                o += 17 + (size_t)cnt;
            }
            break;
        }
        case 0xC0:
        case 0xC1:
        case 0xC2: {  // baseline / extended sequential / progressive, Huffman
            if (sof) return ICX_E_CORRUPT;
            J.progressive = m == 0xC2;
            if (n < 6) return ICX_E_CORRUPT;
            J.h = (s[1] << 8) | s[2];
            J.w = (s[3] << 8) | s[4];
            J.ncomp = s[5];
            // jdinput.c initial_setup: JERR_BAD_PRECISION (the JDK's 6b is built for 8-bit samples)
            if (s[0] != 8) refused = true;
            if (J.w == 0 || J.h == 0 || (J.ncomp != 1 && J.ncomp != 3 && J.ncomp != 4)) unsupported = true;
            if (J.ncomp == 4 && J.progressive) unsupported = true;  // progressive CMYK / YCCK: the host reader
            if (J.ncomp >= 1 && J.ncomp <= 4) {
                if (n < 6 + 3 * (size_t)J.ncomp) return ICX_E_CORRUPT;
                for (int c = 0; c < J.ncomp; c++) {
                    J.id[c] = s[6 + 3 * c];
                    J.hs[c] = s[7 + 3 * c] >> 4;
                    J.vs[c] = s[7 + 3 * c] & 15;
                    J.tq[c] = s[8 + 3 * c];
                    if (J.tq[c] > 3 || J.hs[c] < 1 || J.vs[c] < 1 || J.hs[c] > 4 || J.vs[c] > 4)
                        return ICX_E_CORRUPT;
                }
            }
            sof = true;
            break;
        }
        case 0xDD:  // DRI
            if (n < 2) return ICX_E_CORRUPT;
            J.ri = (s[0] << 8) | s[1];
            break;
        case 0xE0:  // APP0: JFIF
            if (n >= 5 && !memcmp(s, "JFIF\0", 5)) jfif = true;
            break;
        case 0xEE:  // APP14: Adobe colour transform (jdmarker.c examine_app14)
            if (n >= 12 && !memcmp(s, "Adobe", 5)) {
                adobe = true;
                transform = s[11];
            }
            break;
        case 0xDA: {  // SOS
            if (!sof) return ICX_E_CORRUPT;
            if (refused) return ICX_E_REFUSED;
            if (unsupported) return ICX_E_UNSUPPORTED;
            const int ns = n >= 1 ? s[0] : 0;
            if (!J.progressive) {
                if (ns != J.ncomp || n < 1 + 2 * (size_t)ns + 3) return ICX_E_UNSUPPORTED;  // multi-scan
                for (int k = 0; k < ns; k++) {
                    if (s[1 + 2 * k] != J.id[k]) return ICX_E_UNSUPPORTED;
                    J.td[k] = s[2 + 2 * k] >> 4;
                    J.ta[k] = s[2 + 2 * k] & 15;
                    if (J.td[k] > 3 || J.ta[k] > 3) return ICX_E_CORRUPT;
                }
                if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0) return ICX_E_UNSUPPORTED;
            }
            J.scan_off = i;
            if (J.ncomp == 4) {
                // jdapimin.c default_decompress_parms: an Adobe marker's transform 0 ->
                // CMYK, anything else -> YCCK; no marker -> CMYK.  One block per
                // component per MCU only (the CMYK layout libjpeg writes)
                J.cmyk = adobe && transform != 0 ? 2 : 1;
                for (int c = 0; c < 4; c++)
                    if (J.hs[c] != 1 || J.vs[c] != 1) return ICX_E_UNSUPPORTED;
            }
            if (J.ncomp == 3) {
                const int cs = colour_space(J, jfif, exif, adobe, transform);
                if (cs < 0) return ICX_E_UNSUPPORTED;
                J.rgb = cs == 1;
                if (J.hs[1] != 1 || J.vs[1] != 1 || J.hs[2] != 1 || J.vs[2] != 1) return ICX_E_UNSUPPORTED;
                // Y 1x1, 2x1, 2x2 (fancy upsampling when wide enough), 1x2 (4:4:0) and
                // 4x1 (4:1:1): int_upsample replication (jdsample.c jinit_upsampler)
                const int hy = J.hs[0], vy = J.vs[0];
                if (!((hy == 1 && vy == 1) || (hy == 2 && vy == 1) || (hy == 2 && vy == 2) || (hy == 1 && vy == 2) ||
                      (hy == 4 && vy == 1)))
                    return ICX_E_UNSUPPORTED;
            }
            // progressive: tables may be (re)defined between scans; prog_decode checks each scan's
            if (!J.progressive)
                for (int c = 0; c < J.ncomp; c++)
                    if (!J.qt_ok[J.tq[c]] || !J.h_ok[0][J.td[c]] || !J.h_ok[1][J.ta[c]]) return ICX_E_CORRUPT;
            return ICX_OK;
        }
        default:
            if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                // lossless / hierarchical / arithmetic: dimensions only.  The
                // reference's reader (TwelveMonkeys over the JDK's 6b) reads
                // lossless files (SOF3) with its own decoder: the host reader's
                // business; it refuses arithmetic coding (SOF9-11, jdmaster.c
                // JERR_ARITH_NOTIMPL) and hierarchical files (SOF5-7, 13-15,
                // jdmarker.c JERR_SOF_UNSUPPORTED): read() throws
                if (n >= 6) {
                    J.h = (s[1] << 8) | s[2];
                    J.w = (s[3] << 8) | s[4];
                    J.ncomp = s[5];
                }
                return m == 0xC3 ? ICX_E_UNSUPPORTED : ICX_E_REFUSED;
            }
            break;  // APPn, COM, DNL: skipped (ignoreMetadata, ImageCompression.java:126)
        }
    }
}

bool build_dec_huff(const uint8_t* bits, const uint8_t* vals, int n, DecHuff& t, DecSlow& slow)
{
    memset(&t, 0, sizeof(t));
    memset(&slow, 0, sizeof(slow));
    int code = 0, k = 0, nsub = 0;
    for (int l = 1; l <= 16; l++) {
        const int cnt = bits[l - 1];
        // jdhuff.c jpeg_make_d_derived_tbl rejects a length whose codes run
        // into the all-ones code or past it; checked BEFORE any entry of the
        // length is written, so an over-subscribed DHT never indexes past lut
        // (every code written below is < 2^l, its prefix < 2^DEC_LUT_BITS)
        if (code + cnt >= (1 << l) || k + cnt > n) return false;
        slow.valoff[l] = k - code;
        for (int i = 0; i < cnt; i++, code++, k++) {
            const uint16_t e = (uint16_t)((l << 8) | vals[k]);
            if (l <= DEC_LUT_BITS) {
                const int sh = DEC_LUT_BITS - l;
                for (int f = 0; f < (1 << sh); f++) t.lut[(code << sh) | f] = e;
            } else {
                const int pre = code >> (l - DEC_LUT_BITS);  // its 10-bit prefix
                uint16_t& p = t.lut[pre];
                if (p == 0) p = nsub < DEC_NSUB ? (uint16_t)(DEC_SUB | nsub++) : (uint16_t)DEC_SLOW;
                if (p & DEC_SUB) {
                    const int rest = 16 - l, low = (code & ((1 << (l - DEC_LUT_BITS)) - 1)) << rest;
                    for (int f = 0; f < (1 << rest); f++) t.lut2[p & (DEC_NSUB - 1)][low | f] = e;
                }
            }
        }
        slow.maxcode[l] = cnt ? code - 1 : -1;
        code <<= 1;
    }
    if (k != n) return false;
    memcpy(slow.vals, vals, (size_t)n);
    return true;
}

// DecLean of a built table (DC or AC class): every code's state transition,
// and for AC tables the symbol pairs (icx_decode.h): when the first code's
// bits and extra bits leave room in the 10-bit look-ahead for the whole of
// the next code, the entry also carries that code's length, extra bits and
// advance.  ICX_DEC_PAIR=0 builds no pairs (A/B).
void build_dec_lean(const DecHuff& h, bool ac, DecLean& lean)
{
    auto conv = [ac](uint16_t e) -> uint16_t {
        if (e & DEC_SUB) return (uint16_t)(DEC_LEAN_LONG | ((e & (DEC_NSUB - 1)) << 5));  // long-code prefix:
        if (e & DEC_SLOW) return (uint16_t)(DEC_LEAN_LONG | DEC_LEAN_SLOW);                // same second level
        return e ? dec_lean_entry(e >> 8, e & 255, ac) : (uint16_t)0;
    };
    static const bool pairs = !getenv("ICX_DEC_PAIR") || atoi(getenv("ICX_DEC_PAIR")) != 0;
    for (int i = 0; i < (1 << DEC_LUT_BITS); i++) {
        const uint16_t e = h.lut[i];
        uint32_t x = conv(e);
        const bool simple = e && !(e & (DEC_SUB | DEC_SLOW));
        if (pairs && ac && simple) {
            const int len1 = e >> 8, sz1 = e & 15, run1 = (e & 255) >> 4;
            const int c1 = len1 + sz1;
            const bool ends = sz1 == 0 && run1 != 15;  // EOB and the other size-0 symbols end the block
            if (!ends && c1 < DEC_LUT_BITS) {
                const int room = DEC_LUT_BITS - c1;
                const uint16_t e2 = h.lut[(i << c1) & ((1 << DEC_LUT_BITS) - 1)];  // the next code's first bits
                if (e2 && !(e2 & (DEC_SUB | DEC_SLOW)) && (e2 >> 8) <= room) {
                    const uint32_t l2 = conv(e2);                     // (length + extra) | advance | extra
                    const uint32_t len2 = e2 >> 8, sz2 = (l2 >> 12) & 15, zadd2 = (l2 >> 5) & 127;
                    x |= ((len2 + sz2) | sz2 << 5 | zadd2 << 9) << DEC_PAIR_SHIFT;  // bits consumed, extra bits, advance
                }
            }
        }
        lean.lut[i] = x;
    }
    for (int k = 0; k < DEC_NSUB; k++)
        for (int i = 0; i < (1 << (16 - DEC_LUT_BITS)); i++) lean.lut2[k][i] = conv(h.lut2[k][i]);
}

bool build_dec_tab(const JpegHeader& J, DecTab& T)
{
    memset(&T, 0, sizeof(T));
    int slot_of[2][4];  // (class, table id) -> slot
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 4; b++) slot_of[a][b] = -1;
    int ntab = 0;
    for (int c = 0; c < J.ncomp; c++) {
        for (int ac = 0; ac < 2; ac++) {
            const int id = ac ? J.ta[c] : J.td[c];
            int& sl = slot_of[ac][id];
            if (sl < 0) {
                if (ntab == 4) return false;
                sl = ntab++;
                if (!build_dec_huff(J.hbits[ac][id], J.hvals[ac][id], J.hn[ac][id], T.h[sl], T.slow[sl])) return false;
                if (!ac)  // jpeg_make_d_derived_tbl: DC symbols are 0..15 (12..15 the walks leave to seq_decode)
                    for (int q = 0; q < J.hn[ac][id]; q++)
                        if (J.hvals[ac][id][q] > 15) return false;
                build_dec_lean(T.h[sl], ac != 0, T.lean[sl]);
            }
            T.sel[2 * c + ac] = (uint8_t)sl;
        }
        memcpy(T.qt[c], J.qt[J.tq[c]], sizeof(T.qt[c]));
    }
    T.ntab = (uint8_t)ntab;
    return true;
}

uint32_t dec_selector(const DecTab& T)
{
    uint32_t s = 0;
    for (int k = 0; k < 8; k++) s |= (uint32_t)(T.sel[k] & 3) << (4 * k);
    return s;
}

}  // namespace icx
