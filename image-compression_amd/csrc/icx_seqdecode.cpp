// icx_seqdecode.cpp — sequential (baseline / extended Huffman) entropy decode
// on the host with IJG 6b's recovery semantics, for the files the device's
// self-synchronising decode does not settle exactly (icx_decode.cpp).
//
// The reference reads every JPEG through the JDK's JPEGImageReader
// (ImageCompression.java:113-155), i.e. IJG libjpeg 6b, which decodes damaged
// entropy data with warnings only, so such files are compressed, not failed:
//  * end of file inside the scan: the JDK's source manager
//    (imageioJPEG.c imageio_fill_input_buffer) inserts a fake EOI; jdhuff.c
//    jpeg_fill_bit_buffer then supplies zero bits and sets insufficient_data:
//    the MCU being decoded finishes on zeros, every later MCU of the segment
//    stays zero (grey 128);
//  * a bad Huffman code (none within 16 bits) has consumed 17 bits and
//    decodes as symbol 0 (jpeg_huff_decode, JWRN_HUFF_BAD_CODE);
//  * a restart boundary drops the bit buffer and reads the next marker
//    (jdhuff.c process_restart, jdmarker.c read_restart_marker / next_marker):
//    the expected RSTn is swallowed, anything else goes through
//    jpeg_resync_to_restart; insufficient_data is cleared only when no marker
//    is left pending.
// The device path decodes every intact file itself and flags anything that
// departs from the clean case (an invalid code on the settled path, a symbol
// reaching into an interval's padding, an interval of the wrong length, a
// block count short of the frame's); those files come here, and the device
// runs the IDCT, upsampling and colour passes on what this decode leaves (the
// progressive files' route, icx_progressive.cpp).
//
// CPU restatement of the same algorithm, test infrastructure:
// oracle/icx_oracle_decode.c decode_scan; both are pinned by
// tests/golden/recovery_golden.* (libjpeg-turbo decodes of damaged files).
#include <string.h>

#include <vector>

#include "icx_jpeg_parse.h"

namespace icx {

namespace {

const uint8_t kNat[64 + 16] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
                               40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
                               29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
                               47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr int LOOK = 10;
struct Table {
    uint16_t look[1 << LOOK];  // (length << 8) | symbol, 0 = longer than LOOK bits or no code
    int32_t maxcode[18];       // [17] ends the canonical walk (jdhuff.c)
    int32_t valoff[17];
    uint8_t vals[256];
};

bool build(const uint8_t* bits, const uint8_t* vals, int n, bool dc, Table& t)
{
    memset(t.look, 0, sizeof(t.look));
    int code = 0, k = 0;
    for (int l = 1; l <= 16; l++) {
        const int cnt = bits[l - 1];
        // jpeg_make_d_derived_tbl: the codes of a length stay below the all-ones code
        if (code + cnt >= (1 << l) || k + cnt > n) return false;
        t.valoff[l] = k - code;
        for (int i = 0; i < cnt; i++, code++, k++)
            if (l <= LOOK)
                for (int f = 0; f < (1 << (LOOK - l)); f++)
                    t.look[(code << (LOOK - l)) | f] = (uint16_t)((l << 8) | vals[k]);
        t.maxcode[l] = cnt ? code - 1 : -1;
        code <<= 1;
    }
    t.maxcode[17] = 0xFFFFF;
    if (k != n) return false;
    if (dc)  // jpeg_make_d_derived_tbl: DC symbols (difference sizes) are 0..15
        for (int i = 0; i < n; i++)
            if (vals[i] > 15) return false;
    memcpy(t.vals, vals, (size_t)n);
    return true;
}

// The file from the first scan byte on, as the JDK's source manager serves
// it: past the end, FF D9 FF D9 ... (fake EOI markers).
struct Src {
    const uint8_t* p;
    size_t len, pos;
    int byte()
    {
        const size_t i = pos++;
        if (i < len) return p[i];
        return ((i - len) & 1) ? 0xD9 : 0xFF;
    }
};

// Bit reader: the real bits before the marker that stopped the reader, then
// zeros.  insufficient is set when a consumed bit lies past the real ones
// (jpeg_fill_bit_buffer sets it on exactly such a request).
struct Bits {
    Src s;
    uint64_t buf = 0;  // left-aligned
    int cnt = 0;       // bits in buf (real ones, then zeros once marker != 0)
    int real = 0;      // real bits among them
    int marker = 0;    // cinfo->unread_marker
    bool insufficient = false;

    void fill()
    {
        while (cnt <= 56) {
            int c = 0;
            if (!marker) {
                c = s.byte();
                if (c == 0xFF) {
                    do c = s.byte();
                    while (c == 0xFF);
                    if (c == 0) {
                        c = 0xFF;
                    } else {
                        marker = c;
                        c = 0;
                    }
                }
                if (!marker) real += 8;
            }
            buf |= (uint64_t)c << (56 - cnt);
            cnt += 8;
        }
    }
    uint32_t peek(int n)  // n <= 32
    {
        if (cnt < n) fill();
        return (uint32_t)(buf >> (64 - n));
    }
    void skip(int n)
    {
        if (n > real) insufficient = true;
        real = real > n ? real - n : 0;
        buf <<= n;
        cnt -= n;
    }
    int get(int n)
    {
        if (n == 0) return 0;
        const int v = (int)peek(n);
        skip(n);
        return v;
    }
    // HUFF_DECODE / jpeg_huff_decode over real bits then zeros
    int decode(const Table& t)
    {
        const uint32_t w = peek(17);
        const uint16_t e = t.look[w >> (17 - LOOK)];
        if (e) {
            skip(e >> 8);
            return e & 255;
        }
        for (int l = LOOK + 1; l <= 16; l++) {
            const int32_t code = (int32_t)(w >> (17 - l));
            if (code <= t.maxcode[l]) {
                skip(l);
                return t.vals[(t.valoff[l] + code) & 255];
            }
        }
        // also the codes shorter than LOOK bits that match nothing: the
        // canonical walk ends at length 17 (maxcode[17]) with symbol 0
        skip(17);
        return 0;
    }
    // jdmarker.c next_marker
    void next_marker()
    {
        for (;;) {
            int c = s.byte();
            while (c != 0xFF) c = s.byte();
            do c = s.byte();
            while (c == 0xFF);
            if (c != 0) {
                marker = c;
                return;
            }
        }
    }
    // jdmarker.c jpeg_resync_to_restart
    void resync(int desired)
    {
        for (;;) {
            const int m = marker;
            int action;
            if (m < 0xC0) action = 2;
            else if (m < 0xD0 || m > 0xD7) action = 3;
            else if (m == 0xD0 + ((desired + 1) & 7) || m == 0xD0 + ((desired + 2) & 7)) action = 3;
            else if (m == 0xD0 + ((desired - 1) & 7) || m == 0xD0 + ((desired - 2) & 7)) action = 2;
            else action = 1;
            if (action == 1) {
                marker = 0;
                return;
            }
            if (action == 3) return;
            next_marker();
        }
    }
    // jdhuff.c process_restart (the caller resets the DC predictors)
    void restart(int& next_rst)
    {
        buf = 0;
        cnt = real = 0;
        if (!marker) next_marker();
        if (marker == 0xD0 + next_rst) marker = 0;
        else resync(next_rst);
        next_rst = (next_rst + 1) & 7;
        if (!marker) insufficient = false;
    }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// jdapimin.c jpeg_finish_decompress -> jdinput.c consume_markers ->
// jdmarker.c read_markers after the file's only scan, up to EOI: the JDK
// reader runs it once every scanline is read (imageioJPEG.c readImage), and
// an error there throws.  Table segments are only checked (no scan follows);
// past the end of the file the fake EOI ends the walk.
bool trailer_ok(Bits& B)
{
    Src& s = B.s;
    auto rd2 = [&s]() {
        const int a = s.byte();
        return (a << 8) | s.byte();
    };
    for (;;) {
        if (!B.marker) B.next_marker();
        const int m = B.marker;
        B.marker = 0;
        if (m == 0xD9) return true;                              // EOI
        if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;      // RSTn, TEM
        if (m == 0xD8) return false;                             // JERR_SOI_DUPLICATE
        if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xCC) return false;  // SOF duplicate / unsupported
        if (m == 0xDA) return false;                             // JERR_EOI_EXPECTED (a one-scan file)
        if (m == 0xC4) {                                         // get_dht
            long len = rd2() - 2;
            while (len > 16) {
                int index = s.byte(), count = 0;
                for (int i = 0; i < 16; i++) count += s.byte();
                len -= 17;
                if (count > 256 || count > len) return false;    // JERR_BAD_HUFF_TABLE
                for (int i = 0; i < count; i++) s.byte();
                len -= count;
                if (index & 0x10) index -= 0x10;
                if (index >= 4) return false;                    // JERR_DHT_INDEX
            }
            if (len != 0) return false;                          // JERR_BAD_LENGTH
        } else if (m == 0xDB) {                                  // get_dqt
            long len = rd2() - 2;
            while (len > 0) {
                const int n = s.byte();
                if ((n & 15) >= 4) return false;                 // JERR_DQT_INDEX
                for (int i = 0; i < ((n >> 4) ? 128 : 64); i++) s.byte();
                len -= (n >> 4) ? 129 : 65;
            }
            if (len != 0) return false;
        } else if (m == 0xDD) {                                  // get_dri
            if (rd2() != 4) return false;
            rd2();
        } else if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE || m == 0xCC || m == 0xDC) {
            const long len = rd2() - 2;                          // APPn, COM, DAC, DNL: skip_variable
            for (long i = 0; i < len; i++) s.byte();
        } else {
            return false;                                        // JERR_UNKNOWN_MARKER
        }
    }
}

}  // namespace

icx_status seq_decode(const uint8_t* p, size_t len, const JpegHeader& J, int16_t* coefs, int32_t* dc)
{
    if (J.progressive || J.scan_off > len) return ICX_E_INVALID;
    const int nc = J.ncomp;
    const int hs = nc == 3 ? J.hs[0] : 1, vs = nc == 3 ? J.vs[0] : 1;
    const int nby = nc == 3 ? hs * vs : 1;
    const int nbmcu = nc == 3 ? nby + 2 : nc == 4 ? 4 : 1;
    const int64_t mcux = (J.w + 8 * hs - 1) / (8 * hs), mcuy = (J.h + 8 * vs - 1) / (8 * vs);
    // the distinct tables of the scan
    Table T[2][4];
    bool built[2][4] = {};
    int comp_of[10];
    for (int k = 0; k < nbmcu; k++) comp_of[k] = nc == 1 ? 0 : nc == 4 ? k : (k < nby ? 0 : k - nby + 1);
    for (int c = 0; c < nc; c++)
        for (int ac = 0; ac < 2; ac++) {
            const int id = ac ? J.ta[c] : J.td[c];
            if (built[ac][id]) continue;
            if (!J.h_ok[ac][id] || !build(J.hbits[ac][id], J.hvals[ac][id], J.hn[ac][id], !ac, T[ac][id]))
                return ICX_E_CORRUPT;  // JERR_BAD_HUFF_TABLE / JERR_NO_HUFF_TABLE: the JDK reader throws
            built[ac][id] = true;
        }
    Bits B{Src{p + J.scan_off, len - J.scan_off, 0}};
    int last_dc[4] = {0, 0, 0, 0}, next_rst = 0;
    const int64_t nmcu = mcux * mcuy;
    memset(coefs, 0, (size_t)(nmcu * nbmcu) * 128);
    int16_t* blk = coefs;
    for (int64_t m = 0; m < nmcu; m++, blk += 64 * nbmcu) {
        if (J.ri && m > 0 && m % J.ri == 0) {
            B.restart(next_rst);
            last_dc[0] = last_dc[1] = last_dc[2] = last_dc[3] = 0;
        }
        if (B.insufficient) {  // the rest of the segment stays zero
            for (int k = 0; k < nbmcu; k++) dc[m * nbmcu + k] = 0;
            continue;
        }
        for (int k = 0; k < nbmcu; k++) {
            const int c = comp_of[k];
            int16_t* b = blk + 64 * k;
            int v = B.decode(T[0][J.td[c]]);
            if (v) v = extend(B.get(v), v);
            last_dc[c] = (int)((unsigned)last_dc[c] + (unsigned)v);  // jdhuff.c: int, wraps as the JDK's C does
            b[0] = (int16_t)last_dc[c];
            dc[m * nbmcu + k] = b[0];
            const Table& A = T[1][J.ta[c]];
            for (int z = 1; z < 64; z++) {
                const int rs = B.decode(A);
                const int r = rs >> 4, sz = rs & 15;
                if (sz) {
                    z += r;
                    b[kNat[z]] = (int16_t)extend(B.get(sz), sz);
                } else {
                    if (r != 15) break;
                    z += 15;
                }
            }
        }
    }
    return trailer_ok(B) ? ICX_OK : ICX_E_CORRUPT;
}

}  // namespace icx

extern "C" icx_status icx_debug_recovery_coefs(const uint8_t* data, size_t len, int16_t* coefs, size_t ncoefs)
{
    using namespace icx;
    if (!data || !coefs) return ICX_E_NULL;
    JpegHeader J;
    icx_status s = parse_jpeg(data, len, len, J);
    if (s != ICX_OK) return s;
    if (J.progressive) return ICX_E_INVALID;
    const int hs = J.ncomp == 3 ? J.hs[0] : 1, vs = J.ncomp == 3 ? J.vs[0] : 1;
    const int nbmcu = J.ncomp == 3 ? hs * vs + 2 : J.ncomp == 4 ? 4 : 1;
    const size_t nb = (size_t)((J.w + 8 * hs - 1) / (8 * hs)) * ((J.h + 8 * vs - 1) / (8 * vs)) * nbmcu;
    if (nb * 64 > ncoefs) return ICX_E_BUFFER;
    std::vector<int32_t> dc(nb);
    return seq_decode(data, len, J, coefs, dc.data());
}
