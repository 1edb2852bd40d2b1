/*
 * icx_oracle_decode.c — scalar CPU restatement of the reference's JPEG decode
 * (row A11 of SURVEY.md §8a).  TEST INFRASTRUCTURE ONLY (see icx_oracle.h):
 * the checker for the device decoder; never linked into libicx.so.
 *
 * Reference call site: ImageCompression.decodeImageWithSubsampling
 * (core/ImageCompression.java:107-165) reads a JPEG through javax.imageio's
 * JPEGImageReader with ImageReadParam.setSourceSubsampling(s, s, 0, 0)
 * (:150-153) and ignoreMetadata = true (:126).  The arithmetic lives in the
 * JDK's bundled IJG libjpeg 6b (absent from /root/reference); this file
 * restates its published baseline decompression algorithm:
 *   jdmarker.c   SOI/APPn/DQT/DHT/SOF0-1/DRI/SOS parsing
 *   jdhuff.c     decode_mcu: canonical Huffman decode, HUFF_EXTEND, DC
 *                prediction per component reset at every restart interval
 *   jidctint.c   jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2) with the
 *                post-IDCT range-limit table of jdmaster.c
 *   jdcoefct.c   IDCT only for real (non-dummy) blocks
 *   jdsample.c   h2v2/h2v1 "fancy" (triangle) upsampling when
 *                downsampled_width > 2, else box replication; context rows
 *                replicate the first / last real sample row (jdmainct.c)
 *   jdcolor.c    ycc_rgb_convert (SCALEBITS 16 tables); for 4-component
 *                files (jdapimin.c: Adobe transform 0 or no marker -> CMYK,
 *                other transforms -> YCCK) ycck_cmyk_convert or CMYK as stored
 * then keeps pixels (x*s, y*s) as the JDK reader does for source subsampling
 * and returns TYPE_3BYTE_BGR (3 components) or TYPE_BYTE_GRAY.  CMYK / YCCK
 * (SURVEY §8f rank 4): the reference reads them through TwelveMonkeys, whose
 * ICC CMYK -> RGB conversion cannot be restated here (no profile, no CMM:
 * parity unpinned); the RGB step restated is the one the build's host path
 * used before (Pillow: the samples read as Adobe-inverted CMYK, then
 * cmyk2rgb), and oracle_jpeg_decode_cmyk gives libjpeg's CMYK samples, which
 * libjpeg-turbo pins (tests/golden/gen_cmyk_golden.py).
 *
 * Pinned against libjpeg-turbo 3.1.4 (6b API level, via Pillow) decodes of
 * tests/golden/decode/ (gen_decode_golden.py).
 */
#include <stdlib.h>
#include <string.h>

#include "icx_oracle.h"

typedef struct {
    int32_t maxcode[18]; /* largest code of length l, -1 if none; [17] ends the search */
    int32_t valoff[17];  /* huffval index of the first code of length l minus that code */
    uint8_t vals[256];
    int nvals;
    uint8_t look_nbits[256]; /* jdhuff.c HUFF_LOOKAHEAD (8) tables: length of the code */
    uint8_t look_sym[256];   /* starting with these 8 bits (0: longer / none), its symbol */
    int present;
    int bad; /* fails jpeg_make_d_derived_tbl: an error only if the scan uses it */
} dhuff_t;

typedef struct {
    int w, h, ncomp, ri;
    int rgb; /* 3 components stored as R, G, B (colour_space below): no ycc_rgb_convert */
    int cmyk; /* 4 components: 1 CMYK, 2 YCCK */
    int id[4], hs[4], vs[4], tq[4], td[4], ta[4];
    int hmax, vmax, mcux, mcuy;
    uint16_t qt[4][64]; /* natural order */
    int qt_present[4];
    dhuff_t dc[4], ac[4];
    const uint8_t* scan; /* first byte of the entropy-coded segment */
    size_t scan_len;
} jinfo_t;

static const int ZZ_NAT[64 + 16] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    /* jpeg_natural_order's safety tail: corrupt runs past 63 land on 63 */
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

static int build_dhuff(const uint8_t* counts, const uint8_t* vals, int nvals, dhuff_t* t)
{
    /* jdhuff.c jpeg_make_d_derived_tbl: canonical codes, length by length; the
     * codes of a length must leave room below the all-ones code (code < 2^l
     * after them), else JERR_BAD_HUFF_TABLE */
    int code = 0, k = 0;
    memset(t, 0, sizeof(*t));
    for (int l = 1; l <= 16; l++) {
        int n = counts[l - 1];
        t->valoff[l] = k - code;
        for (int i = 0; i < n; i++, code++, k++) {
            if (l <= 8) { /* look-ahead entries of every 8-bit string starting with this code */
                int lb = code << (8 - l);
                for (int f = 0; f < (1 << (8 - l)); f++) {
                    t->look_nbits[lb + f] = (uint8_t)l;
                    t->look_sym[lb + f] = vals[k];
                }
            }
        }
        t->maxcode[l] = n ? code - 1 : -1;
        if (code >= (1 << l)) return 6;
        code <<= 1;
    }
    t->maxcode[17] = 0xFFFFF; /* jdhuff.c: ensures jpeg_huff_decode terminates */
    if (k != nvals) return 6;
    memcpy(t->vals, vals, (size_t)nvals);
    t->nvals = nvals;
    t->present = 1;
    return 0;
}

/* Colour space of a 3-component file as the JDK reader settles it: libjpeg's
 * guess (jdapimin.c default_decompress_parms: JFIF -> YCbCr; an Adobe marker's
 * transform 0 -> RGB, else YCbCr; no marker: ids 1,2,3 -> YCbCr, 'R','G','B'
 * -> RGB, else YCbCr), then OpenJDK imageioJPEG.c's override of a YCbCr guess:
 * an Adobe marker with a transform other than 1 -> unknown (here: unsupported,
 * -1), also next to a JFIF marker; no JFIF and no EXIF marker (IS_EXIF: the
 * first saved COM/APPn marker is an APP1), ids other than 1,2,3 and every
 * component sampled alike -> RGB.  0 YCbCr, 1 RGB. */
static int colour_space(const jinfo_t* J, int jfif, int exif, int adobe, int transform)
{
    /* libjpeg's guess */
    int ycc;
    if (jfif) ycc = 1;
    else if (adobe) ycc = transform != 0;
    else ycc = !(J->id[0] == 'R' && J->id[1] == 'G' && J->id[2] == 'B');
    if (!ycc) return 1;
    /* imageioJPEG.c's override of a YCbCr guess: an Adobe marker whose
     * transform is not 1 -> unknown, even next to a JFIF marker; else, with
     * neither JFIF nor EXIF, ids 1,2,3 keep YCbCr and equal sampling -> RGB */
    if (adobe) return transform == 1 ? 0 : -1;
    if (jfif || exif) return 0;
    if (J->id[0] == 1 && J->id[1] == 2 && J->id[2] == 3) return 0;
    return J->hs[1] == J->hs[0] && J->hs[2] == J->hs[0] && J->vs[1] == J->vs[0] && J->vs[2] == J->vs[0];
}

/* jdmarker.c, baseline subset.  0 ok, 5 unsupported, 6 corrupt. */
static int parse(const uint8_t* p, size_t len, jinfo_t* J)
{
    memset(J, 0, sizeof(*J));
    if (len < 4 || p[0] != 0xFF || p[1] != 0xD8) return 6;
    size_t i = 2;
    int have_sof = 0, jfif = 0, exif = 0, adobe = 0, transform = 0, saved_any = 0;
    for (;;) {
        while (i < len && p[i] != 0xFF) i++; /* jdmarker next_marker: skip garbage */
        while (i < len && p[i] == 0xFF) i++; /* fill bytes */
        if (i >= len) return 6;
        int m = p[i++];
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) return 6; /* EOI before SOS */
        if (i + 2 > len) return 6;
        size_t seg = ((size_t)p[i] << 8) | p[i + 1];
        if (seg < 2 || i + seg > len) return 6;
        const uint8_t* s = p + i + 2;
        size_t n = seg - 2;
        i += seg;
        /* imageioJPEG.c IS_EXIF: the first marker the reader saves (COM,
         * APP0..15) is an APP1, whatever it holds */
        if (!saved_any && (m == 0xFE || (m >= 0xE0 && m <= 0xEF))) {
            saved_any = 1;
            exif = m == 0xE1;
        }
        if (m == 0xDB) { /* DQT */
            size_t o = 0;
            while (o < n) {
                int pq = s[o] >> 4, tq = s[o] & 15;
                if (tq > 3 || pq > 1) return 6;
                size_t need = 1 + (pq ? 128 : 64);
                if (o + need > n) return 6;
                for (int k = 0; k < 64; k++)
                    J->qt[tq][ZZ_NAT[k]] = pq ? (uint16_t)((s[o + 1 + 2 * k] << 8) | s[o + 2 + 2 * k])
                                              : s[o + 1 + k];
                J->qt_present[tq] = 1;
                o += need;
            }
        } else if (m == 0xC4) { /* DHT */
            size_t o = 0;
            while (o < n) {
                if (o + 17 > n) return 6;
                int tc = s[o] >> 4, th = s[o] & 15;
                if (tc > 1 || th > 3) return 6;
                int tot = 0;
                for (int l = 0; l < 16; l++) tot += s[o + 1 + l];
                if (tot > 256 || o + 17 + (size_t)tot > n) return 6;
                dhuff_t* t = tc ? &J->ac[th] : &J->dc[th];
                if (build_dhuff(s + o + 1, s + o + 17, tot, t)) {
                    memset(t, 0, sizeof(*t));
                    t->present = t->bad = 1;
                }
                o += 17 + (size_t)tot;
            }
        } else if (m == 0xC0 || m == 0xC1) { /* SOF0 / SOF1: sequential Huffman */
            if (n < 6) return 6;
            if (s[0] != 8) { /* jdinput.c initial_setup: JERR_BAD_PRECISION (6b is built 8-bit) */
                J->h = (s[1] << 8) | s[2];
                J->w = (s[3] << 8) | s[4];
                J->ncomp = s[5];
                return 8;
            }
            J->h = (s[1] << 8) | s[2];
            J->w = (s[3] << 8) | s[4];
            J->ncomp = s[5];
            if (J->w == 0 || J->h == 0) return 5; /* DNL-defined height */
            if (J->ncomp != 1 && J->ncomp != 3 && J->ncomp != 4) return 5;
            if (n < 6 + 3 * (size_t)J->ncomp) return 6;
            for (int c = 0; c < J->ncomp; c++) {
                J->id[c] = s[6 + 3 * c];
                J->hs[c] = s[7 + 3 * c] >> 4;
                J->vs[c] = s[7 + 3 * c] & 15;
                J->tq[c] = s[8 + 3 * c];
                if (J->tq[c] > 3 || J->hs[c] < 1 || J->vs[c] < 1) return 6;
            }
            have_sof = 1;
        } else if ((m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)) {
            if (n >= 6) { /* progressive / lossless / hierarchical / arithmetic: dims only */
                J->h = (s[1] << 8) | s[2];
                J->w = (s[3] << 8) | s[4];
                J->ncomp = s[5];
            }
            /* refused by the JDK's 6b reader: arithmetic coding (SOF9-11:
             * jdmaster.c JERR_ARITH_NOTIMPL), hierarchical (SOF5-7, 13-15:
             * jdmarker.c JERR_SOF_UNSUPPORTED), a progressive file of another
             * precision (JERR_BAD_PRECISION).  SOF2 (8-bit) and SOF3
             * (lossless: TwelveMonkeys' own decoder) are read, just not here */
            if (m != 0xC2 && m != 0xC3) return 8;
            if (m == 0xC2 && n >= 1 && s[0] != 8) return 8;
            return 5;
        } else if (m == 0xDD) { /* DRI */
            if (n < 2) return 6;
            J->ri = (s[0] << 8) | s[1];
        } else if (m == 0xE0) { /* APP0: JFIF (jdmarker.c examine_app0) */
            if (n >= 5 && !memcmp(s, "JFIF\0", 5)) jfif = 1;
        } else if (m == 0xEE) { /* APP14: Adobe (jdmarker.c examine_app14) */
            if (n >= 12 && !memcmp(s, "Adobe", 5)) {
                adobe = 1;
                transform = s[11];
            }
        } else if (m == 0xDA) { /* SOS */
            if (!have_sof) return 6;
            int ns = s[0];
            if (ns != J->ncomp || n < 1 + 2 * (size_t)ns + 3) return 5; /* single interleaved scan */
            for (int k = 0; k < ns; k++) {
                int cid = s[1 + 2 * k], c;
                for (c = 0; c < J->ncomp && J->id[c] != cid; c++) {}
                if (c != k) return 5;
                J->td[c] = s[2 + 2 * k] >> 4;
                J->ta[c] = s[2 + 2 * k] & 15;
                if (J->td[c] > 3 || J->ta[c] > 3) return 6;
            }
            if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0) return 5;
            J->scan = p + i;
            J->scan_len = len - i;
            break;
        }
        /* APPn, COM, DNL, ...: skipped (ignoreMetadata = true, ImageCompression.java:126) */
    }
    /* sampling: colour = Y (1|2 x 1|2) with Cb, Cr at 1x1 except 1x2 (4:4:0,
     * whose 6b upsampler is not the one libjpeg-turbo uses); grey = any */
    J->hmax = J->vmax = 1;
    if (J->ncomp == 4) { /* CMYK / YCCK: one block per component per MCU only */
        J->cmyk = adobe && transform != 0 ? 2 : 1;
        for (int c = 0; c < 4; c++)
            if (J->hs[c] != 1 || J->vs[c] != 1) return 5;
        J->mcux = (J->w + 7) / 8;
        J->mcuy = (J->h + 7) / 8;
    } else if (J->ncomp == 3) {
        int cs = colour_space(J, jfif, exif, adobe, transform);
        if (cs < 0) return 5;
        J->rgb = cs;
        if (J->hs[1] != 1 || J->vs[1] != 1 || J->hs[2] != 1 || J->vs[2] != 1) return 5;
        /* Y 1x1, 2x1, 2x2 (fancy upsampling), 1x2 (4:4:0) and 4x1 (4:1:1):
         * int_upsample replication (jdsample.c jinit_upsampler) */
        {
            const int hy = J->hs[0], vy = J->vs[0];
            if (!((hy == 1 && vy == 1) || (hy == 2 && vy == 1) || (hy == 2 && vy == 2) || (hy == 1 && vy == 2) ||
                  (hy == 4 && vy == 1)))
                return 5;
        }
        J->hmax = J->hs[0];
        J->vmax = J->vs[0];
        J->mcux = (J->w + 8 * J->hmax - 1) / (8 * J->hmax);
        J->mcuy = (J->h + 8 * J->vmax - 1) / (8 * J->vmax);
    } else { /* non-interleaved single component: one block per MCU */
        J->hs[0] = J->vs[0] = 1;
        J->mcux = (J->w + 7) / 8;
        J->mcuy = (J->h + 7) / 8;
    }
    for (int c = 0; c < J->ncomp; c++) {
        if (!J->qt_present[J->tq[c]] || !J->dc[J->td[c]].present || !J->ac[J->ta[c]].present) return 6;
        if (J->dc[J->td[c]].bad || J->ac[J->ta[c]].bad) return 6;
        /* jdhuff.c jpeg_make_d_derived_tbl: a DC table's symbols are 0..15 */
        const dhuff_t* t = &J->dc[J->td[c]];
        for (int k = 0; k < t->nvals; k++)
            if (t->vals[k] > 15) return 6;
    }
    return 0;
}

int oracle_jpeg_info(const uint8_t* jpg, size_t len, int* w, int* h, int* ncomp)
{
    jinfo_t J;
    int rc = parse(jpg, len, &J);
    if (rc == 0 || rc == 5 || rc == 8) {
        if (w) *w = J.w;
        if (h) *h = J.h;
        if (ncomp) *ncomp = J.ncomp;
    }
    return rc;
}

/* ------------------------------------------- jdhuff.c + jdmarker.c (6b) */
/* The entropy decoder reads the file from the first scan byte on through the
 * JDK's source manager (imageioJPEG.c imageio_fill_input_buffer), which on
 * end of stream warns and inserts a fake EOI marker (FF D9): past the end the
 * bytes read FF D9 FF D9 ...  (Pillow's LOAD_TRUNCATED_IMAGES does the same,
 * JpegImagePlugin.load_read, which is how libjpeg-turbo pins this below.) */
typedef struct {
    const uint8_t* p;
    size_t len, pos;
    uint64_t buf;     /* get_buffer: the low `bits` bits are unread */
    int bits;         /* bits_left */
    int marker;       /* cinfo->unread_marker: 0, or the marker the reader stopped at */
    int insufficient; /* entropy->insufficient_data */
    int next_rst;     /* marker->next_restart_num */
} src6_t;

#define MIN_GET_BITS 25 /* jdhuff.h: BIT_BUF_SIZE (32) - 7 */

static int rd_byte(src6_t* s)
{
    size_t i = s->pos++;
    if (i < s->len) return s->p[i];
    return ((i - s->len) & 1) ? 0xD9 : 0xFF;
}

/* jpeg_fill_bit_buffer: load bytes up to MIN_GET_BITS bits unless a marker
 * stops the reader (FF 00 is a data FF; FF FF... are fill bytes); once it has,
 * a request for more bits than are left warns (JWRN_HIT_MARKER), sets
 * insufficient_data and pads the buffer with zero bits. */
static void fill6(src6_t* s, int nbits)
{
    if (!s->marker) {
        while (s->bits < MIN_GET_BITS) {
            int c = rd_byte(s);
            if (c == 0xFF) {
                do c = rd_byte(s);
                while (c == 0xFF);
                if (c == 0) {
                    c = 0xFF;
                } else {
                    s->marker = c;
                    break;
                }
            }
            s->buf = (s->buf << 8) | (uint64_t)c;
            s->bits += 8;
        }
        if (!s->marker) return;
    }
    if (nbits > s->bits) {
        s->insufficient = 1;
        s->buf <<= MIN_GET_BITS - s->bits;
        s->bits = MIN_GET_BITS;
    }
}

static inline int get_bits6(src6_t* s, int n)
{
    s->bits -= n;
    return (int)((s->buf >> s->bits) & ((1u << n) - 1));
}

/* HUFF_DECODE + jpeg_huff_decode: the 8-bit look-ahead, else the canonical
 * maxcode walk from 9 bits (from 1 bit when fewer than 8 are left).  A bad
 * code (no match within 16 bits) has consumed 17 bits and decodes as symbol
 * 0 (JWRN_HUFF_BAD_CODE: "fake a zero as the safest result"). */
static int huff_decode6(src6_t* s, const dhuff_t* t)
{
    int l;
    if (s->bits < 8) {
        fill6(s, 0);
        if (s->bits < 8) {
            l = 1;
            goto slow;
        }
    }
    {
        const int look = (int)((s->buf >> (s->bits - 8)) & 0xFF);
        const int nb = t->look_nbits[look];
        if (nb) {
            s->bits -= nb;
            return t->look_sym[look];
        }
        l = 9;
    }
slow:
    if (s->bits < l) fill6(s, l);
    int code = get_bits6(s, l);
    while (code > t->maxcode[l]) {
        code <<= 1;
        if (s->bits < 1) fill6(s, 1);
        code |= get_bits6(s, 1);
        l++;
    }
    if (l > 16) return 0;
    return t->vals[(t->valoff[l] + code) & 0xFF];
}

static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

/* jdmarker.c next_marker: skip to the next FF, swallow fill FFs, skip FF 00
 * data pairs, stop at a marker */
static void next_marker6(src6_t* s)
{
    for (;;) {
        int c = rd_byte(s);
        while (c != 0xFF) c = rd_byte(s);
        do c = rd_byte(s);
        while (c == 0xFF);
        if (c != 0) {
            s->marker = c;
            return;
        }
    }
}

/* jdmarker.c jpeg_resync_to_restart: the reader met marker `marker` where
 * RST`desired` was due.  1: discard it and resume; 2: scan to the next marker
 * and decide again; 3: leave it (the entropy decoder then sees an empty
 * segment) */
static void resync6(src6_t* s, int desired)
{
    for (;;) {
        const int m = s->marker;
        int action;
        if (m < 0xC0) action = 2; /* invalid marker */
        else if (m < 0xD0 || m > 0xD7) action = 3; /* a valid non-restart marker */
        else if (m == 0xD0 + ((desired + 1) & 7) || m == 0xD0 + ((desired + 2) & 7)) action = 3;
        else if (m == 0xD0 + ((desired - 1) & 7) || m == 0xD0 + ((desired - 2) & 7)) action = 2;
        else action = 1; /* the desired restart, or too far away */
        if (action == 1) {
            s->marker = 0;
            return;
        }
        if (action == 3) return;
        next_marker6(s);
    }
}

/* jdhuff.c process_restart: drop the bit buffer, read_restart_marker (the
 * expected RSTn is swallowed, anything else resynchronises), reset the DC
 * predictors; insufficient_data is cleared only when no marker is left
 * pending (else the next segment is treated as empty) */
static void process_restart6(src6_t* s, int* last_dc)
{
    s->bits = 0;
    if (!s->marker) next_marker6(s);
    if (s->marker == 0xD0 + s->next_rst) s->marker = 0;
    else resync6(s, s->next_rst);
    s->next_rst = (s->next_rst + 1) & 7;
    last_dc[0] = last_dc[1] = last_dc[2] = last_dc[3] = 0;
    if (!s->marker) s->insufficient = 0;
}

/* jdapimin.c jpeg_finish_decompress -> jdinput.c consume_markers ->
 * jdmarker.c read_markers after the file's only scan, up to EOI: the JDK
 * reader runs it once every scanline is read (imageioJPEG.c readImage), and
 * an error there throws (status 6).  Past the end of the file the fake EOI
 * ends it. */
static int rd2(src6_t* s)
{
    const int a = rd_byte(s);
    return (a << 8) | rd_byte(s);
}

static int trailer6(src6_t* s)
{
    for (;;) {
        if (!s->marker) next_marker6(s);
        const int m = s->marker;
        s->marker = 0;
        if (m == 0xD9) return 0;                               /* EOI */
        if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;    /* RSTn, TEM: nothing */
        if (m == 0xD8) return 6;                               /* JERR_SOI_DUPLICATE */
        if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xCC) return 6; /* SOF / JPG: duplicate, unsupported */
        if (m == 0xDA) return 6;                               /* JERR_EOI_EXPECTED: a one-scan file */
        if (m == 0xC4) {                                       /* get_dht */
            long len = rd2(s) - 2;
            while (len > 16) {
                int index = rd_byte(s), count = 0;
                for (int i = 0; i < 16; i++) count += rd_byte(s);
                len -= 17;
                if (count > 256 || count > len) return 6;      /* JERR_BAD_HUFF_TABLE */
                for (int i = 0; i < count; i++) rd_byte(s);
                len -= count;
                if (index & 0x10) index -= 0x10;
                if (index >= 4) return 6;                      /* JERR_DHT_INDEX */
            }
            if (len != 0) return 6;                            /* JERR_BAD_LENGTH */
        } else if (m == 0xDB) {                                /* get_dqt */
            long len = rd2(s) - 2;
            while (len > 0) {
                const int n = rd_byte(s);
                if ((n & 15) >= 4) return 6;                   /* JERR_DQT_INDEX */
                for (int i = 0; i < 64; i++)
                    if (n >> 4) rd2(s);
                    else rd_byte(s);
                len -= (n >> 4) ? 129 : 65;
            }
            if (len != 0) return 6;
        } else if (m == 0xDD) {                                /* get_dri */
            if (rd2(s) != 4) return 6;
            rd2(s);
        } else if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE || m == 0xCC || m == 0xDC) {
            long len = rd2(s) - 2;                             /* APPn, COM, DAC, DNL: skipped */
            for (long i = 0; i < len; i++) rd_byte(s);
        } else {
            return 6;                                          /* JERR_UNKNOWN_MARKER */
        }
    }
}

/* Decode the scan into quantised coefficients, natural order, scan (MCU) block
 * order including dummy blocks, as jdhuff.c decode_mcu fills the zeroed
 * MCU_buffer (jdcoefct.c decompress_onepass): once insufficient_data is set
 * (bits wanted past a marker or the end of the file: the MCU being decoded
 * finishes on zero bits) every later MCU of the segment stays zero, i.e.
 * uniform grey; a bad Huffman code decodes as 0.  Then the markers up to EOI
 * (trailer6): 6 where the JDK reader would throw there, else 0. */
static int decode_scan(const jinfo_t* J, int16_t* coefs)
{
    src6_t s = {J->scan, J->scan_len, 0, 0, 0, 0, 0, 0};
    int nb_mcu = J->ncomp == 3 ? J->hs[0] * J->vs[0] + 2 : J->ncomp == 4 ? 4 : 1;
    int comp_of[10];
    for (int k = 0; k < nb_mcu; k++)
        comp_of[k] = J->ncomp == 1 ? 0 : J->ncomp == 4 ? k : (k < nb_mcu - 2 ? 0 : k - (nb_mcu - 3));
    long nmcu = (long)J->mcux * J->mcuy;
    int last_dc[4] = {0, 0, 0, 0};
    int16_t* blk = coefs;
    memset(coefs, 0, (size_t)nmcu * nb_mcu * 64 * sizeof(int16_t));
    for (long m = 0; m < nmcu; m++, blk += 64 * nb_mcu) {
        if (J->ri && m > 0 && m % J->ri == 0) process_restart6(&s, last_dc); /* restarts_to_go == 0 */
        if (s.insufficient) continue;
        for (int k = 0; k < nb_mcu; k++) {
            const int c = comp_of[k];
            int16_t* b = blk + 64 * k;
            int v = huff_decode6(&s, &J->dc[J->td[c]]);
            if (v) {
                if (s.bits < v) fill6(&s, v);
                v = extend(get_bits6(&s, v), v);
            }
            last_dc[c] += v;
            b[0] = (int16_t)last_dc[c];
            for (int z = 1; z < 64; z++) {
                const int rs = huff_decode6(&s, &J->ac[J->ta[c]]);
                const int r = rs >> 4, sz = rs & 15;
                if (sz) {
                    z += r;
                    if (s.bits < sz) fill6(&s, sz);
                    b[ZZ_NAT[z]] = (int16_t)extend(get_bits6(&s, sz), sz);
                } else {
                    if (r != 15) break;
                    z += 15;
                }
            }
        }
    }
    return trailer6(&s);
}

/* ------------------------------------------------------------ jidctint.c */
#define CONST_BITS 13
#define PASS1_BITS 2
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

static inline uint8_t idct_limit(int v)
{
    /* IDCT_range_limit(cinfo)[v & RANGE_MASK] of jdmaster.c prepare_range_limit_table */
    int x = v & 1023;
    if (x < 128) return (uint8_t)(x + 128);
    if (x < 512) return 255;
    if (x < 896) return 0;
    return (uint8_t)(x - 896);
}

static void idct_islow(const int16_t* in, const uint16_t* qt, uint8_t* out, int ostride)
{
    int ws[64];
    for (int c = 0; c < 8; c++) { /* pass 1: columns */
        int d[8];
        for (int r = 0; r < 8; r++) d[r] = in[r * 8 + c] * qt[r * 8 + c];
        int z2 = d[2], z3 = d[6];
        int z1 = (z2 + z3) * 4433;                 /* FIX_0_541196100 */
        int t2 = z1 + z3 * (-15137);               /* FIX_1_847759065 */
        int t3 = z1 + z2 * 6270;                   /* FIX_0_765366865 */
        int t0 = (d[0] + d[4]) << CONST_BITS;
        int t1 = (d[0] - d[4]) << CONST_BITS;
        int t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        int o0 = d[7], o1 = d[5], o2 = d[3], o3 = d[1];
        int zz1 = o0 + o3, zz2 = o1 + o2, zz3 = o0 + o2, zz4 = o1 + o3;
        int z5 = (zz3 + zz4) * 9633;               /* FIX_1_175875602 */
        o0 *= 2446; o1 *= 16819; o2 *= 25172; o3 *= 12299;
        zz1 *= -7373; zz2 *= -20995; zz3 *= -16069; zz4 *= -3196;
        zz3 += z5; zz4 += z5;
        o0 += zz1 + zz3; o1 += zz2 + zz4; o2 += zz2 + zz3; o3 += zz1 + zz4;
        ws[0 * 8 + c] = DESCALE(t10 + o3, CONST_BITS - PASS1_BITS);
        ws[7 * 8 + c] = DESCALE(t10 - o3, CONST_BITS - PASS1_BITS);
        ws[1 * 8 + c] = DESCALE(t11 + o2, CONST_BITS - PASS1_BITS);
        ws[6 * 8 + c] = DESCALE(t11 - o2, CONST_BITS - PASS1_BITS);
        ws[2 * 8 + c] = DESCALE(t12 + o1, CONST_BITS - PASS1_BITS);
        ws[5 * 8 + c] = DESCALE(t12 - o1, CONST_BITS - PASS1_BITS);
        ws[3 * 8 + c] = DESCALE(t13 + o0, CONST_BITS - PASS1_BITS);
        ws[4 * 8 + c] = DESCALE(t13 - o0, CONST_BITS - PASS1_BITS);
    }
    for (int r = 0; r < 8; r++) { /* pass 2: rows */
        const int* d = ws + r * 8;
        int z2 = d[2], z3 = d[6];
        int z1 = (z2 + z3) * 4433;
        int t2 = z1 + z3 * (-15137);
        int t3 = z1 + z2 * 6270;
        int t0 = (d[0] + d[4]) << CONST_BITS;
        int t1 = (d[0] - d[4]) << CONST_BITS;
        int t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
        int o0 = d[7], o1 = d[5], o2 = d[3], o3 = d[1];
        int zz1 = o0 + o3, zz2 = o1 + o2, zz3 = o0 + o2, zz4 = o1 + o3;
        int z5 = (zz3 + zz4) * 9633;
        o0 *= 2446; o1 *= 16819; o2 *= 25172; o3 *= 12299;
        zz1 *= -7373; zz2 *= -20995; zz3 *= -16069; zz4 *= -3196;
        zz3 += z5; zz4 += z5;
        o0 += zz1 + zz3; o1 += zz2 + zz4; o2 += zz2 + zz3; o3 += zz1 + zz4;
        const int SH = CONST_BITS + PASS1_BITS + 3;
        uint8_t* o = out + (size_t)r * ostride;
        o[0] = idct_limit(DESCALE(t10 + o3, SH));
        o[7] = idct_limit(DESCALE(t10 - o3, SH));
        o[1] = idct_limit(DESCALE(t11 + o2, SH));
        o[6] = idct_limit(DESCALE(t11 - o2, SH));
        o[2] = idct_limit(DESCALE(t12 + o1, SH));
        o[5] = idct_limit(DESCALE(t12 - o1, SH));
        o[3] = idct_limit(DESCALE(t13 + o0, SH));
        o[4] = idct_limit(DESCALE(t13 - o0, SH));
    }
}

/* ------------------------------------------------------------- jdcolor.c */
static inline uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

long oracle_jpeg_num_blocks(const uint8_t* jpg, size_t len)
{
    jinfo_t J;
    if (parse(jpg, len, &J)) return -1;
    int nb = J.ncomp == 3 ? J.hs[0] * J.vs[0] + 2 : J.ncomp == 4 ? 4 : 1;
    return (long)J.mcux * J.mcuy * nb;
}

int oracle_jpeg_coefs(const uint8_t* jpg, size_t len, int16_t* coefs, size_t nblocks)
{
    jinfo_t J;
    int rc = parse(jpg, len, &J);
    if (rc) return rc;
    int nb = J.ncomp == 3 ? J.hs[0] * J.vs[0] + 2 : J.ncomp == 4 ? 4 : 1;
    if ((size_t)J.mcux * J.mcuy * nb > nblocks) return 4;
    return decode_scan(&J, coefs);
}

/* Sample planes of a 4-component file (every component 1x1): coefficients,
 * then the ISLOW IDCT of each block into its plane (pw x ph, pitch pw). */
static int cmyk_planes(const jinfo_t* J, uint8_t* plane[4], int* pitch)
{
    long nblk = (long)J->mcux * J->mcuy * 4;
    int16_t* coefs = (int16_t*)malloc((size_t)nblk * 64 * sizeof(int16_t));
    if (!coefs) return 2;
    int rc = decode_scan(J, coefs);
    if (rc) {
        free(coefs);
        return rc;
    }
    int pw = J->mcux * 8, ph = J->mcuy * 8;
    *pitch = pw;
    for (int c = 0; c < 4; c++) plane[c] = (uint8_t*)malloc((size_t)pw * ph);
    const int16_t* blk = coefs;
    for (int my = 0; my < J->mcuy; my++)
        for (int mx = 0; mx < J->mcux; mx++)
            for (int c = 0; c < 4; c++, blk += 64)
                idct_islow(blk, J->qt[J->tq[c]], plane[c] + (size_t)my * 8 * pw + mx * 8, pw);
    free(coefs);
    return 0;
}

/* libjpeg's CMYK sample of a pixel (jdcolor.c ycck_cmyk_convert for YCCK:
 * C, M, Y = range_limit[255 - (R, G, B of ycc_rgb_convert)], K as stored) */
static void cmyk_px(const jinfo_t* J, uint8_t* const plane[4], size_t at, int* v)
{
    int y = plane[0][at], c1 = plane[1][at], c2 = plane[2][at];
    v[3] = plane[3][at];
    if (J->cmyk == 2) {
        int cb = c1 - 128, cr = c2 - 128;
        v[0] = clamp255(255 - (y + ((91881 * cr + 32768) >> 16)));
        v[1] = clamp255(255 - (y + ((-22554 * cb + 32768 - 46802 * cr) >> 16)));
        v[2] = clamp255(255 - (y + ((116130 * cb + 32768) >> 16)));
    } else {
        v[0] = y;
        v[1] = c1;
        v[2] = c2;
    }
}

int oracle_jpeg_decode_cmyk(const uint8_t* jpg, size_t len, uint8_t* out, size_t cap, int* ow, int* oh)
{
    jinfo_t J;
    int rc = parse(jpg, len, &J);
    if (rc) return rc;
    if (J.ncomp != 4) return 1;
    *ow = J.w;
    *oh = J.h;
    if ((size_t)J.w * J.h * 4 > cap) return 4;
    uint8_t* plane[4];
    int pitch;
    if ((rc = cmyk_planes(&J, plane, &pitch))) return rc;
    for (int y = 0; y < J.h; y++)
        for (int x = 0; x < J.w; x++) {
            int v[4];
            cmyk_px(&J, plane, (size_t)y * pitch + x, v);
            for (int k = 0; k < 4; k++) out[((size_t)y * J.w + x) * 4 + k] = (uint8_t)v[k];
        }
    for (int c = 0; c < 4; c++) free(plane[c]);
    return 0;
}

/* luma_only: the first component's samples alone (GRAY8), as a reader asked
 * for JCS_GRAYSCALE output of a YCbCr file gives them (jdcolor.c
 * grayscale_convert) - what the 4:4:0 fixtures can pin */
static int decode_impl(const uint8_t* jpg, size_t len, int s, uint8_t* out, size_t cap, int* ow, int* oh,
                       int* ofmt, int luma_only)
{
    jinfo_t J;
    int rc = parse(jpg, len, &J);
    if (rc) return rc;
    if (s < 1) return 1;
    if (luma_only && J.ncomp != 3) return 1;
    int W = J.w, H = J.h;
    int dw = (W + s - 1) / s, dh = (H + s - 1) / s;
    int nch = J.ncomp == 1 || luma_only ? 1 : 3;
    *ow = dw;
    *oh = dh;
    *ofmt = nch == 3 ? OR_BGR24 : OR_GRAY8;
    if ((size_t)dw * dh * nch > cap) return 4;
    if (J.ncomp == 4) { /* to BGR: Pillow's read as Adobe-inverted CMYK, then cmyk2rgb */
        uint8_t* plane[4];
        int pitch;
        if ((rc = cmyk_planes(&J, plane, &pitch))) return rc;
        for (int y = 0; y < dh; y++)
            for (int x = 0; x < dw; x++) {
                int v[4];
                cmyk_px(&J, plane, (size_t)(y * s) * pitch + x * s, v);
                int nk = v[3]; /* 255 - (255 - K) */
                uint8_t* o = out + ((size_t)y * dw + x) * 3;
                for (int q = 0; q < 3; q++) {
                    int t = (255 - v[q]) * nk + 128;
                    o[2 - q] = clamp255(nk - (((t >> 8) + t) >> 8));
                }
            }
        for (int c = 0; c < 4; c++) free(plane[c]);
        return 0;
    }

    int nb_mcu = J.ncomp == 3 ? J.hs[0] * J.vs[0] + 2 : 1;
    long nblk = (long)J.mcux * J.mcuy * nb_mcu;
    int16_t* coefs = (int16_t*)malloc((size_t)nblk * 64 * sizeof(int16_t));
    if (!coefs) return 2;
    rc = decode_scan(&J, coefs);
    if (rc) {
        free(coefs);
        return rc;
    }
    /* component sample planes: width_in_blocks*8 x height_in_blocks*8; the
     * real part is downsampled_width x downsampled_height (jdmaster.c) */
    int cw[3], ch[3], pw[3], ph[3];
    uint8_t* plane[3] = {0, 0, 0};
    for (int c = 0; c < J.ncomp; c++) {
        cw[c] = (W * J.hs[c] + J.hmax - 1) / J.hmax;
        ch[c] = (H * J.vs[c] + J.vmax - 1) / J.vmax;
        pw[c] = (cw[c] + 7) / 8 * 8;
        ph[c] = (ch[c] + 7) / 8 * 8;
        plane[c] = (uint8_t*)malloc((size_t)pw[c] * ph[c]);
    }
    /* IDCT of the real blocks of every MCU (jdcoefct.c decompress_onepass) */
    const int16_t* blk = coefs;
    for (int my = 0; my < J.mcuy; my++)
        for (int mx = 0; mx < J.mcux; mx++)
            for (int c = 0; c < J.ncomp; c++)
                for (int by = 0; by < J.vs[c]; by++)
                    for (int bx = 0; bx < J.hs[c]; bx++, blk += 64) {
                        int X = (mx * J.hs[c] + bx) * 8, Y = (my * J.vs[c] + by) * 8;
                        if (X >= pw[c] || Y >= ph[c]) continue; /* dummy block */
                        idct_islow(blk, J.qt[J.tq[c]], plane[c] + (size_t)Y * pw[c] + X, pw[c]);
                    }
    free(coefs);

    if (nch == 1) {
        for (int y = 0; y < dh; y++)
            for (int x = 0; x < dw; x++) out[(size_t)y * dw + x] = plane[0][(size_t)(y * s) * pw[0] + x * s];
        for (int c = 0; c < J.ncomp; c++) free(plane[c]);
        return 0;
    }
    /* upsample Cb/Cr to full width/height rows (jdsample.c), then convert */
    int hx = J.hmax, vy = J.vmax;
    /* jdsample.c jinit_upsampler: h2v1 / h2v2 fancy when do_fancy &&
     * downsampled_width > 2, their box versions otherwise; any other integral
     * ratio (1x2 = 4:4:0, 4x1 = 4:1:1) int_upsample replication */
    int fancy = hx == 2 && cw[1] > 2;
    int fullw = cw[1] * hx;
    int* up[2];
    up[0] = (int*)malloc(sizeof(int) * (size_t)fullw * 2);
    up[1] = up[0] + fullw;
    for (int y = 0; y < dh; y++) {
        int Y = y * s; /* full-resolution output row */
        for (int k = 0; k < 2; k++) {
            const uint8_t* P = plane[1 + k];
            int stride = pw[1 + k];
            int* o = up[k];
            int r0 = Y / vy;
            if (hx == 1 && vy == 1) {
                for (int x = 0; x < cw[1]; x++) o[x] = P[(size_t)r0 * stride + x];
            } else if (!fancy) { /* h2v1_upsample / h2v2_upsample / int_upsample: replication */
                for (int x = 0; x < fullw; x++) o[x] = P[(size_t)r0 * stride + x / hx];
            } else if (vy == 1) { /* h2v1_fancy_upsample */
                const uint8_t* in = P + (size_t)r0 * stride;
                int n = cw[1];
                o[0] = in[0];
                o[1] = (in[0] * 3 + in[1] + 2) >> 2;
                for (int i = 1; i < n - 1; i++) {
                    o[2 * i] = (in[i] * 3 + in[i - 1] + 1) >> 2;
                    o[2 * i + 1] = (in[i] * 3 + in[i + 1] + 2) >> 2;
                }
                o[2 * n - 2] = (in[n - 1] * 3 + in[n - 2] + 1) >> 2;
                o[2 * n - 1] = in[n - 1];
            } else { /* h2v2_fancy_upsample with replicated context rows */
                int rn = (Y & 1) ? r0 + 1 : r0 - 1;
                if (rn < 0) rn = 0;
                if (rn > ch[1] - 1) rn = ch[1] - 1;
                const uint8_t* a = P + (size_t)r0 * stride;
                const uint8_t* b = P + (size_t)rn * stride;
                int n = cw[1];
                int cs0 = a[0] * 3 + b[0], cs1 = a[1] * 3 + b[1];
                o[0] = (cs0 * 4 + 8) >> 4;
                o[1] = (cs0 * 3 + cs1 + 7) >> 4;
                int last = cs0, cur = cs1;
                for (int i = 1; i < n - 1; i++) {
                    int nxt = a[i + 1] * 3 + b[i + 1];
                    o[2 * i] = (cur * 3 + last + 8) >> 4;
                    o[2 * i + 1] = (cur * 3 + nxt + 7) >> 4;
                    last = cur;
                    cur = nxt;
                }
                o[2 * n - 2] = (cur * 3 + last + 8) >> 4;
                o[2 * n - 1] = (cur * 4 + 7) >> 4;
            }
        }
        const uint8_t* yrow = plane[0] + (size_t)Y * pw[0];
        uint8_t* orow = out + (size_t)y * dw * 3;
        for (int x = 0; x < dw; x++) {
            int X = x * s;
            int yy = yrow[X], cb = up[0][X] - 128, cr = up[1][X] - 128;
            int rr, gg, bb;
            if (J.rgb) { /* jdcolor.c null_convert: the components are R, G, B */
                rr = yy;
                gg = cb + 128;
                bb = cr + 128;
            } else { /* ycc_rgb_convert: FIX(x) = (int)(x * 65536 + 0.5), ONE_HALF = 1 << 15 */
                rr = yy + ((91881 * cr + 32768) >> 16);
                gg = yy + ((-22554 * cb + 32768 - 46802 * cr) >> 16);
                bb = yy + ((116130 * cb + 32768) >> 16);
            }
            orow[3 * x + 0] = clamp255(bb);
            orow[3 * x + 1] = clamp255(gg);
            orow[3 * x + 2] = clamp255(rr);
        }
    }
    free(up[0]);
    for (int c = 0; c < 3; c++) free(plane[c]);
    return 0;
}

int oracle_jpeg_decode(const uint8_t* jpg, size_t len, int s, uint8_t* out, size_t cap, int* ow, int* oh,
                       int* ofmt)
{
    return decode_impl(jpg, len, s, out, cap, ow, oh, ofmt, 0);
}

int oracle_jpeg_decode_luma(const uint8_t* jpg, size_t len, uint8_t* out, size_t cap, int* ow, int* oh)
{
    int fmt;
    return decode_impl(jpg, len, 1, out, cap, ow, oh, &fmt, 1);
}
