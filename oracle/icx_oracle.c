/*
 * icx_oracle.c — scalar CPU restatement of the reference's JPEG target-size
 * path.  TEST INFRASTRUCTURE ONLY (see icx_oracle.h): the checker for the HIP
 * path and the timed CPU baseline ("kind": "port").  Never linked into
 * libicx.so.
 *
 * The JPEG arithmetic lives in a third-party dependency that is absent from
 * /root/reference: OpenJDK 21 java.desktop (com.sun.imageio.plugins.jpeg +
 * bundled IJG libjpeg 6b, "libjavajpeg"), reached from
 * ImageCompressionJpg.java:136-147.  This file restates the published IJG 6b
 * algorithm (jccolor.c, jcprepct.c, jcsample.c, jcdctmgr.c, jfdctint.c,
 * jccoefct.c, jchuff.c, jcmarker.c) and the JDK's quality handling, written
 * fresh from those algorithms' specifications.  Every function cites the
 * reference call site it serves.
 */
#include "icx_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* constants (ITU-T T.81 Annex K; JPEGQTable.K1Luminance/K2Chrominance) */
/* ------------------------------------------------------------------ */
static const int K1[64] = {
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const int K2[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
/* zig-zag index -> natural index */
static const int ZZ[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
/* Huffman specs: counts for code lengths 1..16, then symbols */
static const uint8_t DC_L_BITS[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t DC_C_BITS[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t DC_VALS[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t AC_L_BITS[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t AC_L_VALS[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};
static const uint8_t AC_C_BITS[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t AC_C_VALS[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};

/* ------------------------------------------------------------------ */
/* A6: quality -> tables.  Float32 throughout, as Java evaluates it.     */
/* ------------------------------------------------------------------ */
static float linear_quality(float q) /* JPEG.convertToLinearQuality */
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

static void scale_table(const int* base, float lin, uint16_t* out)
{ /* JPEGQTable.getScaledInstance(lin, forceBaseline=true) */
    for (int i = 0; i < 64; i++) {
        volatile float p = (float)base[i] * lin; /* volatile: no FMA contraction */
        volatile float s = p + 0.5f;
        int sv = (int)s;
        if (sv < 1) sv = 1;
        if (sv > 255) sv = 255;
        out[i] = (uint16_t)sv;
    }
}

void oracle_qtables(float q, uint16_t lum[64], uint16_t chrom[64])
{ /* reached from ImageCompressionJpg.java:140-143 (MODE_EXPLICIT, setCompressionQuality) */
    float lin = linear_quality(q);
    scale_table(K1, lin, lum);
    scale_table(K2, lin, chrom);
}

/* ------------------------------------------------------------------ */
/* geometry                                                            */
/* ------------------------------------------------------------------ */
typedef struct {
    int w, h, ncomp;
    int mcux, mcuy;         /* MCUs across / down */
    int ywb, yhb;           /* Y width/height in blocks (ceil(W/8), ceil(H/8)) */
    int cw, ch;             /* chroma plane size (downsampled, MCU-padded) */
    long nblocks;
} geom_t;

static void geom(int w, int h, int fmt, geom_t* g)
{
    g->w = w;
    g->h = h;
    g->ncomp = (fmt == OR_GRAY8) ? 1 : 3;
    g->ywb = (w + 7) / 8;
    g->yhb = (h + 7) / 8;
    if (g->ncomp == 1) {
        g->mcux = g->ywb;
        g->mcuy = g->yhb;
        g->nblocks = (long)g->mcux * g->mcuy;
        g->cw = g->ch = 0;
    } else {
        g->mcux = (w + 15) / 16;
        g->mcuy = (h + 15) / 16;
        g->nblocks = (long)g->mcux * g->mcuy * 6;
        g->cw = g->mcux * 8;
        g->ch = g->mcuy * 8;
    }
}

long oracle_num_blocks(int w, int h, int fmt)
{
    geom_t g;
    if (w <= 0 || h <= 0) return 0;
    geom(w, h, fmt, &g);
    return g.nblocks;
}

/* ------------------------------------------------------------------ */
/* A7: rgb_ycc_convert (jccolor.c), 16-bit fixed point with tables      */
/* ------------------------------------------------------------------ */
#define SCALEBITS 16
#define ONE_HALF ((int32_t)1 << (SCALEBITS - 1))
#define CBCR_OFFSET ((int32_t)128 << SCALEBITS)
#define FIXC(x) ((int32_t)((x) * (1L << SCALEBITS) + 0.5))

static int32_t tab_r_y[256], tab_g_y[256], tab_b_y[256], tab_r_cb[256], tab_g_cb[256],
    tab_b_cb[256], tab_g_cr[256], tab_b_cr[256];
static pthread_once_t tab_once = PTHREAD_ONCE_INIT;
static void init_tabs(void)
{
    for (int i = 0; i < 256; i++) {
        tab_r_y[i] = FIXC(0.29900) * i;
        tab_g_y[i] = FIXC(0.58700) * i;
        tab_b_y[i] = FIXC(0.11400) * i + ONE_HALF;
        tab_r_cb[i] = (-FIXC(0.16874)) * i;
        tab_g_cb[i] = (-FIXC(0.33126)) * i;
        tab_b_cb[i] = FIXC(0.50000) * i + CBCR_OFFSET + ONE_HALF - 1; /* also R->Cr */
        tab_g_cr[i] = (-FIXC(0.41869)) * i;
        tab_b_cr[i] = (-FIXC(0.08131)) * i;
    }
}

static void pixel_rgb(const uint8_t* p, int fmt, int* r, int* g, int* b)
{
    if (fmt == OR_BGR24) {
        *b = p[0]; *g = p[1]; *r = p[2];
    } else {
        *r = p[0]; *g = p[1]; *b = p[2];
    }
}

/* Colour planes + libjpeg edge expansion (jcprepct.c expand_bottom_edge,
 * jcsample.c expand_right_edge) + h2v2_downsample.  Y is returned padded to
 * ywb*8 x yhb*8... (actually mcu-padded), chroma already downsampled. */
typedef struct {
    uint8_t* Y;   /* stride yw, rows yh (MCU padded) */
    uint8_t* Cb;  /* stride cw, rows ch */
    uint8_t* Cr;
    int yw, yh;
} planes_t;

static int make_planes(const uint8_t* px, int stride, int fmt, const geom_t* g, planes_t* P)
{
    pthread_once(&tab_once, init_tabs);
    const int W = g->w, H = g->h;
    int yw = (g->ncomp == 1) ? g->mcux * 8 : g->mcux * 16;
    int yh = (g->ncomp == 1) ? g->mcuy * 8 : g->mcuy * 16;
    P->yw = yw;
    P->yh = yh;
    P->Y = (uint8_t*)malloc((size_t)yw * yh);
    P->Cb = P->Cr = NULL;
    if (!P->Y) return -1;
    if (g->ncomp == 1) {
        for (int y = 0; y < yh; y++) {
            const uint8_t* row = px + (size_t)(y < H ? y : H - 1) * stride;
            for (int x = 0; x < yw; x++) P->Y[(size_t)y * yw + x] = row[x < W ? x : W - 1];
        }
        return 0;
    }
    /* full-resolution YCbCr for the real rows, width expanded to yw */
    int rows = H + (H & 1); /* row group of 2 padded (expand_bottom_edge on color_buf) */
    uint8_t* fy = (uint8_t*)malloc((size_t)yw * rows);
    uint8_t* fcb = (uint8_t*)malloc((size_t)yw * rows);
    uint8_t* fcr = (uint8_t*)malloc((size_t)yw * rows);
    P->Cb = (uint8_t*)malloc((size_t)g->cw * g->ch);
    P->Cr = (uint8_t*)malloc((size_t)g->cw * g->ch);
    if (!fy || !fcb || !fcr || !P->Cb || !P->Cr) {
        free(fy); free(fcb); free(fcr);
        return -1;
    }
    for (int y = 0; y < rows; y++) {
        const uint8_t* row = px + (size_t)(y < H ? y : H - 1) * stride;
        for (int x = 0; x < yw; x++) {
            int sx = x < W ? x : W - 1;
            int r, gg, b;
            pixel_rgb(row + 3 * sx, fmt, &r, &gg, &b);
            size_t o = (size_t)y * yw + x;
            fy[o] = (uint8_t)((tab_r_y[r] + tab_g_y[gg] + tab_b_y[b]) >> SCALEBITS);
            fcb[o] = (uint8_t)((tab_r_cb[r] + tab_g_cb[gg] + tab_b_cb[b]) >> SCALEBITS);
            fcr[o] = (uint8_t)((tab_b_cb[r] + tab_g_cr[gg] + tab_b_cr[b]) >> SCALEBITS);
        }
    }
    /* Y: rows beyond the image replicate the last Y row */
    for (int y = 0; y < yh; y++) {
        int sy = y < rows ? y : rows - 1;
        memcpy(P->Y + (size_t)y * yw, fy + (size_t)sy * yw, (size_t)yw);
    }
    /* chroma: h2v2_downsample over row pairs, then the last downsampled row is
     * replicated to the iMCU height (expand_bottom_edge on the output buffer) */
    int crows = rows / 2;
    for (int r = 0; r < g->ch; r++) {
        int sr = r < crows ? r : crows - 1;
        const uint8_t *b0 = fcb + (size_t)(2 * sr) * yw, *b1 = b0 + yw;
        const uint8_t *c0 = fcr + (size_t)(2 * sr) * yw, *c1 = c0 + yw;
        for (int c = 0; c < g->cw; c++) {
            int bias = (c & 1) ? 2 : 1;
            P->Cb[(size_t)r * g->cw + c] =
                (uint8_t)((b0[2 * c] + b0[2 * c + 1] + b1[2 * c] + b1[2 * c + 1] + bias) >> 2);
            P->Cr[(size_t)r * g->cw + c] =
                (uint8_t)((c0[2 * c] + c0[2 * c + 1] + c1[2 * c] + c1[2 * c + 1] + bias) >> 2);
        }
    }
    free(fy); free(fcb); free(fcr);
    return 0;
}

static void free_planes(planes_t* P)
{
    free(P->Y); free(P->Cb); free(P->Cr);
}

/* ------------------------------------------------------------------ */
/* A9: jpeg_fdct_islow (jfdctint.c, IJG 6b), data in natural order      */
/* ------------------------------------------------------------------ */
#define CONST_BITS 13
#define PASS1_BITS 2
#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

static void fdct_islow(int32_t* d)
{
    int32_t t0, t1, t2, t3, t4, t5, t6, t7, t10, t11, t12, t13, z1, z2, z3, z4, z5;
    for (int r = 0; r < 8; r++) {
        int32_t* p = d + 8 * r;
        t0 = p[0] + p[7]; t7 = p[0] - p[7];
        t1 = p[1] + p[6]; t6 = p[1] - p[6];
        t2 = p[2] + p[5]; t5 = p[2] - p[5];
        t3 = p[3] + p[4]; t4 = p[3] - p[4];
        t10 = t0 + t3; t13 = t0 - t3; t11 = t1 + t2; t12 = t1 - t2;
        p[0] = (t10 + t11) << PASS1_BITS;
        p[4] = (t10 - t11) << PASS1_BITS;
        z1 = (t12 + t13) * FIX_0_541196100;
        p[2] = DESCALE(z1 + t13 * FIX_0_765366865, CONST_BITS - PASS1_BITS);
        p[6] = DESCALE(z1 - t12 * FIX_1_847759065, CONST_BITS - PASS1_BITS);
        z1 = t4 + t7; z2 = t5 + t6; z3 = t4 + t6; z4 = t5 + t7;
        z5 = (z3 + z4) * FIX_1_175875602;
        t4 *= FIX_0_298631336; t5 *= FIX_2_053119869;
        t6 *= FIX_3_072711026; t7 *= FIX_1_501321110;
        z1 *= -FIX_0_899976223; z2 *= -FIX_2_562915447;
        z3 *= -FIX_1_961570560; z4 *= -FIX_0_390180644;
        z3 += z5; z4 += z5;
        p[7] = DESCALE(t4 + z1 + z3, CONST_BITS - PASS1_BITS);
        p[5] = DESCALE(t5 + z2 + z4, CONST_BITS - PASS1_BITS);
        p[3] = DESCALE(t6 + z2 + z3, CONST_BITS - PASS1_BITS);
        p[1] = DESCALE(t7 + z1 + z4, CONST_BITS - PASS1_BITS);
    }
    for (int c = 0; c < 8; c++) {
        int32_t* p = d + c;
        t0 = p[0] + p[56]; t7 = p[0] - p[56];
        t1 = p[8] + p[48]; t6 = p[8] - p[48];
        t2 = p[16] + p[40]; t5 = p[16] - p[40];
        t3 = p[24] + p[32]; t4 = p[24] - p[32];
        t10 = t0 + t3; t13 = t0 - t3; t11 = t1 + t2; t12 = t1 - t2;
        p[0] = DESCALE(t10 + t11, PASS1_BITS);
        p[32] = DESCALE(t10 - t11, PASS1_BITS);
        z1 = (t12 + t13) * FIX_0_541196100;
        p[16] = DESCALE(z1 + t13 * FIX_0_765366865, CONST_BITS + PASS1_BITS);
        p[48] = DESCALE(z1 - t12 * FIX_1_847759065, CONST_BITS + PASS1_BITS);
        z1 = t4 + t7; z2 = t5 + t6; z3 = t4 + t6; z4 = t5 + t7;
        z5 = (z3 + z4) * FIX_1_175875602;
        t4 *= FIX_0_298631336; t5 *= FIX_2_053119869;
        t6 *= FIX_3_072711026; t7 *= FIX_1_501321110;
        z1 *= -FIX_0_899976223; z2 *= -FIX_2_562915447;
        z3 *= -FIX_1_961570560; z4 *= -FIX_0_390180644;
        z3 += z5; z4 += z5;
        p[56] = DESCALE(t4 + z1 + z3, CONST_BITS + PASS1_BITS);
        p[40] = DESCALE(t5 + z2 + z4, CONST_BITS + PASS1_BITS);
        p[24] = DESCALE(t6 + z2 + z3, CONST_BITS + PASS1_BITS);
        p[8] = DESCALE(t7 + z1 + z4, CONST_BITS + PASS1_BITS);
    }
}

/* forward_DCT (jcdctmgr.c): level shift, DCT, store zig-zag raw output */
static void block_fdct(const uint8_t* plane, int pstride, int x0, int y0, int16_t* out_zz)
{
    int32_t d[64];
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) d[8 * r + c] = (int32_t)plane[(size_t)(y0 + r) * pstride + x0 + c] - 128;
    fdct_islow(d);
    for (int k = 0; k < 64; k++) out_zz[k] = (int16_t)d[ZZ[k]];
}

static void dummy_block(int16_t* out_zz, int16_t dc)
{
    memset(out_zz, 0, 64 * sizeof(int16_t));
    out_zz[0] = dc;
}

/* jccoefct.c compress_data: MCU order, dummy blocks at the right/bottom edge
 * of the Y component get AC=0 and the DC of MCU_buffer[blkn-1] (right) or of
 * the last block of the previous row of the MCU (bottom). */
static void planes_to_coefs(const planes_t* P, const geom_t* g, int16_t* coefs)
{
    long b = 0;
    if (g->ncomp == 1) {
        for (int my = 0; my < g->mcuy; my++)
            for (int mx = 0; mx < g->mcux; mx++) block_fdct(P->Y, P->yw, mx * 8, my * 8, coefs + 64 * (b++));
        return;
    }
    for (int my = 0; my < g->mcuy; my++) {
        for (int mx = 0; mx < g->mcux; mx++) {
            int16_t* mcu = coefs + 64 * b;
            for (int yi = 0; yi < 2; yi++) {
                int brow = 2 * my + yi;
                int16_t* rowblk = mcu + 64 * (2 * yi);
                if (brow < g->yhb) {
                    for (int xi = 0; xi < 2; xi++) {
                        int bcol = 2 * mx + xi;
                        if (bcol < g->ywb)
                            block_fdct(P->Y, P->yw, bcol * 8, brow * 8, rowblk + 64 * xi);
                        else
                            dummy_block(rowblk + 64 * xi, rowblk[64 * (xi - 1)]);
                    }
                } else {
                    int16_t dc = rowblk[-64]; /* MCU_buffer[blkn-1] */
                    dummy_block(rowblk, dc);
                    dummy_block(rowblk + 64, dc);
                }
            }
            block_fdct(P->Cb, g->cw, mx * 8, my * 8, mcu + 64 * 4);
            block_fdct(P->Cr, g->cw, mx * 8, my * 8, mcu + 64 * 5);
            b += 6;
        }
    }
}

long oracle_fdct(const uint8_t* px, int w, int h, int stride, int fmt, int16_t* coefs)
{
    geom_t g;
    planes_t P;
    if (w <= 0 || h <= 0 || !px || !coefs) return -1;
    geom(w, h, fmt, &g);
    if (make_planes(px, stride, fmt, &g, &P)) return -1;
    planes_to_coefs(&P, &g, coefs);
    free_planes(&P);
    return g.nblocks;
}

/* ------------------------------------------------------------------ */
/* A9 quantiser + A10 Huffman / markers                                */
/* ------------------------------------------------------------------ */
typedef struct {
    uint16_t code[256];
    uint8_t size[256];
} huff_t;

static void make_huff(const uint8_t* bits, const uint8_t* vals, huff_t* t)
{ /* jchuff.c jpeg_make_c_derived_tbl */
    memset(t, 0, sizeof(*t));
    unsigned code = 0;
    int k = 0;
    for (int l = 1; l <= 16; l++) {
        for (int i = 0; i < bits[l - 1]; i++, k++) {
            t->code[vals[k]] = (uint16_t)code;
            t->size[vals[k]] = (uint8_t)l;
            code++;
        }
        code <<= 1;
    }
}

static huff_t H_DC_L, H_DC_C, H_AC_L, H_AC_C;
static pthread_once_t huff_once = PTHREAD_ONCE_INIT;
static void init_huff(void)
{
    make_huff(DC_L_BITS, DC_VALS, &H_DC_L);
    make_huff(DC_C_BITS, DC_VALS, &H_DC_C);
    make_huff(AC_L_BITS, AC_L_VALS, &H_AC_L);
    make_huff(AC_C_BITS, AC_C_VALS, &H_AC_C);
}

typedef struct {
    uint8_t* out;
    size_t cap, pos;
    uint64_t acc;
    int nbits;
} bw_t;

static inline void put_byte(bw_t* w, uint8_t v)
{
    if (w->pos < w->cap) w->out[w->pos] = v;
    w->pos++;
}

static inline void emit_bits(bw_t* w, uint32_t code, int size)
{ /* jchuff.c emit_bits: MSB first, 0xFF stuffed with 0x00 */
    w->acc = (w->acc << size) | (code & ((1u << size) - 1));
    w->nbits += size;
    while (w->nbits >= 8) {
        uint8_t c = (uint8_t)(w->acc >> (w->nbits - 8));
        put_byte(w, c);
        if (c == 0xFF) put_byte(w, 0);
        w->nbits -= 8;
    }
}

static void flush_bits(bw_t* w)
{ /* jchuff.c flush_bits: fill the last byte with 1-bits */
    emit_bits(w, 0x7F, 7);
    w->acc = 0;
    w->nbits = 0;
}

static inline int quantize(int c, int qv8)
{ /* jcdctmgr.c forward_DCT, divisor = quantval<<3, round half away from 0 */
    if (c < 0) {
        c = -c + (qv8 >> 1);
        c = c >= qv8 ? c / qv8 : 0;
        return -c;
    }
    c += qv8 >> 1;
    return c >= qv8 ? c / qv8 : 0;
}

static void encode_block(bw_t* w, const int16_t* zz, const int* div_zz, int* last_dc,
                         const huff_t* dct, const huff_t* act)
{ /* jchuff.c encode_one_block */
    int q[64];
    for (int k = 0; k < 64; k++) q[k] = quantize(zz[k], div_zz[k]);
    int t = q[0] - *last_dc, t2 = t;
    *last_dc = q[0];
    if (t < 0) { t = -t; t2--; }
    int nbits = 0;
    while (t) { nbits++; t >>= 1; }
    emit_bits(w, dct->code[nbits], dct->size[nbits]);
    if (nbits) emit_bits(w, (uint32_t)t2, nbits);
    int r = 0;
    for (int k = 1; k < 64; k++) {
        if ((t = q[k]) == 0) {
            r++;
            continue;
        }
        while (r > 15) {
            emit_bits(w, act->code[0xF0], act->size[0xF0]);
            r -= 16;
        }
        t2 = t;
        if (t < 0) { t = -t; t2--; }
        nbits = 1;
        while ((t >>= 1)) nbits++;
        int s = (r << 4) + nbits;
        emit_bits(w, act->code[s], act->size[s]);
        emit_bits(w, (uint32_t)t2, nbits);
        r = 0;
    }
    if (r > 0) emit_bits(w, act->code[0], act->size[0]);
}

static void put16(bw_t* w, int v)
{
    put_byte(w, (uint8_t)(v >> 8));
    put_byte(w, (uint8_t)v);
}

static void emit_dqt_table(bw_t* w, int index, const uint16_t* tbl)
{
    put_byte(w, (uint8_t)index);
    for (int k = 0; k < 64; k++) put_byte(w, (uint8_t)tbl[ZZ[k]]);
}

static void emit_dht_table(bw_t* w, int index, const uint8_t* bits, const uint8_t* vals)
{
    int n = 0;
    for (int i = 0; i < 16; i++) n += bits[i];
    put_byte(w, (uint8_t)index);
    for (int i = 0; i < 16; i++) put_byte(w, bits[i]);
    for (int i = 0; i < n; i++) put_byte(w, vals[i]);
}

static int dht_len(const uint8_t* bits)
{
    int n = 0;
    for (int i = 0; i < 16; i++) n += bits[i];
    return 17 + n;
}

/* Marker layout of the tables (SURVEY.md §7 hard part 2): 0 = one DQT and
 * one DHT segment per table, as libjpeg 6b's jcmarker.c writes them when the
 * JDK hands it the tables (623 B colour / 328 B grey header); 1 = every
 * quantisation table in one DQT segment and every Huffman table in one DHT
 * segment, the grouping of a JDK DQT/DHT metadata marker segment holding
 * several tables (607 B / 324 B).  Same entropy-coded data either way.
 * Process-wide; set before encoding (test infrastructure). */
static int g_table_layout = 0;

void oracle_set_table_layout(int grouped) { g_table_layout = grouped ? 1 : 0; }

/* Marker layout: SOI; APP0 JFIF written by the JDK's Java metadata writer
 * (JFIFMarkerSegment: version 1.02, aspect-ratio units, density 1x1); DQT,
 * SOF0, DHT, SOS written by libjpeg (jcmarker.c), tables per g_table_layout. */
static void write_header(bw_t* w, const geom_t* g, const uint16_t* lum, const uint16_t* chrom)
{
    static const uint8_t app0[18] = {0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00,
                                     0x01, 0x02, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    const int nt = g->ncomp == 3 ? 2 : 1; /* tables of each kind */
    put_byte(w, 0xFF); put_byte(w, 0xD8);
    for (int i = 0; i < 18; i++) put_byte(w, app0[i]);
    for (int t = 0; t < nt; t++) {
        if (t == 0 || !g_table_layout) {
            put_byte(w, 0xFF); put_byte(w, 0xDB);
            put16(w, 2 + (g_table_layout ? nt : 1) * 65);
        }
        emit_dqt_table(w, t, t ? chrom : lum);
    }
    put_byte(w, 0xFF); put_byte(w, 0xC0);
    put16(w, 8 + 3 * g->ncomp);
    put_byte(w, 8);
    put16(w, g->h);
    put16(w, g->w);
    put_byte(w, (uint8_t)g->ncomp);
    if (g->ncomp == 1) {
        put_byte(w, 1); put_byte(w, 0x11); put_byte(w, 0);
    } else {
        put_byte(w, 1); put_byte(w, 0x22); put_byte(w, 0);
        put_byte(w, 2); put_byte(w, 0x11); put_byte(w, 1);
        put_byte(w, 3); put_byte(w, 0x11); put_byte(w, 1);
    }
    const uint8_t* bits[4] = {DC_L_BITS, AC_L_BITS, DC_C_BITS, AC_C_BITS};
    const uint8_t* vals[4] = {DC_VALS, AC_L_VALS, DC_VALS, AC_C_VALS};
    const int idx[4] = {0x00, 0x10, 0x01, 0x11};
    int total = 0;
    for (int t = 0; t < 2 * nt; t++) total += dht_len(bits[t]);
    for (int t = 0; t < 2 * nt; t++) {
        if (t == 0 || !g_table_layout) {
            put_byte(w, 0xFF); put_byte(w, 0xC4);
            put16(w, 2 + (g_table_layout ? total : dht_len(bits[t])));
        }
        emit_dht_table(w, idx[t], bits[t], vals[t]);
    }
    put_byte(w, 0xFF); put_byte(w, 0xDA);
    put16(w, 6 + 2 * g->ncomp);
    put_byte(w, (uint8_t)g->ncomp);
    if (g->ncomp == 1) {
        put_byte(w, 1); put_byte(w, 0x00);
    } else {
        put_byte(w, 1); put_byte(w, 0x00);
        put_byte(w, 2); put_byte(w, 0x11);
        put_byte(w, 3); put_byte(w, 0x11);
    }
    put_byte(w, 0); put_byte(w, 63); put_byte(w, 0);
}

static int encode_coefs(const int16_t* coefs, const geom_t* g, float q, uint8_t* out, size_t cap,
                        size_t* len)
{
    pthread_once(&huff_once, init_huff);
    uint16_t lum[64], chrom[64];
    int dl[64], dc[64];
    oracle_qtables(q, lum, chrom);
    for (int k = 0; k < 64; k++) {
        dl[k] = lum[ZZ[k]] << 3;
        dc[k] = chrom[ZZ[k]] << 3;
    }
    bw_t w = {out, cap, 0, 0, 0};
    write_header(&w, g, lum, chrom);
    int last[3] = {0, 0, 0};
    long b = 0;
    if (g->ncomp == 1) {
        for (; b < g->nblocks; b++) encode_block(&w, coefs + 64 * b, dl, &last[0], &H_DC_L, &H_AC_L);
    } else {
        for (long m = 0; m < g->nblocks / 6; m++) {
            for (int i = 0; i < 4; i++, b++) encode_block(&w, coefs + 64 * b, dl, &last[0], &H_DC_L, &H_AC_L);
            encode_block(&w, coefs + 64 * b, dc, &last[1], &H_DC_C, &H_AC_C); b++;
            encode_block(&w, coefs + 64 * b, dc, &last[2], &H_DC_C, &H_AC_C); b++;
        }
    }
    flush_bits(&w);
    put_byte(&w, 0xFF);
    put_byte(&w, 0xD9);
    *len = w.pos;
    return w.pos > cap ? 4 : 0;
}

int oracle_encode(const uint8_t* px, int w, int h, int stride, int fmt, float q, uint8_t* out,
                  size_t cap, size_t* len)
{ /* ImageCompressionJpg.compressJpgToStream :136-147 -> JDK JPEGImageWriter.write */
    geom_t g;
    planes_t P;
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535 || !px || !len) return 1;
    if (fmt != OR_BGR24 && fmt != OR_RGB24 && fmt != OR_GRAY8) return 1;
    geom(w, h, fmt, &g);
    int16_t* coefs = (int16_t*)malloc((size_t)g.nblocks * 64 * sizeof(int16_t));
    if (!coefs) return 2;
    if (make_planes(px, stride, fmt, &g, &P)) {
        free(coefs);
        return 2;
    }
    planes_to_coefs(&P, &g, coefs);
    free_planes(&P);
    int rc = encode_coefs(coefs, &g, q, out, cap, len);
    free(coefs);
    return rc;
}

static int64_t encoded_size(const uint8_t* px, int w, int h, int stride, int fmt, float q)
{
    size_t len = 0;
    int rc = oracle_encode(px, w, h, stride, fmt, q, NULL, 0, &len);
    return (rc == 0 || rc == 4) ? (int64_t)len : -1;
}

/* ------------------------------------------------------------------ */
/* A3: findBestQualityByBinarySearch (ImageCompressionJpg.java:158-200) */
/* ------------------------------------------------------------------ */
float oracle_find_best_quality(const uint8_t* px, int w, int h, int stride, int fmt, int64_t target,
                               float q0, float* trial_q, int64_t* trial_size, int* ntrials)
{
    volatile float lo = 0.0f, hi = q0, best = -1.0f;
    int n = 0;
    for (int i = 0; i < 8; i++) {
        volatile float sum = lo + hi;
        volatile float mid = sum / 2.0f;
        if (mid < 0.01f) break;
        int64_t size = encoded_size(px, w, h, stride, fmt, mid);
        if (trial_q) trial_q[n] = mid;
        if (trial_size) trial_size[n] = size;
        n++;
        if (size >= 0 && size <= target) {
            best = mid;
            lo = mid;
        } else {
            hi = mid;
        }
        volatile float diff = hi - lo;
        if (diff < 0.01f) break;
    }
    if (ntrials) *ntrials = n;
    return best;
}

/* ------------------------------------------------------------------ */
/* A12: ImageTools.resizeImage -> Graphics2D.drawImage, BILINEAR.        */
/* Java2D: DrawImage.renderImageXform -> TransformHelper (native):      */
/* inverse scale in 32.32 fixed point, sample at centre-0.5, edge clamp,*/
/* 8-bit fraction weights (BilinearInterp), round at bit 16.            */
/* ------------------------------------------------------------------ */
void oracle_scaled_dims(int w, int h, double scale, int* dw, int* dh)
{ /* ImageTools.java:8-9 */
    int nw = (int)(w * scale), nh = (int)(h * scale);
    *dw = nw < 1 ? 1 : nw;
    *dh = nh < 1 ? 1 : nh;
}

static inline int64_t dbl_to_long(double d) { return (int64_t)(d * 4294967296.0); }

/* Java2D AlphaMath.c initAlphaTables: mul8table[a][c] ~ a*c/255 and
 * div8table[a][c] ~ c*255/a (c < a; 255 from c = a on), both in 8.24 fixed
 * point with the tables' own rounding.  Row/column 0 of mul8table is 0. */
static inline int mul8(int a, int c)
{
    const uint32_t inc = (uint32_t)a * 0x010101u;
    return (int)((c * inc + (1u << 23)) >> 24) & 0xff;
}

static inline int div8(int a, int c)
{
    if (c >= a) return 255;
    const uint32_t inc = ((0xffu << 24) + (uint32_t)a / 2) / (uint32_t)a;
    return (int)(((1u << 23) + (uint32_t)c * inc) >> 24);
}

/* Four-byte pixels (ImageTools.java:12-15 keeps the type; TYPE_CUSTOM with
 * alpha becomes TYPE_INT_ARGB): TransformHelper fetches the four neighbours
 * as IntArgbPre (colours premultiplied by mul8table, an opaque type's alpha
 * 0xff), interpolates all four channels as above, and the SrcOver mask blit
 * onto the new all-zero image stores alpha 0 as untouched zero pixels,
 * alpha 0xff as is, and otherwise un-premultiplies with div8table.  An
 * XRGB (TYPE_INT_RGB) destination stores 0 in its unused byte. */
static int resize4(const uint8_t* src, int sw, int sh, int sstride, int fmt, uint8_t* dst, int dw, int dh,
                   int dstride)
{
    const int ab = fmt == OR_ABGR32 ? 0 : 3;  /* alpha byte */
    const int opaque = fmt == OR_XRGB32;
    double ix = 1.0 / ((double)dw / sw), iy = 1.0 / ((double)dh / sh);
    int64_t dxl = dbl_to_long(ix), dyl = dbl_to_long(iy);
    int64_t x0l = dbl_to_long(0.5 * ix), y0l = dbl_to_long(0.5 * iy);
    const int64_t half = (int64_t)1 << 31;
    for (int dy = 0; dy < dh; dy++) {
        int64_t yl = y0l + (int64_t)dy * dyl - half;
        int yw = (int)(yl >> 32), yf = (int)((uint32_t)yl >> 24), ya, yb;
        if (yw < 0) ya = yb = 0;
        else if (yw + 1 >= sh) ya = yb = yw;
        else { ya = yw; yb = yw + 1; }
        for (int dx = 0; dx < dw; dx++) {
            int64_t xl = x0l + (int64_t)dx * dxl - half;
            int xw = (int)(xl >> 32), xf = (int)((uint32_t)xl >> 24), xa, xb;
            if (xw < 0) xa = xb = 0;
            else if (xw + 1 >= sw) xa = xb = xw;
            else { xa = xw; xb = xw + 1; }
            const uint8_t* q[4] = {src + (size_t)ya * sstride + 4 * xa, src + (size_t)ya * sstride + 4 * xb,
                                   src + (size_t)yb * sstride + 4 * xa, src + (size_t)yb * sstride + 4 * xb};
            int pre[4][4];
            for (int s = 0; s < 4; s++) {
                const int a = opaque ? 255 : q[s][ab];
                for (int b = 0; b < 4; b++) pre[s][b] = b == ab ? a : mul8(a, q[s][b]);
            }
            int v[4];
            for (int b = 0; b < 4; b++) {
                int top = (pre[0][b] << 8) + (pre[1][b] - pre[0][b]) * xf;
                int bot = (pre[2][b] << 8) + (pre[3][b] - pre[2][b]) * xf;
                v[b] = (((top << 8) + (bot - top) * yf) + (1 << 15)) >> 16;
            }
            uint8_t* o = dst + (size_t)dy * dstride + 4 * dx;
            const int a = v[ab];
            for (int b = 0; b < 4; b++) {
                if (opaque) o[b] = b == ab ? 0 : (uint8_t)v[b];
                else if (a == 0) o[b] = 0;
                else if (b == ab || a == 255) o[b] = (uint8_t)v[b];
                else o[b] = (uint8_t)div8(a, v[b]);
            }
        }
    }
    return 0;
}

/* TYPE_USHORT_GRAY (a 16-bit grey PNG as the JDK reads it; ImageTools keeps
 * the type).  Java2D's UshortGray loops (UshortGray.h) carry it through the
 * 8-bit IntArgbPre the bilinear TransformHelper works in: the fetch keeps
 * gray >> 8, the four taps are interpolated as for 8-bit grey, and the
 * store composes a 16-bit grey from r = g = b = v as (19672 r + 38621 g +
 * 7500 b) >> 8 = 257 v.  Restated from the published OpenJDK source, no JDK
 * here to pin it (parity unpinned, like the rest of A12). */
static int resize16(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh, int dstride)
{
    uint8_t* hi = (uint8_t*)malloc((size_t)sw * sh);
    uint8_t* lo = (uint8_t*)malloc((size_t)dw * dh);
    if (!hi || !lo) { free(hi); free(lo); return 1; }
    for (int y = 0; y < sh; y++) {
        const uint16_t* r = (const uint16_t*)(src + (size_t)y * sstride);
        for (int x = 0; x < sw; x++) hi[(size_t)y * sw + x] = (uint8_t)(r[x] >> 8);
    }
    oracle_resize(hi, sw, sh, sw, OR_GRAY8, lo, dw, dh, dw);
    for (int y = 0; y < dh; y++) {
        uint16_t* o = (uint16_t*)(dst + (size_t)y * dstride);
        for (int x = 0; x < dw; x++) o[x] = (uint16_t)(lo[(size_t)y * dw + x] * 257);
    }
    free(hi);
    free(lo);
    return 0;
}

int oracle_resize(const uint8_t* src, int sw, int sh, int sstride, int fmt, uint8_t* dst, int dw,
                  int dh, int dstride)
{
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || !src || !dst) return 1;
    if (fmt == OR_GRAY16) return resize16(src, sw, sh, sstride, dst, dw, dh, dstride);
    if (fmt >= OR_XRGB32) return resize4(src, sw, sh, sstride, fmt, dst, dw, dh, dstride);
    int nch = (fmt == OR_GRAY8) ? 1 : 3;
    double ix = 1.0 / ((double)dw / sw), iy = 1.0 / ((double)dh / sh);
    int64_t dxl = dbl_to_long(ix), dyl = dbl_to_long(iy);
    int64_t x0l = dbl_to_long(0.5 * ix), y0l = dbl_to_long(0.5 * iy);
    const int64_t half = (int64_t)1 << 31;
    for (int dy = 0; dy < dh; dy++) {
        int64_t yl = y0l + (int64_t)dy * dyl - half;
        int yw = (int)(yl >> 32);
        int yf = (int)((uint32_t)yl >> 24);
        int ya, yb;
        if (yw < 0) ya = yb = 0;
        else if (yw + 1 >= sh) ya = yb = yw;
        else { ya = yw; yb = yw + 1; }
        const uint8_t* ra = src + (size_t)ya * sstride;
        const uint8_t* rb = src + (size_t)yb * sstride;
        uint8_t* out = dst + (size_t)dy * dstride;
        for (int dx = 0; dx < dw; dx++) {
            int64_t xl = x0l + (int64_t)dx * dxl - half;
            int xw = (int)(xl >> 32);
            int xf = (int)((uint32_t)xl >> 24);
            int xa, xb;
            if (xw < 0) xa = xb = 0;
            else if (xw + 1 >= sw) xa = xb = xw;
            else { xa = xw; xb = xw + 1; }
            for (int c = 0; c < nch; c++) {
                int p00 = ra[nch * xa + c], p01 = ra[nch * xb + c];
                int p10 = rb[nch * xa + c], p11 = rb[nch * xb + c];
                int top = (p00 << 8) + (p01 - p00) * xf;
                int bot = (p10 << 8) + (p11 - p10) * xf;
                int v = (top << 8) + (bot - top) * yf;
                out[nch * dx + c] = (uint8_t)((v + (1 << 15)) >> 16);
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* A12, palette rasters (ImageTools.java:12-17 keeps TYPE_BYTE_INDEXED / */
/* TYPE_BYTE_BINARY, so `new BufferedImage(nw, nh, type)` gets Java2D's   */
/* DEFAULT colour map, not the source's).  Restated from the published    */
/* OpenJDK java.desktop sources, no JDK here to pin them (parity unpinned):*/
/*  - BufferedImage(TYPE_BYTE_INDEXED): a 6x6x6 cube at 0, 51, ..., 255   */
/*    (r outer, b inner), then a grey ramp 18, 24, ..., 252 (256/40 = 6); */
/*    TYPE_BYTE_BINARY: {black, white}, 1 bit.                            */
/*  - the source is fetched as IntArgbPre through its own colour map      */
/*    (CopyByteIndexedToIntArgbPre: alpha 0 -> 0, else mul8 premultiply), */
/*    the taps interpolated as for the four-byte formats, and the alpha   */
/*    mask blit (SrcOver) composes onto the new image's pixel 0 = opaque  */
/*    black: the result is the premultiplied colour, alpha 255;           */
/*  - ByteIndexed store (StoreByteIndexedFrom3ByteRgb): unless r, g, b are */
/*    each 0 or 255 and the map "represents primaries", the 8x8 ordered   */
/*    dither errors (make_dither_arrays: make_sgn_ordered_dither_array    */
/*    over [-20, 20) for a 256-entry map, green mirrored horizontally,    */
/*    blue vertically) are added at (x & 7, y & 7), components clamped,   */
/*    then the inverse colour map of 32x32x32 cells (initCubemap: an L1   */
/*    flood fill from the map's entries, inserted 0, n-1, 1, n-2, ...,    */
/*    level by level, first claim wins) gives the index;                  */
/*  - ByteBinary1Bit store: the inverse map alone, no dither.             */
/* ------------------------------------------------------------------ */
void oracle_default_palette(int binary, uint32_t pal[256], int* n)
{
    if (binary) {
        pal[0] = 0xff000000u;
        pal[1] = 0xffffffffu;
        *n = 2;
        return;
    }
    int i = 0;
    for (int r = 0; r < 256; r += 51)
        for (int g = 0; g < 256; g += 51)
            for (int b = 0; b < 256; b += 51) pal[i++] = 0xff000000u | (uint32_t)(r << 16) | (uint32_t)(g << 8) | (uint32_t)b;
    const int incr = 256 / (256 - i);
    for (int gray = incr * 3; i < 256; i++, gray += incr)
        pal[i] = 0xff000000u | (uint32_t)(gray << 16) | (uint32_t)(gray << 8) | (uint32_t)gray;
    *n = 256;
}

static int cube_insert(uint8_t* used, uint8_t* lut, uint16_t* list, uint8_t* idx, int n, int rgb, int index)
{
    if (used[rgb]) return n;
    used[rgb] = 1;
    lut[rgb] = (uint8_t)index;
    list[n] = (uint16_t)rgb;
    idx[n] = (uint8_t)index;
    return n + 1;
}

void oracle_inverse_cube(const uint32_t* cmap, int n, uint8_t cube[32768])
{
    uint8_t* used = (uint8_t*)calloc(32768, 1);
    uint16_t* cur = (uint16_t*)malloc(32768 * 2 * sizeof(uint16_t));
    uint8_t* cidx = (uint8_t*)malloc(32768 * 2);
    uint16_t* nxt = cur + 32768;
    uint8_t* nidx = cidx + 32768;
    int nc = 0;
    const int mid = (n >> 1) + (n & 1);
    for (int i = 0; i < mid; i++) {
        const int k[2] = {i, n - i - 1};
        for (int e = 0; e < 2; e++) {
            const uint32_t px = cmap[k[e]];
            const int rgb = (int)(((px & 0x00f80000u) >> 9) | ((px & 0x0000f800u) >> 6) | ((px & 0xf8u) >> 3));
            nc = cube_insert(used, cube, cur, cidx, nc, rgb, k[e]);
        }
    }
    static const int mask[3] = {0x7c00, 0x03e0, 0x001f}, delta[3] = {0x0400, 0x0020, 0x0001};
    while (nc) {
        int nn = 0;
        for (int i = 0; i < nc; i++) {
            const int rgb = cur[i], index = cidx[i];
            for (int a = 0; a < 3; a++) {
                if ((rgb & mask[a]) + delta[a] <= mask[a]) nn = cube_insert(used, cube, nxt, nidx, nn, rgb + delta[a], index);
                if ((rgb & mask[a]) >= delta[a]) nn = cube_insert(used, cube, nxt, nidx, nn, rgb - delta[a], index);
            }
        }
        memcpy(cur, nxt, (size_t)nn * sizeof(uint16_t));
        memcpy(cidx, nidx, (size_t)nn);
        nc = nn;
    }
    free(used);
    free(cur);
    free(cidx);
}

/* the three 8x8 dither error tables, [(y & 7) * 8 + (x & 7)] */
void oracle_dither_tables(int cmapsize, int8_t red[64], int8_t green[64], int8_t blue[64])
{
    const int e = (int)(256 / pow(cmapsize, 1.0 / 3.0));
    const int lo = -e / 2, hi = e - e / 2;
    int oda[64];
    oda[0] = 0;
    for (int k = 1; k < 8; k *= 2)
        for (int i = 0; i < k; i++)
            for (int j = 0; j < k; j++) {
                oda[i * 8 + j] = oda[i * 8 + j] * 4;
                oda[(i + k) * 8 + (j + k)] = oda[i * 8 + j] + 1;
                oda[i * 8 + (j + k)] = oda[i * 8 + j] + 2;
                oda[(i + k) * 8 + j] = oda[i * 8 + j] + 3;
            }
    for (int i = 0; i < 64; i++) red[i] = green[i] = blue[i] = (int8_t)(oda[i] * (hi - lo) / 64 + lo);
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) {
            int8_t t = green[i * 8 + j];
            green[i * 8 + j] = green[i * 8 + 7 - j];
            green[i * 8 + 7 - j] = t;
            t = blue[j * 8 + i];
            blue[j * 8 + i] = blue[(7 - j) * 8 + i];
            blue[(7 - j) * 8 + i] = t;
        }
}

/* BufImgSurfaceData.c calculatePrimaryColorsApproximation: every corner cell
 * of the inverse map holds a colour within 5 of that corner's primary */
static int represents_primaries(const uint32_t* cmap, const uint8_t* cube)
{
    for (int i = 0; i < 32; i += 31)
        for (int j = 0; j < 32; j += 31)
            for (int k = 0; k < 32; k += 31) {
                const uint32_t c = cmap[cube[(i << 10) | (j << 5) | k]];
                const int r = (c >> 16) & 255, g = (c >> 8) & 255, b = c & 255;
                const int er = i ? 255 : 0, eg = j ? 255 : 0, eb = k ? 255 : 0;
                if (abs(r - er) > 5 || abs(g - eg) > 5 || abs(b - eb) > 5) return 0;
            }
    return 1;
}

static inline int clamp_byte(int c) { return (c >> 8) ? (~(c >> 31)) & 255 : c; }

int oracle_resize_indexed(const uint8_t* src, int sw, int sh, int sstride, const uint32_t* pal, int binary,
                          uint8_t* dst, int dw, int dh, int dstride)
{
    if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || !src || !dst || !pal) return 1;
    uint32_t dpal[256];
    int dn;
    oracle_default_palette(binary, dpal, &dn);
    uint8_t* cube = (uint8_t*)malloc(32768);
    if (!cube) return 2;
    oracle_inverse_cube(dpal, dn, cube);
    int8_t er[64], eg[64], eb[64];
    oracle_dither_tables(256, er, eg, eb);
    const int prims = represents_primaries(dpal, cube);
    double ix = 1.0 / ((double)dw / sw), iy = 1.0 / ((double)dh / sh);
    int64_t dxl = dbl_to_long(ix), dyl = dbl_to_long(iy);
    int64_t x0l = dbl_to_long(0.5 * ix), y0l = dbl_to_long(0.5 * iy);
    const int64_t half = (int64_t)1 << 31;
    for (int dy = 0; dy < dh; dy++) {
        int64_t yl = y0l + (int64_t)dy * dyl - half;
        int yw = (int)(yl >> 32), yf = (int)((uint32_t)yl >> 24), ya, yb;
        if (yw < 0) ya = yb = 0;
        else if (yw + 1 >= sh) ya = yb = yw;
        else { ya = yw; yb = yw + 1; }
        for (int dx = 0; dx < dw; dx++) {
            int64_t xl = x0l + (int64_t)dx * dxl - half;
            int xw = (int)(xl >> 32), xf = (int)((uint32_t)xl >> 24), xa, xb;
            if (xw < 0) xa = xb = 0;
            else if (xw + 1 >= sw) xa = xb = xw;
            else { xa = xw; xb = xw + 1; }
            const uint32_t q[4] = {pal[src[(size_t)ya * sstride + xa]], pal[src[(size_t)ya * sstride + xb]],
                                   pal[src[(size_t)yb * sstride + xa]], pal[src[(size_t)yb * sstride + xb]]};
            int pre[4][4];  /* [tap][b, g, r, a] */
            for (int s = 0; s < 4; s++) {
                const int a = (int)(q[s] >> 24);
                for (int b = 0; b < 3; b++) pre[s][b] = mul8(a, (int)(q[s] >> (8 * b)) & 255);
                pre[s][3] = a;
            }
            int v[3];
            for (int b = 0; b < 3; b++) {
                int top = (pre[0][b] << 8) + (pre[1][b] - pre[0][b]) * xf;
                int bot = (pre[2][b] << 8) + (pre[3][b] - pre[2][b]) * xf;
                v[b] = (((top << 8) + (bot - top) * yf) + (1 << 15)) >> 16;
            }
            /* SrcOver onto opaque black: the premultiplied colour */
            int r = v[2], g = v[1], b = v[0];
            if (!binary) {
                const int prim = (r == 0 || r == 255) && (g == 0 || g == 255) && (b == 0 || b == 255) && prims;
                if (!prim) {
                    const int e = (dy & 7) * 8 + (dx & 7);
                    r += er[e];
                    g += eg[e];
                    b += eb[e];
                }
                if ((r | g | b) >> 8) {
                    r = clamp_byte(r);
                    g = clamp_byte(g);
                    b = clamp_byte(b);
                }
            }
            dst[(size_t)dy * dstride + dx] = cube[((r >> 3) << 10) | ((g >> 3) << 5) | (b >> 3)];
        }
    }
    free(cube);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A2 + A4: compressJpgWithTargetSize / tryCachedParams                */
/* ------------------------------------------------------------------ */
int oracle_compress_jpg_with_target_size(const uint8_t* px, int w, int h, int stride, int fmt,
                                         int64_t target, float q0, int have_cached, float cached_q,
                                         double cached_scale, uint8_t* out, size_t cap, size_t* len,
                                         float* best_q, double* best_scale, int* encodes,
                                         int* cached_hit)
{
    int nch = (fmt == OR_GRAY8) ? 1 : 3;
    int n_enc = 0;
    if (cached_hit) *cached_hit = 0;
    uint8_t* tmp = (uint8_t*)malloc((size_t)w * h * nch);
    if (!tmp) return -2;
    if (have_cached) { /* tryCachedParams :216-238 */
        const uint8_t* img = px;
        int iw = w, ih = h, is = stride;
        if (cached_scale < 1.0) {
            oracle_scaled_dims(w, h, cached_scale, &iw, &ih);
            oracle_resize(px, w, h, stride, fmt, tmp, iw, ih, iw * nch);
            img = tmp;
            is = iw * nch;
        }
        size_t l = 0;
        int rc = oracle_encode(img, iw, ih, is, fmt, cached_q, out, cap, &l);
        n_enc++;
        if ((rc == 0 || rc == 4) && (int64_t)l <= target) {
            *len = l;
            *best_q = cached_q;
            *best_scale = cached_scale;
            if (encodes) *encodes = n_enc;
            if (cached_hit) *cached_hit = 1;
            free(tmp);
            return rc == 0 ? 1 : -4;
        }
    }
    const double STEP = 0.85; /* :91-115 */
    for (double scale = 1.0; scale > 0.1; scale = (scale == 1.0) ? STEP : scale * STEP) {
        const uint8_t* img = px;
        int iw = w, ih = h, is = stride;
        if (scale < 1.0) { /* every resize starts from the original (:99) */
            oracle_scaled_dims(w, h, scale, &iw, &ih);
            oracle_resize(px, w, h, stride, fmt, tmp, iw, ih, iw * nch);
            img = tmp;
            is = iw * nch;
        }
        int nt = 0;
        float best = oracle_find_best_quality(img, iw, ih, is, fmt, target, q0, NULL, NULL, &nt);
        n_enc += nt;
        if (best > 0) { /* saveCompressedImage re-encodes at best (:255-260) */
            size_t l = 0;
            int rc = oracle_encode(img, iw, ih, is, fmt, best, out, cap, &l);
            n_enc++;
            *len = l;
            *best_q = best;
            *best_scale = scale;
            if (encodes) *encodes = n_enc;
            free(tmp);
            return rc == 0 ? 1 : -4;
        }
    }
    if (encodes) *encodes = n_enc;
    free(tmp);
    return 0;
}

/* ------------------------------------------------------------------ */
/* A11, A13                                                             */
/* ------------------------------------------------------------------ */
int oracle_subsampling(int w, int h)
{ /* ImageCompression.java:140-153 */
    int maxd = w > h ? w : h;
    int s = 1;
    if (maxd > 4096) s = (int)floor((double)maxd / 4096);
    if (s > 1) {
        int hb = 1;
        while (hb * 2 <= s) hb *= 2;
        s = hb;
    }
    return s;
}

void oracle_create_key(int w, int h, int64_t file_size, int* wb, int* hb, int64_t* sb)
{ /* CacheTools.java:14-21 */
    *wb = w / 100;
    *hb = h / 100;
    *sb = file_size / 102400;
}

/* ------------------------------------------------------------------ */
/* thread pool batch (CompressionBatch.java:64-88 fixed pool)           */
/* ------------------------------------------------------------------ */
typedef struct {
    int n, fmt, have_cached;
    const uint8_t* const* px;
    const int *w, *h, *stride;
    int64_t target;
    float q0, cached_q;
    double cached_scale;
    int64_t* out_sizes;
    float* out_q;
    double* out_scale;
    long encodes;
    int next;
    pthread_mutex_t mu;
} batch_t;

static void* batch_worker(void* arg)
{
    batch_t* B = (batch_t*)arg;
    long enc = 0;
    for (;;) {
        pthread_mutex_lock(&B->mu);
        int i = B->next++;
        pthread_mutex_unlock(&B->mu);
        if (i >= B->n) break;
        int nch = (B->fmt == OR_GRAY8) ? 1 : 3;
        size_t cap = (size_t)B->w[i] * B->h[i] * nch * 2 + 4096;
        uint8_t* out = (uint8_t*)malloc(cap);
        size_t len = 0;
        float bq = -1;
        double bs = 0;
        int ne = 0;
        int rc = oracle_compress_jpg_with_target_size(B->px[i], B->w[i], B->h[i], B->stride[i], B->fmt,
                                                      B->target, B->q0, B->have_cached, B->cached_q,
                                                      B->cached_scale, out, cap, &len, &bq, &bs, &ne, NULL);
        free(out);
        enc += ne;
        if (B->out_sizes) B->out_sizes[i] = rc == 1 ? (int64_t)len : -1;
        if (B->out_q) B->out_q[i] = bq;
        if (B->out_scale) B->out_scale[i] = bs;
    }
    pthread_mutex_lock(&B->mu);
    B->encodes += enc;
    pthread_mutex_unlock(&B->mu);
    return NULL;
}

long oracle_fit_batch(int n, const uint8_t* const* px, const int* w, const int* h, const int* stride,
                      int fmt, int64_t target, float q0, int have_cached, float cached_q,
                      double cached_scale, int nthreads, int64_t* out_sizes, float* out_q,
                      double* out_scale)
{
    batch_t B = {n, fmt, have_cached, px, w, h, stride, target, q0, cached_q, cached_scale,
                 out_sizes, out_q, out_scale, 0, 0, PTHREAD_MUTEX_INITIALIZER};
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &B);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    return B.encodes;
}
