// icx_jpeg_parse.h — host-side JPEG marker parsing for the device decoder.
//
// The JDK reader (reached from ImageCompression.java:119-155) parses the
// header with libjpeg's jdmarker.c; this is the baseline subset the device
// decoder implements: SOF0/SOF1 8-bit, one interleaved scan (or a single grey
// component), Huffman coding, optional DRI; and SOF2 progressive files (8-bit
// Huffman, same components and sampling) whose scans icx_progressive.cpp
// decodes on the host; 3-component files in the colour space the JDK reader
// settles on (colour_space: YCbCr, or RGB without conversion).  Everything
// else (arithmetic, lossless, 12-bit, CMYK/YCCK, an unknown colour space,
// multi-scan sequential,
// 4:4:0 and exotic sampling) is reported as ICX_E_UNSUPPORTED with the image
// dimensions filled in, so the caller can still apply the dimension gate
// (ImageCompression.java:131) and route the file to a host decoder.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/icx.h"
#include "icx_decode.h"

namespace icx {

struct JpegHeader {
    int w = 0, h = 0, ncomp = 0, ri = 0;
    int id[4] = {}, hs[4] = {}, vs[4] = {}, tq[4] = {}, td[4] = {}, ta[4] = {};
    uint16_t qt[4][64] = {};  // natural order
    bool qt_ok[4] = {};
    uint8_t hbits[2][4][16] = {};   // [dc|ac][slot] counts per code length
    uint8_t hvals[2][4][256] = {};
    int hn[2][4] = {};
    bool h_ok[2][4] = {};
    size_t scan_off = 0;  // first byte of the entropy-coded segment (progressive: of the first scan)
    bool progressive = false;  // SOF2: td/ta/scan_off unused, prog_decode walks every scan
    bool rgb = false;          // 3 components stored as R, G, B (colour_space): no YCbCr conversion
    int cmyk = 0;              // 4 components: 1 CMYK, 2 YCCK (jdapimin.c default_decompress_parms)
};

// Parse markers up to the SOS.  `avail` bytes of the file are present at p
// (the file is `total` bytes long).  Returns ICX_OK, ICX_E_UNSUPPORTED (w, h,
// ncomp valid), ICX_E_CORRUPT, or ICX_E_BUFFER when more bytes are needed.
icx_status parse_jpeg(const uint8_t* p, size_t avail, size_t total, JpegHeader& J);

// 0 YCbCr, 1 RGB, -1 unknown: the JDK reader's colour space of a 3-component file.
int colour_space(const JpegHeader& J, bool jfif, bool exif, bool adobe, int transform);

// jpeg_make_d_derived_tbl equivalent; false if the table is invalid.
bool build_dec_huff(const uint8_t* bits, const uint8_t* vals, int n, DecHuff& t, DecSlow& slow);
void build_dec_lean(const DecHuff& h, bool ac, DecLean& lean);

// Per-image decode tables (distinct Huffman tables + per-component selectors,
// dequantisation per component).
bool build_dec_tab(const JpegHeader& J, DecTab& T);

// DecTab::sel packed 4 bits per entry, as dec_walk takes it.
uint32_t dec_selector(const DecTab& T);

// Entropy decode of a progressive file (icx_progressive.cpp) whose header
// parse_jpeg accepted: all scans into coefs (nblocks x 64, zeroed by the
// caller, natural order, MCU order as dec_geometry lays blocks out; DC value
// in [0]) and dc (nblocks DC values); qt receives each component's latched
// dequantisation table (natural order).  ICX_E_UNSUPPORTED: the JDK would
// block-smooth this file (AC 1..5 not fully refined); ICX_E_CORRUPT: any
// stream anomaly libjpeg would only warn about.
icx_status prog_decode(const uint8_t* p, size_t len, const JpegHeader& J, int16_t* coefs, int32_t* dc,
                       uint16_t (*qt)[64]);

// Entropy decode of a sequential Huffman file (icx_seqdecode.cpp) whose header
// parse_jpeg accepted, with IJG 6b's recovery semantics (fake EOI at the end
// of the file, zero MCUs after insufficient data, symbol 0 for a bad code,
// jdmarker.c's restart resynchronisation): coefs (nblocks x 64, natural
// order, MCU order as dec_geometry lays blocks out; DC value in [0]) and dc
// (nblocks DC values).  ICX_E_CORRUPT only where the JDK reader throws (a
// Huffman table the scan uses is invalid; a bad marker between the scan and
// EOI, which jpeg_finish_decompress reads).
icx_status seq_decode(const uint8_t* p, size_t len, const JpegHeader& J, int16_t* coefs, int32_t* dc);

}  // namespace icx
