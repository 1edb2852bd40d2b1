// asan_parse.cpp — TEST INFRASTRUCTURE: host-side header parser and Huffman
// table builder of the device decoder (csrc/icx_jpeg_parse.cpp) under
// AddressSanitizer + UBSan.  Built and run by tests/test_parse_asan.py.
//
// Over-subscribed DHT code counts must be rejected (jdhuff.c
// jpeg_make_d_derived_tbl: JERR_BAD_HUFF_TABLE -> ICX_E_CORRUPT in the
// product) without any write past DecHuff::lut, and the parser must survive
// truncated and bit-flipped headers.  Exit status 0 = every expectation held;
// a sanitizer report aborts with a nonzero status.
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "icx_jpeg_parse.h"

using namespace icx;

static int failures = 0;
#define EXPECT(c)                                                   \
    do {                                                            \
        if (!(c)) {                                                 \
            fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #c); \
            failures++;                                             \
        }                                                           \
    } while (0)

// ITU-T T.81 Annex K.3: luminance DC and AC code counts (valid tables)
static const uint8_t kDcBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t kAcBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};

static bool build(const uint8_t* bits)
{
    int n = 0;
    for (int l = 0; l < 16; l++) n += bits[l];
    std::vector<uint8_t> vals(256);
    for (int i = 0; i < 256; i++) vals[i] = (uint8_t)i;
    // heap-allocated so ASan sees the exact object bounds
    DecHuff* t = new DecHuff;
    DecSlow* s = new DecSlow;
    const bool ok = n <= 256 && build_dec_huff(bits, vals.data(), n, *t, *s);
    delete t;
    delete s;
    return ok;
}

int main()
{
    EXPECT(build(kDcBits));
    EXPECT(build(kAcBits));
    {   // three 1-bit codes (the advisor's example): would write lut[1024..]
        uint8_t b[16] = {3};
        EXPECT(!build(b));
    }
    {   // 255 one-bit codes
        uint8_t b[16] = {255};
        EXPECT(!build(b));
    }
    {   // two 1-bit codes: the second is the all-ones code
        uint8_t b[16] = {2};
        EXPECT(!build(b));
        uint8_t c[16] = {1, 1};  // '0', '10': valid
        EXPECT(build(c));
        uint8_t d[16] = {1, 2};  // '0', '10', '11': all-ones
        EXPECT(!build(d));
    }
    {   // codes '0', '10', ..., '111111110' leave the one 9-bit prefix '111111111':
        // 2^(l-9) codes of length l > 9 remain, the last of them all-ones
        for (int l = 12; l <= 16; l += 4) {
            uint8_t b[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1};
            const int room = 1 << (l - 9);
            b[l - 1] = (uint8_t)(room - 1);
            EXPECT(build(b));
            b[l - 1] = (uint8_t)room;  // takes the all-ones code
            EXPECT(!build(b));
            b[l - 1] = (uint8_t)(room + 1);  // over-subscribed: old code wrote lut[1024]
            EXPECT(!build(b));
        }
    }

    // header parser on truncated and bit-flipped copies of a small valid
    // header (SOI, DQT, SOF0, DHT x2, SOS): must never read out of bounds
    std::vector<uint8_t> hdr = {0xFF, 0xD8};
    auto seg = [&](uint8_t m, const std::vector<uint8_t>& p) {
        hdr.push_back(0xFF);
        hdr.push_back(m);
        hdr.push_back((uint8_t)((p.size() + 2) >> 8));
        hdr.push_back((uint8_t)(p.size() + 2));
        hdr.insert(hdr.end(), p.begin(), p.end());
    };
    std::vector<uint8_t> dqt(65, 1);
    dqt[0] = 0;
    seg(0xDB, dqt);
    seg(0xC0, {8, 0, 16, 0, 16, 1, 1, 0x11, 0});
    std::vector<uint8_t> dht = {0x00};
    dht.insert(dht.end(), kDcBits, kDcBits + 16);
    for (int i = 0; i < 12; i++) dht.push_back((uint8_t)i);
    seg(0xC4, dht);
    std::vector<uint8_t> aht = {0x10};
    aht.insert(aht.end(), kAcBits, kAcBits + 16);
    for (int i = 0; i < 162; i++) aht.push_back((uint8_t)i);
    seg(0xC4, aht);
    seg(0xDA, {1, 1, 0x00, 0, 63, 0});
    hdr.push_back(0x00);
    {
        JpegHeader J;
        EXPECT(parse_jpeg(hdr.data(), hdr.size(), hdr.size(), J) == ICX_OK);
        DecTab* T = new DecTab;
        EXPECT(build_dec_tab(J, *T));
        delete T;
    }
    {   // the same header with an over-subscribed DC table: parses, tables rejected
        std::vector<uint8_t> bad = hdr;
        for (size_t i = 0; i + 1 < bad.size(); i++)
            if (bad[i] == 0xFF && bad[i + 1] == 0xC4) {
                bad[i + 5] = 0x00;  // class/id byte stays DC 0
                bad[i + 5 + 1] = 3;  // three 1-bit codes
                break;
            }
        JpegHeader J;
        const icx_status st = parse_jpeg(bad.data(), bad.size(), bad.size(), J);
        DecTab* T = new DecTab;
        EXPECT(st != ICX_OK || !build_dec_tab(J, *T));
        delete T;
    }
    std::mt19937 rng(1234);
    for (int it = 0; it < 20000; it++) {
        std::vector<uint8_t> f = hdr;
        const int flips = 1 + (int)(rng() % 4);
        for (int k = 0; k < flips; k++) f[rng() % f.size()] ^= (uint8_t)(1u << (rng() % 8));
        const size_t len = (it & 1) ? f.size() : 2 + rng() % (f.size() - 1);
        // exact-size heap copy so any overread is caught
        uint8_t* p = new uint8_t[len];
        memcpy(p, f.data(), len);
        JpegHeader J;
        if (parse_jpeg(p, len, len, J) == ICX_OK) {
            DecTab* T = new DecTab;
            build_dec_tab(J, *T);
            delete T;
        }
        delete[] p;
    }
    if (failures) {
        fprintf(stderr, "%d expectation(s) failed\n", failures);
        return 1;
    }
    printf("asan_parse: ok\n");
    return 0;
}
