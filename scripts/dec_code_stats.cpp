// dec_code_stats.cpp - CPU count of how often the decoder's symbol step needs
// a Huffman table's second level (codes longer than DEC_LUT_BITS): the write
// pass keeps only first levels in LDS, so such a symbol is a global-memory
// load in the walk (and, on a 64-lane wave, any lane needing it stalls the
// wave).  Walks the true path of one JPEG file with the product's state
// machine (icx_decode.h):
//   g++ -O2 -std=c++17 -I image-compression_amd/csrc -I include scripts/dec_code_stats.cpp \
//       image-compression_amd/csrc/icx_jpeg_parse.cpp -o /tmp/dcs && /tmp/dcs file.jpg
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <vector>
#include "icx_decode.h"
#include "icx_jpeg_parse.h"
using namespace icx;

int main(int argc, char** argv)
{
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    std::vector<uint8_t> jpg(40 << 20);
    size_t len = fread(jpg.data(), 1, jpg.size(), f);
    fclose(f);
    JpegHeader J;
    if (parse_jpeg(jpg.data(), len, len, J)) return 1;
    static DecTab T;
    build_dec_tab(J, T);
    const uint32_t sel = dec_selector(T);
    DecDesc d{};
    d.ncomp = J.ncomp;
    d.hs = J.hs[0]; d.vs = J.vs[0]; d.nby = d.hs * d.vs; d.nbmcu = J.ncomp == 3 ? d.nby + 2 : 1;
    d.wmcu = dec_walk_mcu(J.ncomp, d.nbmcu, J.td, J.ta);
    const uint8_t* sc = jpg.data() + J.scan_off;
    const int64_t sl = (int64_t)(len - J.scan_off);
    std::vector<uint8_t> ent;
    std::vector<uint32_t> seg{0};
    for (int64_t i = 0; i < sl; i++) {
        if (sc[i] == 0xFF && i + 1 < sl && sc[i + 1] != 0x00 && sc[i + 1] != 0xFF && !(sc[i + 1] >= 0xD0 && sc[i + 1] <= 0xD7)) break;
        int rst;
        const int k = dec_unstuff_rule(i ? sc[i - 1] : 0, sc[i], i + 1 < sl ? sc[i + 1] : 0, &rst);
        if (rst) { for (int p = 0; p < DEC_PAD; p++) ent.push_back(0xFF); seg.push_back((uint32_t)ent.size()); }
        else if (k) ent.push_back(sc[i]);
    }
    const uint32_t ent_bits = (uint32_t)ent.size() * 8;
    for (int p = 0; p < DEC_TAIL + 64 + 4 * DEC_WIN; p++) ent.push_back(0xFF);
    while (ent.size() % 4) ent.push_back(0xFF);
    std::vector<uint32_t> words(ent.size() / 4 + 2, 0xFFFFFFFFu);
    memcpy(words.data(), ent.data(), ent.size());
    DecLeanWalker<const DecLean*> w = dec_lean_walker(d, (const DecLean*)T.lean, T.slow, sel, words.data(), seg.data(),
                                                      (uint32_t)seg.size(), ent_bits);
    w.start(dec_pack(0, 0, 0));
    uint64_t sym = 0, second = 0, slow = 0, dc = 0;
    while (w.running(ent_bits)) {
        w.R.refill();
        const uint32_t pk = w.R.peek16();
        const uint32_t e = T.lean[w.ti].lut[pk >> (16 - DEC_LUT_BITS)];
        if (!(e & 31) && e) {
            second++;
            if (e & DEC_SLOW) slow++;
        }
        if (w.z == 0) dc++;
        w.step();
        sym++;
    }
    const double p = (double)second / sym;
    printf("{\"file\": \"%s\", \"bits\": %u, \"symbols\": %llu, \"bits_per_symbol\": %.2f, \"dc_symbols\": %llu, "
           "\"second_level\": %llu, \"slow\": %llu, \"p\": %.5f, \"p_any_of_64\": %.4f, \"blocks\": %u}\n",
           argv[1], ent_bits, (unsigned long long)sym, (double)ent_bits / sym, (unsigned long long)dc,
           (unsigned long long)second, (unsigned long long)slow, p, 1 - pow(1 - p, 64), w.n);
    return 0;
}
