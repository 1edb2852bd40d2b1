// dec_warmup_stats.cpp - CPU study of the decoder's relaxation:
// how often a k_dec_init warm-up estimate is the true entry state of its
// subsequence, how long the runs of consecutive wrong estimates are (= the
// re-walk launches a file needs), and whether K candidate warm-ups per
// subsequence (mode 0: lengths warm, 2 warm, ...; mode m > 0: start offsets
// warm + i * m bits; mode -1: warm-ups starting in each block of the MCU)
// would contain the true state.  Uses the product's state
// machine (icx_decode.h) on one JPEG file:
//   g++ -O2 -std=c++17 -I image-compression_amd/csrc -I include scripts/dec_warmup_stats.cpp \
//       image-compression_amd/csrc/icx_jpeg_parse.cpp -o /tmp/dws
//   /tmp/dws file.jpg [sub_bits=16384] [warm=8192] [K=4] [mode=0]
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include <set>
#include "icx_decode.h"
#include "icx_jpeg_parse.h"
using namespace icx;

int main(int argc, char** argv)
{
    FILE* f = fopen(argv[1], "rb");
    std::vector<uint8_t> jpg(20 << 20);
    size_t len = fread(jpg.data(), 1, jpg.size(), f);
    fclose(f);
    const uint32_t S = argc > 2 ? atoi(argv[2]) : 16384;
    const uint32_t warm = argc > 3 ? atoi(argv[3]) : 8192;
    JpegHeader J;
    if (parse_jpeg(jpg.data(), len, len, J)) return 1;
    static DecTab T;
    build_dec_tab(J, T);
    const uint32_t sel = dec_selector(T);
    DecDesc d{};
    d.ncomp = J.ncomp;
    d.hs = J.hs[0]; d.vs = J.vs[0]; d.nby = d.hs * d.vs; d.nbmcu = d.nby + 2;
    d.mcux = (J.w + 8 * d.hs - 1) / (8 * d.hs);
    d.mcuy = (J.h + 8 * d.vs - 1) / (8 * d.vs);
    d.ri = J.ri;
    d.nblocks = (int64_t)d.mcux * d.mcuy * d.nbmcu;
    d.wmcu = dec_walk_mcu(J.ncomp, d.nbmcu, J.td, J.ta);
    const uint8_t* sc = jpg.data() + J.scan_off;
    const int64_t sl = (int64_t)(len - J.scan_off);
    int64_t end = sl;
    for (int64_t i = 0; i + 1 < sl; i++)
        if (sc[i] == 0xFF && sc[i + 1] != 0x00 && sc[i + 1] != 0xFF && !(sc[i + 1] >= 0xD0 && sc[i + 1] <= 0xD7)) { end = i; break; }
    std::vector<uint8_t> ent;
    std::vector<uint32_t> seg{0};
    for (int64_t i = 0; i < end; i++) {
        int rst;
        const int k = dec_unstuff_rule(i ? sc[i - 1] : 0, sc[i], i + 1 < sl ? sc[i + 1] : 0, &rst);
        if (rst) { for (int p = 0; p < DEC_PAD; p++) ent.push_back(0xFF); seg.push_back((uint32_t)ent.size()); }
        else if (k) ent.push_back(sc[i]);
    }
    const uint32_t ent_len = (uint32_t)ent.size();
    for (int p = 0; p < DEC_TAIL + 64 + 4 * DEC_WIN; p++) ent.push_back(0xFF);
    while (ent.size() % 4) ent.push_back(0xFF);
    std::vector<uint32_t> words(ent.size() / 4 + 2, 0xFFFFFFFFu);
    memcpy(words.data(), ent.data(), ent.size());
    const uint32_t nsub = (ent_len * 8 + S - 1) / S;
    auto walk = [&](uint64_t st, uint32_t stop) {
        uint32_t n; NoSink ns;
        return dec_walk<false>(d, T.h, T.slow, sel, words.data(), seg.data(), (uint32_t)seg.size(), ent_len * 8, st, stop, n, 0, ns);
    };
    std::vector<uint64_t> tru(nsub + 1);
    tru[0] = dec_pack(0, 0, 0);
    for (uint32_t j = 0; j < nsub; j++) tru[j + 1] = walk(tru[j], (j + 1) * S);
    // candidate estimates: K warm-ups of lengths warm * (1 + m) ... or offsets
    const int K = argc > 4 ? atoi(argv[4]) : 4;
    const int mode = argc > 5 ? atoi(argv[5]) : 0;
    std::vector<std::vector<uint64_t>> cand(nsub + 1);
    int hit1 = 0, hitK = 0, posok = 0;
    std::vector<int> ok1(nsub + 1, 1), okK(nsub + 1, 1);
    for (uint32_t j = 1; j < nsub; j++) {
        std::set<uint64_t> cs;
        for (int m = 0; m < K; m++) {
            // mode -1: one warm-up per starting block of the MCU (block phase m)
            uint32_t w = mode == 0 ? warm * (m + 1) : mode < 0 ? warm : warm + m * (mode);
            const int b0 = mode < 0 ? m % d.nbmcu : 0;
            uint64_t e = walk(dec_pack(j * S > w ? j * S - w : 0, b0, 0), j * S);
            if (m == 0) { ok1[j] = e == tru[j]; hit1 += ok1[j]; posok += dec_pos(e) == dec_pos(tru[j]); }
            cs.insert(e);
        }
        okK[j] = cs.count(tru[j]) > 0;
        hitK += okK[j];
        cand[j].assign(cs.begin(), cs.end());
    }
    auto chain = [&](const std::vector<int>& ok) {
        int best = 0, run = 0; long tot = 0;
        for (uint32_t j = 1; j < nsub; j++) { if (!ok[j]) { run++; tot++; best = std::max(best, run); } else run = 0; }
        return std::make_pair(best, tot);
    };
    auto c1 = chain(ok1), cK = chain(okK);
    size_t ncand = 0; for (auto& c : cand) ncand += c.size();
    printf("nsub %u  warm-up hit %.4f (pos ok %.4f)  K=%d hit %.4f  mean distinct cands %.2f  max miss run: 1 -> %d, K -> %d  misses %ld -> %ld\n",
           nsub, hit1 / double(nsub - 1), posok / double(nsub - 1), K, hitK / double(nsub - 1), ncand / double(nsub - 1),
           c1.first, cK.first, c1.second, cK.second);
    return 0;
}
