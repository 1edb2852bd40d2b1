// dec_emu.cpp — TEST INFRASTRUCTURE: serial CPU emulation of the device JPEG
// entropy decoder's algorithm (unstuff -> self-synchronising subsequence
// decode -> block offsets -> coefficient write -> DC prediction), built from
// the product's own state machine (image-compression_amd/csrc/icx_decode.h)
// and header parser.  Lets the CPU suite check the synchronisation logic
// against the oracle's coefficients; the GPU tests check the kernels.
//
// "Threads" of one sync launch run in a shuffled order and read entry states
// that other threads of the same launch may already have rewritten, which is
// the interleaving the device kernel allows.
#include <stdint.h>
#include <string.h>

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "icx_decode.h"
#include "icx_jpeg_parse.h"

using namespace icx;

extern "C" {
long dec_emu_walks = 0;  // subsequence walks in the sync launches of the last call (work measure)
long dec_emu_nsub = 0;
long dec_emu_early = 0;  // re-walks that stopped at a checkpoint of their previous walk
}

extern "C" int dec_emu_coefs(const uint8_t* jpg, size_t len, int16_t* out, size_t nblocks_cap, int seed,
                             int sub_bits, int* iterations)
{
    const bool warm_up = seed % 2 == 0;  // odd seeds: plain guesses, even seeds: warm-up estimates (k_dec_init)
    JpegHeader J;
    icx_status st = parse_jpeg(jpg, len, len, J);
    if (st) return (int)st;
    static DecTab T;
    if (!build_dec_tab(J, T)) return ICX_E_CORRUPT;
    const uint32_t sel = dec_selector(T);
    DecDesc d{};
    d.ncomp = J.ncomp;
    if (J.ncomp == 3) {
        d.hs = J.hs[0];
        d.vs = J.vs[0];
        d.nby = d.hs * d.vs;
        d.nbmcu = d.nby + 2;
        d.mcux = (J.w + 8 * d.hs - 1) / (8 * d.hs);
        d.mcuy = (J.h + 8 * d.vs - 1) / (8 * d.vs);
    } else if (J.ncomp == 4) {  // CMYK / YCCK: four 1x1 components (icx_decode.cpp dec_geometry)
        d.hs = d.vs = 1;
        d.nby = 1;
        d.nbmcu = 4;
        d.mcux = (J.w + 7) / 8;
        d.mcuy = (J.h + 7) / 8;
    } else {
        d.hs = d.vs = 1;
        d.nby = d.nbmcu = 1;
        d.mcux = (J.w + 7) / 8;
        d.mcuy = (J.h + 7) / 8;
    }
    d.ri = J.ri;
    d.nblocks = (int64_t)d.mcux * d.mcuy * d.nbmcu;
    d.wmcu = dec_walk_mcu(J.ncomp, d.nbmcu, J.td, J.ta);
    if ((size_t)d.nblocks > nblocks_cap) return ICX_E_BUFFER;

    // ---- unstuff
    const uint8_t* sc = jpg + J.scan_off;
    const int64_t sl = (int64_t)(len - J.scan_off);
    int64_t end = sl;
    for (int64_t i = 0; i + 1 < sl; i++)
        if (sc[i] == 0xFF && sc[i + 1] != 0x00 && sc[i + 1] != 0xFF && !(sc[i + 1] >= 0xD0 && sc[i + 1] <= 0xD7)) {
            end = i;
            break;
        }
    // as k_unstuff_scan: trailing FFs at the end of the file start the fake
    // EOI; a scan that ends at a marker other than EOI, or an RSTn out of
    // sequence (below), is not the clean case
    bool fake = false;
    if (end == sl && sl > 0 && sc[sl - 1] == 0xFF) {
        end = sl - 1;
        while (end > 0 && sc[end - 1] == 0xFF) end--;
        fake = true;
    }
    if (!fake && end + 1 < sl && sc[end + 1] != 0xD9) return ICX_E_CORRUPT;
    std::vector<uint8_t> ent;
    std::vector<uint32_t> seg{0};
    for (int64_t i = 0; i < end; i++) {
        int rst;
        const int k = dec_unstuff_rule(i ? sc[i - 1] : 0, sc[i], i + 1 < sl ? sc[i + 1] : 0, &rst);
        if (rst) {
            if ((sc[i] & 7) != ((seg.size() - 1) & 7)) return ICX_E_CORRUPT;
            for (int p = 0; p < DEC_PAD; p++) ent.push_back(0xFF);
            seg.push_back((uint32_t)ent.size());
        } else if (k) {
            ent.push_back(sc[i]);
        }
    }
    const uint32_t ent_len = (uint32_t)ent.size();
    for (int p = 0; p < DEC_TAIL + 64 + 4 * DEC_WIN_MAX; p++) ent.push_back(0xFF);
    while (ent.size() % 4) ent.push_back(0xFF);
    std::vector<uint32_t> words(ent.size() / 4 + 2, 0xFFFFFFFFu);
    memcpy(words.data(), ent.data(), ent.size());

    // ---- self-synchronising decode
    const uint32_t S = (uint32_t)sub_bits;
    const uint32_t nsub = (ent_len * 8 + S - 1) / S;
    std::vector<uint64_t> est(nsub + 1);
    std::vector<uint32_t> ncnt(nsub, 0);
    uint32_t warm = std::min<uint32_t>(4096, S / 4);  // as icx_decode.cpp warm_bits
    if (const char* e = getenv("ICX_DEC_WARM")) warm = (uint32_t)atol(e);
    for (uint32_t j = 0; j <= nsub; j++) {
        est[j] = dec_pack(j * S, 0, 0);
        if (j > 0 && j < nsub && warm_up) {
            uint32_t n;
            est[j] = dec_lean_walk(d, (const DecLean*)T.lean, T.slow, sel, words.data(), seg.data(),
                                   (uint32_t)seg.size(), ent_len * 8, dec_pack(j * S > warm ? j * S - warm : 0, 0, 0),
                                   j * S, n);
        }
    }
    std::mt19937 rng((uint32_t)seed);
    // launch 0 walks everything; launch r > 0 walks the worklist launch r-1 appended to (as k_dec_sync)
    std::vector<uint32_t> work(nsub);
    for (uint32_t j = 0; j < nsub; j++) work[j] = j;
    int it = 0;
    dec_emu_walks = 0;
    dec_emu_nsub = nsub;
    // checkpoints as k_dec_sync: launch 0 records, later launches compare and stop early
    const int nck = dec_ck_slots(S);
    std::vector<uint64_t> ck((size_t)(nsub + 1) * DEC_CK_MAX, 0x5A5A5A5A5A5A5A5Aull);
    dec_emu_early = 0;
    for (;; it++) {
        if (it > (int)nsub + 2) return ICX_E_CORRUPT;  // cannot happen: one subsequence settles per launch
        if (seed) std::shuffle(work.begin(), work.end(), rng);
        std::vector<uint32_t> next;
        for (uint32_t j : work) {
            dec_emu_walks++;
            uint32_t n;
            bool early;
            uint64_t x;
            uint64_t* mine = ck.data() + (size_t)j * DEC_CK_MAX;
            if (it == 0) {
                CkRecord<uint64_t*> rec{mine, nck};
                x = dec_sync_walk(d, (const DecLean*)T.lean, T.slow, sel, words.data(), seg.data(), (uint32_t)seg.size(), ent_len * 8,
                                  est[j], j * S, S, n, early, rec);
            } else {
                CkInPlace<uint64_t*> cmp{mine, nck, ncnt[j], nck > 0 ? mine[0] : DEC_CK_NONE};
                x = dec_sync_walk(d, (const DecLean*)T.lean, T.slow, sel, words.data(), seg.data(), (uint32_t)seg.size(), ent_len * 8,
                                  est[j], j * S, S, n, early, cmp);
                if (early) dec_emu_early++;
            }
            ncnt[j] = n;
            if (!early && x != est[j + 1]) {
                est[j + 1] = x;
                if (j + 1 < nsub) next.push_back(j + 1);
            }
        }
        if (next.empty()) break;
        work.swap(next);
    }
    if (iterations) *iterations = it + 1;
    std::vector<uint32_t> boff(nsub + 1, 0);
    for (uint32_t j = 0; j < nsub; j++) boff[j + 1] = boff[j] + ncnt[j];
    if ((int64_t)boff[nsub] != d.nblocks) return ICX_E_CORRUPT;

    // ---- write pass: blocks owned by the subsequence where their DC starts,
    // assembled in a per-thread buffer and flushed whole (no pre-zeroing:
    // the coefficient array starts as garbage to prove every block is written)
    std::vector<int16_t> coefs((size_t)d.nblocks * 64, (int16_t)0x5A5A);
    std::vector<int32_t> dc((size_t)d.nblocks, 0x5A5A5A5A);
    d.coefs = coefs.data();
    d.dc = dc.data();
    struct Sink {
        int16_t buf[65] = {};  // [64]: the discard slot
        int16_t* out;
        int32_t* dcs;
        void put(int z, int v) { buf[z < 64 ? dec_nat(z) : 64] = (int16_t)v; }
        void put2(int z2, int v) { put(z2 >> 1, v); }
        void flush_if(bool c, int64_t bi)
        {
            if (!c) return;
            memcpy(out + bi * 64, buf, 64 * sizeof(int16_t));
            dcs[bi] = buf[0];
            memset(buf, 0, sizeof(buf));
        }
    };
    // (as k_dec_write: one walk per piece of a subsequence, split at its checkpoints)
    bool bad = false;
    const int np = dec_pieces(S);
    std::vector<uint32_t> order((size_t)nsub * np);
    for (uint32_t t = 0; t < order.size(); t++) order[t] = t;
    if (seed) std::shuffle(order.begin(), order.end(), rng);
    for (uint32_t t : order) {
        Sink sk;
        sk.out = coefs.data();
        sk.dcs = dc.data();
        const uint32_t j = t / np;
        const DecPiece pc = dec_piece(est.data(), ck.data(), boff.data(), j, (int)(t % np), S);
        if (!pc.have || (dec_pos(pc.e) >= pc.stop && (pc.e & 63) == 0)) continue;
        DecLeanWriter<const DecLean*> w = dec_lean_writer(d, (const DecLean*)T.lean, T.slow, sel, words.data(),
                                                          seg.data(), (uint32_t)seg.size(), ent_len * 8, pc.blk);
        w.start(pc.e);
        while (w.running(pc.stop)) w.step(sk);
        bad |= w.bad || (pc.have && w.overran());  // as k_dec_write: not the clean case
    }
    if (bad) return ICX_E_CORRUPT;
    // ---- DC prediction per component, reset every restart interval
    int pred[4] = {0, 0, 0, 0};
    for (int64_t b = 0; b < d.nblocks; b++) {
        const int64_t m = b / d.nbmcu;
        const int k = (int)(b % d.nbmcu);
        if (k == 0 && d.ri && m % d.ri == 0) pred[0] = pred[1] = pred[2] = pred[3] = 0;
        const int c = k < d.nby ? 0 : k - d.nby + 1;
        pred[c] += dc[b];
        coefs[(size_t)b * 64] = (int16_t)pred[c];
    }
    memcpy(out, coefs.data(), coefs.size() * sizeof(int16_t));
    return 0;
}

// DecLeanWalker (k_dec_init / k_dec_sync) against DecWalker<false> (the write
// pass's state machine): from `nstarts` random states - any bit position,
// block-in-MCU and zig-zag index, i.e. mostly wrong-start paths, which meet
// invalid codes, overshooting runs and interval jumps - both walk `steps`
// symbols and must agree on the state and block count after every one.
// Returns the number of disagreeing steps (0), or a negative status.
extern "C" long dec_emu_pairs = 0;  // symbol-pair steps the lean checks met (all calls)
extern "C" long dec_emu_lean_check(const uint8_t* jpg, size_t len, int nstarts, int steps, int seed)
{
    JpegHeader J;
    icx_status st = parse_jpeg(jpg, len, len, J);
    if (st) return -(long)st;
    static DecTab T;
    if (!build_dec_tab(J, T)) return -(long)ICX_E_CORRUPT;
    const uint32_t sel = dec_selector(T);
    DecDesc d{};
    d.ncomp = J.ncomp;
    d.nby = J.ncomp == 3 ? J.hs[0] * J.vs[0] : 1;
    d.nbmcu = J.ncomp == 3 ? d.nby + 2 : J.ncomp == 4 ? 4 : 1;
    d.wmcu = dec_walk_mcu(J.ncomp, d.nbmcu, J.td, J.ta);
    d.ri = J.ri;
    const uint8_t* sc = jpg + J.scan_off;
    const int64_t sl = (int64_t)(len - J.scan_off);
    std::vector<uint8_t> ent;
    std::vector<uint32_t> seg{0};
    for (int64_t i = 0; i < sl; i++) {
        if (i + 1 < sl && sc[i] == 0xFF && sc[i + 1] != 0x00 && sc[i + 1] != 0xFF && !(sc[i + 1] >= 0xD0 && sc[i + 1] <= 0xD7))
            break;
        int rst;
        const int k = dec_unstuff_rule(i ? sc[i - 1] : 0, sc[i], i + 1 < sl ? sc[i + 1] : 0, &rst);
        if (rst) {
            for (int p = 0; p < DEC_PAD; p++) ent.push_back(0xFF);
            seg.push_back((uint32_t)ent.size());
        } else if (k) {
            ent.push_back(sc[i]);
        }
    }
    const uint32_t ent_len = (uint32_t)ent.size();
    if (!ent_len) return 0;
    for (int p = 0; p < DEC_TAIL + 64 + 4 * DEC_WIN_MAX; p++) ent.push_back(0xFF);
    while (ent.size() % 4) ent.push_back(0xFF);
    std::vector<uint32_t> words(ent.size() / 4 + 2, 0xFFFFFFFFu);
    memcpy(words.data(), ent.data(), ent.size());
    std::mt19937 rng((uint32_t)seed);
    long bad = 0, pairs = 0;
    for (int s = 0; s < nstarts; s++) {
        const uint64_t e0 = dec_pack(rng() % (ent_len * 8), (int)(rng() % (uint32_t)d.wmcu), (int)(rng() % 64));
        DecWalker<false, const DecHuff*> a = dec_walker<false>(d, (const DecHuff*)T.h, T.slow, sel, words.data(),
                                                               seg.data(), (uint32_t)seg.size(), ent_len * 8, 0);
        DecLeanWalker<const DecLean*> b = dec_lean_walker(d, (const DecLean*)T.lean, T.slow, sel, words.data(),
                                                          seg.data(), (uint32_t)seg.size(), ent_len * 8);
        a.start(e0);
        b.start(e0);
        NoSink ns;
        for (int k = 0; k < steps && a.running(DEC_END) && b.running(DEC_END); k++) {
            a.step(ns);
            if (rng() % 4 == 0) {  // an idle lane's step (device loops) changes no state or count
                // (on a copy: a lane never walks again after an idle step, and its next-table
                // index may move - ICX_DEC_BSEL32's table_after)
                DecLeanWalker<const DecLean*> c = b;
                c.step(false);
                if (c.state() != b.state() || c.n != b.n) {
                    bad++;
                    break;
                }
            }
            b.step();
            if (b.two) {  // a symbol pair: the spec's next symbol too (the same block's next AC code)
                pairs++;
                if (!a.running(DEC_END) || a.z == 0) {
                    bad++;
                    break;
                }
                a.step(ns);
            }
            if (a.state() != b.state() || a.n != b.n) {
                bad++;
                break;
            }
        }
        if (a.running(DEC_END) != b.running(DEC_END)) bad++;
    }
    // the write walks: every sink call (index, value; flushed block) in order
    struct Rec {
        std::vector<int64_t> ev;
        // the value puts; a 0 lands in a zeroed slot position that nothing
        // else writes in the block, so where it lands is free (the lean writer
        // puts a size-0 symbol's 0 at the end of its zero run, DecWalker at z)
        void put(int z, int v)
        {
            if (v) ev.push_back(((int64_t)z << 32) ^ (uint32_t)v);
        }
        void put2(int z2, int v) { put(z2 >> 1, v); }
        void flush_if(bool c, int64_t bi)
        {
            if (c) ev.push_back(-1 - bi);
        }
    };
    d.nblocks = 1 << 20;
    for (int s = 0; s < nstarts; s++) {
        const uint64_t e0 = dec_pack(rng() % (ent_len * 8), (int)(rng() % (uint32_t)d.wmcu), (int)(rng() % 64));
        const int64_t base = (int64_t)(rng() % 4096);
        DecWalker<true, const DecHuff*> a = dec_walker<true>(d, (const DecHuff*)T.h, T.slow, sel, words.data(),
                                                             seg.data(), (uint32_t)seg.size(), ent_len * 8, base);
        DecLeanWriter<const DecLean*> b = dec_lean_writer(d, (const DecLean*)T.lean, T.slow, sel, words.data(),
                                                          seg.data(), (uint32_t)seg.size(), ent_len * 8, base);
        a.start(e0);
        b.start(e0);
        Rec ra, rb;
        for (int k = 0; k < steps && a.running(DEC_END) && b.running(DEC_END); k++) {
            a.step(ra);
            b.step(rb);
            if (b.two) {
                pairs++;
                if (!a.running(DEC_END) || a.z == 0) {
                    bad++;
                    break;
                }
                a.step(ra);
            }
            if (a.state() != b.state() || a.n != b.n || a.bad != b.bad || (a.own != 0) != (b.own != 0)) {
                bad++;
                break;
            }
        }
        if (ra.ev != rb.ev) bad++;
    }
    dec_emu_pairs += pairs;
    return bad;
}

