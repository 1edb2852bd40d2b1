// icx_decode.cpp — host driver of the device JPEG decoder (row A11), behind
// icx_decode_jpg / icx_decode_jpg_batch / icx_jpeg_info in include/icx.h.
//
// Replaces ImageCompression.decodeImageWithSubsampling's JPEG read
// (core/ImageCompression.java:107-165): the JDK JPEGImageReader with
// ImageReadParam.setSourceSubsampling(s, s, 0, 0) and ignoreMetadata = true.
// Per sub-batch: headers are parsed on the host (icx_jpeg_parse.cpp), the
// entropy-coded segments are copied to HBM once, and everything else —
// unstuffing, the self-synchronising Huffman decode (icx_decode.h), DC
// prediction, IDCT, upsampling, colour conversion and subsampling — runs as
// launches on the context's stream.  The host synchronises once per few sync
// launches (to learn whether the entry states have settled) and once at the end.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/icx.h"
#include "icx_context.h"
#include "icx_decode.h"
#include "icx_decode_kernels.h"
#include "icx_jpeg_parse.h"

using namespace icx;

namespace {

struct DecItem {
    icx_decode_job* job;
    JpegHeader J;
    bool dev_in = false, host_out = false;
    int nch = 3, s = 1;
    int64_t ntiles = 0, nsub_max = 0, nblocks = 0;
    size_t ent_cap = 0;
};

// Headers of device-resident files: their first bytes are gathered into one
// device buffer by k_stage and downloaded in one copy; a file whose header runs
// past what was fetched goes again with 8x more (4 KiB, 32 KiB, ...).
icx_status fetch_headers(icx_ctx* c, const icx_decode_job* jobs, int n, const std::vector<char>& dev_in,
                         std::vector<JpegHeader>& J, std::vector<icx_status>& st)
{
    std::vector<int> pend;
    std::vector<size_t> avail(n, 0);
    for (int i = 0; i < n; i++)
        if (dev_in[i]) {
            pend.push_back(i);
            avail[i] = std::min<size_t>(jobs[i].len, 4096);
        }
    while (!pend.empty()) {
        const int m = (int)pend.size();
        size_t bytes = 0;
        for (int i : pend) bytes += align_up(avail[i], 64);
        const size_t up = Uploader::need<StageJob>(m) + Uploader::need<int64_t>(m + 1);
        hipError_t e = c->dev.reserve(bytes + up + 4096);
        if (e == hipSuccess) e = c->host.reserve(bytes + up + 4096);
        if (e != hipSuccess) return hip_fail(c, e, "header staging");
        c->dev.used = c->host.used = 0;
        uint8_t* dbuf = (uint8_t*)c->dev.take(bytes);
        uint8_t* hbuf = (uint8_t*)c->host.take(bytes);
        Uploader U(c, up);
        StageJob* hj;
        int64_t* hp;
        const StageJob* dj = U.alloc<StageJob>(m, &hj);
        const int64_t* dp = U.alloc<int64_t>(m + 1, &hp);
        if (U.overflow || !hbuf) return fail(c, ICX_E_NOMEM, "header staging exhausted");
        std::vector<size_t> at(m);
        size_t off = 0;
        hp[0] = 0;
        for (int k = 0; k < m; k++) {
            const int i = pend[k];
            const int64_t dl = (int64_t)align_up(avail[i], 16);
            hj[k] = StageJob{jobs[i].data, dbuf + off, (int64_t)avail[i], dl};
            hp[k + 1] = hp[k] + (dl + STAGE_TILE - 1) / STAGE_TILE;
            at[k] = off;
            off += align_up(avail[i], 64);
        }
        const int64_t nwg = hp[m];
        if (icx_status s = U.flush()) return s;
        launch_stage(dj, Plan{nullptr, dp, m}, nwg, c->stream);
        e = hipMemcpyAsync(hbuf, dbuf, bytes, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "header download");
        std::vector<int> next;
        for (int k = 0; k < m; k++) {
            const int i = pend[k];
            st[i] = parse_jpeg(hbuf + at[k], avail[i], jobs[i].len, J[i]);
            if (st[i] == ICX_E_BUFFER && avail[i] < jobs[i].len) {
                avail[i] = std::min<size_t>(jobs[i].len, avail[i] * 8);
                next.push_back(i);
            }
        }
        pend.swap(next);
    }
    return ICX_OK;
}

// Geometry of the decode (jdmaster.c jpeg_calc_output_dimensions / per-component dims).
void dec_geometry(const JpegHeader& J, int s, DecDesc& d)
{
    d.w = J.w;
    d.h = J.h;
    d.ncomp = J.ncomp;
    d.ri = J.ri;
    if (J.ncomp == 3) {
        d.hs = J.hs[0];
        d.vs = J.vs[0];
        d.nby = d.hs * d.vs;
        d.nbmcu = d.nby + 2;
        d.mcux = (J.w + 8 * d.hs - 1) / (8 * d.hs);
        d.mcuy = (J.h + 8 * d.vs - 1) / (8 * d.vs);
    } else if (J.ncomp == 4) {  // CMYK / YCCK, every component 1x1: four blocks per MCU
        d.hs = d.vs = 1;
        d.nby = 1;
        d.nbmcu = 4;
        d.mcux = (J.w + 7) / 8;
        d.mcuy = (J.h + 7) / 8;
    } else {  // non-interleaved single component: one block per MCU
        d.hs = d.vs = 1;
        d.nby = d.nbmcu = 1;
        d.mcux = (J.w + 7) / 8;
        d.mcuy = (J.h + 7) / 8;
    }
    d.nblocks = (int64_t)d.mcux * d.mcuy * d.nbmcu;
    for (int c = 0; c < 4; c++) d.pw[c] = d.ph[c] = d.cw[c] = d.ch[c] = 0;
    for (int c = 0; c < J.ncomp; c++) {
        const int hc = J.ncomp == 3 ? (c == 0 ? d.hs : 1) : 1, vc = J.ncomp == 3 ? (c == 0 ? d.vs : 1) : 1;
        d.cw[c] = (J.w * hc + d.hs - 1) / d.hs;  // downsampled_width
        d.ch[c] = (J.h * vc + d.vs - 1) / d.vs;
        d.pw[c] = (d.cw[c] + 7) / 8 * 8;
        d.ph[c] = (d.ch[c] + 7) / 8 * 8;
    }
    d.fancy = J.ncomp == 3 && d.hs == 2 && d.cw[1] > 2;  // do_fancy_upsampling && downsampled_width > 2
    d.rgb = J.ncomp == 3 && J.rgb;
    d.cmyk = J.ncomp == 4 ? J.cmyk : 0;
    d.wmcu = dec_walk_mcu(J.ncomp, d.nbmcu, J.td, J.ta);
    d.fuse420 = s == 1 && J.ncomp == 3 && d.hs == 2 && d.vs == 2 && d.fancy && !d.rgb;
    d.s = s;
    d.ow = (J.w + s - 1) / s;
    d.oh = (J.h + s - 1) / s;
}

uint32_t pick_sub_bits(uint64_t total_bits)
{
    if (const char* e = getenv("ICX_DEC_SUB_BITS")) {
        const long v = atol(e);
        if (v >= 64 && (v & (v - 1)) == 0) return (uint32_t)v;
    }
    // Long subsequences re-walk least and need fewer warm-ups (k_dec_init walks
    // `warm` bits per subsequence), short ones give the chip threads and keep
    // the relaxation's re-walk launches short.  Measured on 4K q95 (half noise,
    // e2e leg, ab_r4g_dec.txt / ab_r4h_dec_sub.txt / ab_r4i_dec_sub.txt):
    // 1000 frames per call (62 Gbit) 16384 / 32768 / 65536 / 131072 bits:
    // 96.6 / 93.5 / 90.3 / 96.0 ms; 200 frames (12.4 Gbit) 16384 / 32768 /
    // 65536: 22.4 / 22.8 / 23.9 ms.  With the two-step walks (round 4 end,
    // ab_r4zf_dec_win_sub.txt / ab_r4zg_dec_sub.txt) 200 frames: 16384 /
    // 32768 / 65536 = 20.7 / 20.2 / 21.9 ms.  65536 while at least 2^19 of
    // them remain, 32768 while 2^16 do (round 5: files -> files, two workers
    // on one GPU, 64-frame calls: 32768 instead of 16384 gave 4105 / 3571
    // files/s against 3880 / 3183, 65536 3075 / 2693 - one relaxation launch
    // fewer per call, profiles/r5/pipeline/ab_r5q_pipeline.txt); below that
    // 16384, and shorter only when the batch would not give the chip ~64k
    // threads.
    // Round 6 (profiles/r6/ab/ab_r6_sub_small.txt): a call under 2^32 bits
    // (~69 4K q95 frames: the files -> files path's 64-frame groups) takes
    // 16384 with a 24576-bit warm-up (warm_bits): 64 frames 7.80 -> 7.40 ms per
    // call; 200 frames keep 32768 (16384 there: +4 %).
    uint32_t S = 65536;
    if (total_bits / S < (1u << 19)) S = total_bits >= (1ull << 32) ? 32768 : 16384;
    while (S > 2048 && total_bits / S < 65536) S /= 2;
    return S;
}

// Warm-up walk before each subsequence (k_dec_init): long enough for typical
// content to resynchronise, short against the subsequence.  Measured on 200
// 4K q95 frames (half noise): 2048 bits 33.7-34.2 ms per call, 4096 33.2,
// 8192 32.7-32.9 (init +1.1 ms, sync -1.4 ms), 16384 34.0.  A small call
// (under 2^32 bits, 16384-bit subsequences: pick_sub_bits) leaves the chip
// part-idle in the warm-up launch, and a long warm-up there cuts the noise
// subsequences' misses (scripts/sync_stats.cpp: 8192 bits 33 %, 16384 11 %,
// 32768 1.5 %) and with them the relaxation's launches: 64 frames at 16384
// bits per subsequence, warm-up 16384 / 24576 bits: 7.52-7.60 / 7.39-7.41 ms
// per call (profiles/r6/ab/ab_r6_sub_small.txt, ab_r6_warm_small.txt).
uint32_t warm_bits(uint32_t sub_bits, uint64_t total_bits)
{
    if (const char* e = getenv("ICX_DEC_WARM")) return (uint32_t)atol(e);
    if (sub_bits == 16384 && total_bits < (1ull << 32)) return 24576;
    return std::min<uint32_t>(8192, sub_bits / 2);
}

// The header tables build_dec_tab reads are equal (so are the DecTabs).
bool same_tables(const JpegHeader& a, const JpegHeader& b)
{
    return a.ncomp == b.ncomp && !memcmp(a.td, b.td, sizeof(a.td)) && !memcmp(a.ta, b.ta, sizeof(a.ta)) &&
           !memcmp(a.tq, b.tq, sizeof(a.tq)) && !memcmp(a.qt, b.qt, sizeof(a.qt)) &&
           !memcmp(a.qt_ok, b.qt_ok, sizeof(a.qt_ok)) && !memcmp(a.hn, b.hn, sizeof(a.hn)) &&
           !memcmp(a.h_ok, b.h_ok, sizeof(a.h_ok)) && !memcmp(a.hbits, b.hbits, sizeof(a.hbits)) &&
           !memcmp(a.hvals, b.hvals, sizeof(a.hvals));
}

struct WPlan {
    Plan p;
    int64_t total;
};

WPlan plan_of(Uploader& U, const std::vector<int64_t>& counts, const int32_t* d_ids)
{
    std::vector<int64_t> pre(counts.size() + 1, 0);
    for (size_t i = 0; i < counts.size(); i++) pre[i + 1] = pre[i] + counts[i];
    WPlan out{};
    out.p.ids = d_ids;
    out.p.prefix = U.put(pre.data(), pre.size());
    out.p.m = (int32_t)counts.size();
    out.total = pre.back();
    // 2-D launch (no slot search at workgroup start: a binary search of the
    // prefix array is a chain of dependent loads, which short workgroups such
    // as a 4 KiB unstuff tile would mostly wait on) unless more than a third
    // of its workgroups would find nothing to do
    const int64_t maxc = counts.empty() ? 0 : *std::max_element(counts.begin(), counts.end());
    if (out.p.m > 1 && out.p.m <= 65535 && maxc > 0 && maxc < (1ll << 31) && maxc * out.p.m * 2 <= out.total * 3)
        out.p.width = (int32_t)maxc;
    return out;
}

// Host threads for the progressive entropy decode: the affinity set, at most
// 16 (ICX_HOST_THREADS overrides).
int host_threads()
{
    if (const char* e = getenv("ICX_HOST_THREADS")) return std::max(1, atoi(e));
    cpu_set_t set;
    int n = 1;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    return std::max(1, std::min(n, 16));
}

// Files whose entropy decode runs on host threads: progressive files (SOF2,
// icx_progressive.cpp: one sequential walk per scan), and sequential files
// the device's decode flagged (icx_seqdecode.cpp: IJG 6b's recovery from
// truncated scans, bad codes and restart markers out of sequence).  Each
// file's coefficients go straight into pinned staging, in the layout
// k_dec_write leaves for baseline files; one copy per file takes the
// coefficients and DC values to HBM, and the device's IDCT and colour passes
// (the same launches as the baseline tail) produce the pixels.
// Device-resident files are downloaded first.
icx_status run_host_entropy(icx_ctx* c, std::vector<DecItem>& items, int16_t* coef_out, size_t coef_cap)
{
    size_t pos = 0;
    while (pos < items.size()) {
        std::vector<DecItem*> sub;
        std::vector<DecDesc> desc;
        size_t need = 2 << 20, hneed = 2 << 20;
        while (pos < items.size()) {
            DecItem& it = items[pos];
            DecDesc d{};
            dec_geometry(it.J, it.s, d);
            const size_t nb = (size_t)d.nblocks;
            size_t per = align_up(nb * 128, 256) + align_up(nb * 4, 256) + 4096;
            for (int k = 0; k < 4; k++) per += align_up((size_t)d.pw[k] * d.ph[k] + DEC_PLANE_SPARE, 256);
            const bool host_out = !coef_out && !is_device_ptr(it.job->out);
            if (host_out) per += align_up(it.job->out_len, 256);
            const size_t hper = align_up(nb * 128, 64) + align_up(nb * 4, 64) + (it.dev_in ? align_up(it.job->len, 64) : 0);
            // pinned staging of coefficients: at most 2 GiB per sub-batch
            if (!sub.empty() && (need + per > c->budget || hneed + hper > std::min<size_t>(c->budget, 2ull << 30)))
                break;
            need += per;
            hneed += hper;
            it.host_out = host_out;
            sub.push_back(&it);
            desc.push_back(d);
            pos++;
        }
        const int m = (int)sub.size();
        // (three plans below: Wb, Wr, Wp)
        const size_t up = Uploader::need<DecTab>(m) + Uploader::need<DecDesc>(m) + Uploader::need<DecState>(m) +
                          Uploader::need<int32_t>(m) + 3 * Uploader::need<int64_t>(m + 1) + 4096;
        hipError_t e = c->dev.reserve(need + up);
        if (e == hipSuccess) e = c->host.reserve(hneed + up);
        if (e != hipSuccess) return hip_fail(c, e, "progressive decode workspace");
        c->dev.used = c->host.used = 0;
        Uploader U(c, up);
        std::vector<int16_t*> hco(m);
        std::vector<int32_t*> hdc(m);
        std::vector<const uint8_t*> file(m);
        for (int k = 0; k < m; k++) {
            const size_t nb = (size_t)desc[k].nblocks;
            hco[k] = (int16_t*)c->host.take(nb * 128);
            hdc[k] = (int32_t*)c->host.take(nb * 4);
            file[k] = sub[k]->job->data;
            if (sub[k]->dev_in) {
                uint8_t* h = (uint8_t*)c->host.take(sub[k]->job->len);
                if (!h) return fail(c, ICX_E_NOMEM, "pinned staging exhausted");
                e = hipMemcpyAsync(h, file[k], sub[k]->job->len, hipMemcpyDeviceToHost, c->stream);
                if (e != hipSuccess) return hip_fail(c, e, "progressive file download");
                file[k] = h;
            }
            if (!hco[k] || !hdc[k]) return fail(c, ICX_E_NOMEM, "pinned staging exhausted");
        }
        // the previous sub-batch's (and the dev-in files') copies from this staging have finished
        e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "progressive staging");
        DecTab* h_tab;
        DecTab* d_tab = U.alloc<DecTab>(m, &h_tab);
        if (U.overflow) return fail(c, ICX_E_NOMEM, "upload staging exhausted");
        std::vector<icx_status> st(m, ICX_OK);
        {
            HostSpan hs{c, sub[0]->J.progressive ? "host.dec_progressive" : "host.dec_recovery"};
            std::atomic<int> next{0};
            auto work = [&]() {
                for (int k; (k = next++) < m;) {
                    const JpegHeader& J = sub[k]->J;
                    h_tab[k] = DecTab{};
                    if (J.progressive) {
                        memset(hco[k], 0, (size_t)desc[k].nblocks * 128);
                        st[k] = prog_decode(file[k], sub[k]->job->len, J, hco[k], hdc[k], h_tab[k].qt);
                    } else {
                        for (int q = 0; q < J.ncomp; q++) memcpy(h_tab[k].qt[q], J.qt[J.tq[q]], sizeof(h_tab[k].qt[q]));
                        st[k] = seq_decode(file[k], sub[k]->job->len, J, hco[k], hdc[k]);
                    }
                }
            };
            const int nt = std::min(m, host_threads());
            std::vector<std::thread> pool;
            for (int t = 1; t < nt; t++) pool.emplace_back(work);
            work();
            for (auto& t : pool) t.join();
        }
        std::vector<DecState> states(m);
        std::vector<int32_t> ids;
        std::vector<int64_t> cnt_blk, cnt_px, cnt_rows;
        int64_t tpx = 0;
        for (int k = 0; k < m; k++) {
            icx_decode_job& j = *sub[k]->job;
            DecDesc& d = desc[k];
            if (st[k] != ICX_OK) {
                j.status = st[k];
                states[k].status = 6;
                continue;
            }
            if (coef_out) {
                const size_t nb = (size_t)d.nblocks;
                if (nb * 64 > coef_cap) j.status = ICX_E_BUFFER;
                else memcpy(coef_out, hco[k], nb * 128);
                continue;
            }
            d.coefs = (int16_t*)c->dev.take((size_t)d.nblocks * 128);
            d.dc = (int32_t*)c->dev.take((size_t)d.nblocks * 4);
            e = hipMemcpyAsync(d.coefs, hco[k], (size_t)d.nblocks * 128, hipMemcpyHostToDevice, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(d.dc, hdc[k], (size_t)d.nblocks * 4, hipMemcpyHostToDevice, c->stream);
            if (e != hipSuccess) return hip_fail(c, e, "coefficient upload");
            for (int q = d.fuse420 ? 1 : 0; q < d.ncomp; q++)
                d.plane[q] = (uint8_t*)c->dev.take((size_t)d.pw[q] * d.ph[q] + DEC_PLANE_SPARE);
            d.out = sub[k]->host_out ? (uint8_t*)c->dev.take(j.out_len) : j.out;
            d.ostride = d.ow * sub[k]->nch;
            d.tab = d_tab + k;
            const int64_t nmcu = (int64_t)d.mcux * d.mcuy;
            ids.push_back(k);
            cnt_blk.push_back(dec_idct_items(d.fuse420 ? (2 * nmcu + 31) / 32 : (d.nblocks + 31) / 32));
            cnt_px.push_back(d.fuse420 ? 0 : ((int64_t)d.oh * ((d.ow + 3) / 4) + 255) / 256);
            cnt_rows.push_back(d.fuse420 ? (int64_t)dec_lc_items(d.mcux, d.mcuy) : 0);
            tpx += (int64_t)d.w * d.h;
        }
        if (coef_out || ids.empty()) continue;
        const DecDesc* d_desc = U.put(desc.data(), m);
        const DecState* d_state = U.put(states.data(), m);
        const int32_t* d_ids = U.put(ids.data(), ids.size());
        const WPlan Wb = plan_of(U, cnt_blk, d_ids), Wr = plan_of(U, cnt_rows, d_ids), Wp = plan_of(U, cnt_px, d_ids);
        if (icx_status s = U.flush()) return s;
        {
            Timed tm(c, "dec_idct", tpx);
            launch_dec_idct(d_desc, d_state, Wb.p, Wb.total, c->stream);
        }
        {
            Timed tm(c, "dec_color", tpx);
            launch_dec_luma_color_420(d_desc, d_state, Wr.p, Wr.total, c->stream);
            launch_dec_color(d_desc, d_state, Wp.p, Wp.total, c->stream);
        }
        for (int k : ids)
            if (sub[k]->host_out) {
                e = hipMemcpyAsync(sub[k]->job->out, desc[k].out, sub[k]->job->out_len, hipMemcpyDeviceToHost,
                                   c->stream);
                if (e != hipSuccess) return hip_fail(c, e, "output download");
            }
        e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(c, e, "progressive decode");
        resolve_profile(c);
    }
    return ICX_OK;
}

// mode 0: decode to pixels; mode 1: coefficients only (debug: natural order, DC in [0]).
// raw4: 4-component files out as libjpeg's CMYK samples (4 bytes a pixel, debug)
icx_status run_decode_impl(icx_ctx* c, icx_decode_job* jobs, int n, int16_t* coef_out, size_t coef_cap,
                           bool raw4);

// Every decode call returns with its device work finished, on the error paths
// too ("entropy decode did not settle", a failed launch or copy mid-tail):
// the aux streams' tails may still read scan and plane buffers that the caller
// frees after an error, and a recycled buffer can be rewritten at once by an
// upload on another copy stream (pool_free's invariant).
icx_status run_decode(icx_ctx* c, icx_decode_job* jobs, int n, int16_t* coef_out, size_t coef_cap,
                      bool raw4 = false)
{
    const icx_status s = run_decode_impl(c, jobs, n, coef_out, coef_cap, raw4);
    if (s != ICX_OK) {
        std::lock_guard<std::recursive_mutex> lk(c->mu);
        (void)hipStreamSynchronize(c->stream);
        for (int k = 0; k < c->n_dec_aux; k++) (void)hipStreamSynchronize(c->dec_aux[k]);
        (void)hipGetLastError();
    }
    return s;
}

icx_status run_decode_impl(icx_ctx* c, icx_decode_job* jobs, int n, int16_t* coef_out, size_t coef_cap,
                           bool raw4)
{
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    HostSpan call{c, "host.call_decode"};  // the whole call, wall time (profiling)
    hipError_t he = hipSetDevice(c->device);
    if (he != hipSuccess) return hip_fail(c, he, "hipSetDevice");
    std::vector<DecItem> items, prog;
    items.reserve(n);
    std::vector<char> dev_in(n, 0);
    for (int i = 0; i < n; i++) dev_in[i] = jobs[i].data && is_device_ptr(jobs[i].data);
    std::vector<JpegHeader> hdr(n);
    std::vector<icx_status> hst(n, ICX_OK);
    {
        HostSpan hs{c, "host.dec_headers"};
        if (icx_status s = fetch_headers(c, jobs, n, dev_in, hdr, hst)) return s;
    }
    for (int i = 0; i < n; i++) {
        icx_decode_job& j = jobs[i];
        j.width = j.height = j.src_width = j.src_height = 0;
        j.fmt = ICX_BGR24;
        j.out_len = 0;
        if (!j.data) {
            j.status = ICX_E_NULL;
            continue;
        }
        DecItem it;
        it.job = &j;
        it.dev_in = dev_in[i];
        if (it.dev_in) {
            it.J = hdr[i];
            j.status = hst[i];
        } else {
            j.status = parse_jpeg(j.data, j.len, j.len, it.J);
        }
        j.src_width = it.J.w;
        j.src_height = it.J.h;
        if (j.status != ICX_OK) continue;
        const int s = j.subsampling > 0 ? j.subsampling : icx_subsampling_factor(it.J.w, it.J.h);
        it.s = s;
        it.nch = it.J.ncomp == 1 ? 1 : it.J.ncomp == 4 && raw4 ? 4 : 3;  // CMYK / YCCK: BGR24 (k_dec_color)
        j.fmt = it.nch == 1 ? ICX_GRAY8 : ICX_BGR24;
        j.width = (it.J.w + s - 1) / s;
        j.height = (it.J.h + s - 1) / s;
        j.out_len = (size_t)j.width * j.height * it.nch;
        if (!coef_out && !j.out) {
            j.status = ICX_E_NULL;
            continue;
        }
        if (!coef_out && j.cap < j.out_len) {
            j.status = ICX_E_BUFFER;
            continue;
        }
        (it.J.progressive ? prog : items).push_back(it);
    }
    if (!prog.empty())
        if (icx_status s = run_host_entropy(c, prog, coef_out, coef_cap)) return s;
    std::vector<DecItem> recover;  // flagged by the device decode: icx_seqdecode.cpp
    size_t pos = 0;
    while (pos < items.size()) {
        // ---- size a sub-batch against the workspace budget
        std::vector<DecItem*> sub;
        std::vector<DecDesc> desc;
        size_t need = 2 << 20;
        uint64_t bits = 0;
        while (pos < items.size()) {
            DecItem& it = items[pos];
            DecDesc d{};
            dec_geometry(it.J, it.s, d);
            d.raw4 = raw4;
            const int64_t scan_len = (int64_t)(it.job->len - it.J.scan_off);
            const int64_t nmcu = (int64_t)d.mcux * d.mcuy;
            d.nseg_max = it.J.ri ? (int32_t)((nmcu + it.J.ri - 1) / it.J.ri) + 1 : 1;
            it.ent_cap = (size_t)scan_len + (size_t)(DEC_PAD - 2) * d.nseg_max + DEC_TAIL + 64 + 4 * DEC_WIN_MAX;
            it.ntiles = (scan_len + DEC_TILE - 1) / DEC_TILE;
            it.nblocks = d.nblocks;
            size_t per = (it.dev_in ? 0 : align_up(scan_len, 256)) + align_up(it.ent_cap, 256) + it.ntiles * 8 + 512 +
                         (size_t)d.nseg_max * 4 + (size_t)d.nblocks * (128 + 4) + sizeof(DecTab) + 4096;
            for (int k = 0; k < 4; k++) per += align_up((size_t)d.pw[k] * d.ph[k] + DEC_PLANE_SPARE, 256);
            per += (size_t)(it.ent_cap * 8 / 2048 + 2) * (8 + 2 + 4 + 4);  // subsequence arrays at S >= 2048
            per += (size_t)(it.ent_cap * 8 / 2048 + 2) * DEC_CK_MAX * 8;  // checkpoints
            if (!coef_out && !is_device_ptr(it.job->out)) per += align_up(it.job->out_len, 256);
            if (!sub.empty() && need + per > c->budget) break;
            need += per;
            bits += (uint64_t)scan_len * 8;
            sub.push_back(&it);
            desc.push_back(d);
            pos++;
        }
        const int m = (int)sub.size();
        const uint32_t S = pick_sub_bits(bits);
        // every small argument array of the sub-batch travels in one packed upload
        // (three whole-sub-batch plans below: Pt, Pc, Ps)
        const size_t up = Uploader::need<DecTab>(m) + Uploader::need<DecDesc>(m) + Uploader::need<DecState>(m) +
                          Uploader::need<int32_t>(m) + 3 * Uploader::need<int64_t>(m + 1) +
                          // the decode tails (subsets settled at one check): ids and 4 plans each; each
                          // image is in one tail, so at most m + 1 tails of 36 B per image + alignment
                          36 * (size_t)m + (size_t)(m + 1) * (64 + 4 * 72);
        hipError_t e = c->dev.reserve(need + up + (size_t)m * 64 * 1024 + (16 << 20));
        if (e != hipSuccess) {
            for (DecItem* it : sub) it->job->status = ICX_E_NOMEM;
            (void)hipGetLastError();
            c->err = "device workspace allocation failed";
            continue;
        }
        c->dev.used = 0;
        c->dev.overflow = false;
        size_t host_need = (64 << 20) + up;
        for (DecItem* it : sub)
            if (!it->dev_in && !is_pinned_ptr(it->job->data)) host_need += align_up(it->job->len, 64);
        e = c->host.reserve(host_need);
        if (e != hipSuccess) return hip_fail(c, e, "hipHostMalloc");
        c->host.used = 0;
        Uploader U(c, up);

        // Decode tables once per distinct header tables (a batch of files from
        // one encoder shares them): images point at their table set.
        std::vector<int> tab_of(m);
        std::vector<int> uniq;  // first image of each distinct set
        for (int k = 0; k < m; k++) {
            int u = -1;
            for (int q = (int)uniq.size() - 1; q >= 0 && q >= (int)uniq.size() - 4; q--)
                if (same_tables(sub[k]->J, sub[uniq[q]]->J)) {
                    u = q;
                    break;
                }
            if (u < 0) {
                u = (int)uniq.size();
                uniq.push_back(k);
            }
            tab_of[k] = u;
        }
        DecTab* h_tab;
        DecTab* d_tab = U.alloc<DecTab>(uniq.size(), &h_tab);
        if (U.overflow) return fail(c, ICX_E_NOMEM, "upload staging exhausted");
        std::vector<DecState> states(m);
        std::vector<char> tab_ok(uniq.size(), 0);
        int64_t max_nsub = 0;
        for (int k = 0; k < m; k++) {
            HostSpan hs_tab{c, "host.dec_setup"};
            DecItem& it = *sub[k];
            DecDesc& d = desc[k];
            if (uniq[tab_of[k]] == k) {
                h_tab[tab_of[k]] = DecTab{};
                tab_ok[tab_of[k]] = build_dec_tab(it.J, h_tab[tab_of[k]]);
            }
            if (!tab_ok[tab_of[k]]) {
                it.job->status = ICX_E_CORRUPT;
                states[k].status = 6;
            }
            const int64_t scan_len = (int64_t)(it.job->len - it.J.scan_off);
            d.scan_len = scan_len;
            d.ntiles = (int32_t)it.ntiles;
            // k_unstuff_* read the stuffed scan at any alignment and never past
            // scan_len's 16-B chunk: a device file is read where it lies, a host
            // file takes one DMA (pageable: via pinned staging)
            const uint8_t* src = it.job->data + it.J.scan_off;
            if (!it.dev_in) {
                uint8_t* scan = (uint8_t*)c->dev.take(align_up(scan_len, 256));
                if (!is_pinned_ptr(it.job->data)) {
                    uint8_t* h = (uint8_t*)c->host.take(scan_len);
                    if (h) {
                        memcpy(h, src, scan_len);
                        src = h;
                    }
                }
                e = hipMemcpyAsync(scan, src, scan_len, hipMemcpyHostToDevice, c->stream);
                if (e != hipSuccess) return hip_fail(c, e, "scan upload");
                src = scan;
            }
            d.scan = src;
            d.ent = (uint8_t*)c->dev.take(align_up(it.ent_cap, 256));
            d.ent_cap = (int64_t)it.ent_cap;
            d.tile_cnt = (uint32_t*)c->dev.take(it.ntiles * 4 + 4);
            d.tile_rst = (uint32_t*)c->dev.take(it.ntiles * 4 + 4);
            d.seg = (uint32_t*)c->dev.take((size_t)d.nseg_max * 4);
            d.nsub_max = (int32_t)((it.ent_cap * 8 + S - 1) / S);
            max_nsub = std::max<int64_t>(max_nsub, d.nsub_max);
            d.est = (uint64_t*)c->dev.take((size_t)(d.nsub_max + 1) * 8);
            d.ck = (uint64_t*)c->dev.take((size_t)(d.nsub_max + 1) * DEC_CK_MAX * 8);
            d.wl[0] = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.wl[1] = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.ncnt = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.boff = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            // d.dc right behind the coefficients: k_dec_write stores a block's
            // coefficients and its DC difference with one instruction
            d.coefs = (int16_t*)c->dev.take((size_t)d.nblocks * 132);
            d.dc = (int32_t*)((uint8_t*)d.coefs + (size_t)d.nblocks * 128);
            if (!coef_out) {
                for (int q = d.fuse420 ? 1 : 0; q < d.ncomp; q++)  // fuse420: luma stays in LDS
                    d.plane[q] = (uint8_t*)c->dev.take((size_t)d.pw[q] * d.ph[q] + DEC_PLANE_SPARE);
                it.host_out = !is_device_ptr(it.job->out);
                d.out = it.host_out ? (uint8_t*)c->dev.take(it.job->out_len) : it.job->out;
                d.ostride = d.ow * it.nch;
            }
            d.tab = d_tab + tab_of[k];
            states[k].end = scan_len;  // coefficients need no clearing: the write pass stores whole blocks
        }
        const int max_it = (int)max_nsub + 8;  // each launch settles at least one more subsequence
        uint32_t* d_changed = (uint32_t*)c->dev.take((size_t)max_it * 4);
        uint32_t* d_wlcnt = (uint32_t*)c->dev.take((size_t)m * max_it * 4);
        for (int k = 0; k < m; k++) desc[k].wl_cnt = d_wlcnt;
        if (c->dev.overflow) return fail(c, ICX_E_NOMEM, "device workspace overrun (workspace sizing)");
        uint32_t* h_changed = (uint32_t*)c->host.take(4);
        std::vector<int32_t> ids(m);
        for (int k = 0; k < m; k++) ids[k] = k;
        const DecDesc* d_desc = U.put(desc.data(), m);
        DecState* d_state = U.put(states.data(), m);
        const int32_t* d_ids = U.put(ids.data(), m);

        std::vector<int64_t> cnt_tiles(m), cnt_ctiles(m), cnt_subs(m), cnt_pieces(m), cnt_blk(m), cnt_px(m), cnt_rows(m);
        int64_t stuffed = 0;
        for (int k = 0; k < m; k++) {
            cnt_tiles[k] = (sub[k]->ntiles + DEC_SCATTER_TILES - 1) / DEC_SCATTER_TILES;  // k_unstuff_scatter
            cnt_ctiles[k] = (sub[k]->ntiles + DEC_UNSTUFF_TILES - 1) / DEC_UNSTUFF_TILES;  // k_unstuff_count
            cnt_subs[k] = (desc[k].nsub_max + 1 + DEC_SYNC_NT - 1) / DEC_SYNC_NT;
            cnt_pieces[k] = ((int64_t)(desc[k].nsub_max + 1) * dec_pieces(S) + DEC_WRITE_NT - 1) / DEC_WRITE_NT;  // k_dec_write
            // colour: luma IDCT fused with upsampling + conversion for s == 1 4:2:0 fancy (chroma
            // blocks alone go through k_dec_idct), the per-pixel gather kernel otherwise
            const DecDesc& q = desc[k];
            const int64_t nmcu = (int64_t)q.mcux * q.mcuy;
            cnt_blk[k] = dec_idct_items(q.fuse420 ? (2 * nmcu + 31) / 32 : (q.nblocks + 31) / 32);
            cnt_px[k] = q.fuse420 ? 0 : ((int64_t)q.oh * ((q.ow + 3) / 4) + 255) / 256;
            cnt_rows[k] = q.fuse420 ? (int64_t)dec_lc_items(q.mcux, q.mcuy) : 0;
            stuffed += desc[k].scan_len;
        }
        // plans of the whole sub-batch; the pixel stages get theirs per tail
        const WPlan Pt = plan_of(U, cnt_tiles, d_ids), Pc = plan_of(U, cnt_ctiles, d_ids),
                    Ps = plan_of(U, cnt_subs, d_ids);
        icx_status st = U.flush();
        if (st) return st;
        e = hipMemsetAsync(d_changed, 0, (size_t)max_it * 4, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(d_wlcnt, 0, (size_t)m * max_it * 4, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "counter clear");
        {
            Timed tm(c, "dec_unstuff", stuffed);
            launch_unstuff(d_desc, d_state, Pc.p, Pc.total, Pt.p, Pt.total, d_ids, m, S, c->stream);
        }
        if (getenv("ICX_DEC_DEBUG_UNSTUFF")) {  // development check: the device stream against the host rule
            (void)hipStreamSynchronize(c->stream);
            std::vector<DecState> hs(m);
            (void)hipMemcpy(hs.data(), d_state, sizeof(DecState) * m, hipMemcpyDeviceToHost);
            for (int k = 0; k < std::min(m, 3); k++) {
                const DecDesc& dd = desc[k];
                std::vector<uint8_t> sc(dd.scan_len), en(hs[k].ent_len);
                (void)hipMemcpy(sc.data(), dd.scan, dd.scan_len, hipMemcpyDefault);
                (void)hipMemcpy(en.data(), dd.ent, en.size(), hipMemcpyDeviceToHost);
                std::vector<uint8_t> ref;
                int64_t end = dd.scan_len;
                for (int64_t i = 0; i + 1 < dd.scan_len; i++)
                    if (sc[i] == 0xFF && sc[i + 1] != 0x00 && sc[i + 1] != 0xFF && !(sc[i + 1] >= 0xD0 && sc[i + 1] <= 0xD7)) {
                        end = i;
                        break;
                    }
                int nr = 0;
                for (int64_t i = 0; i < end; i++) {
                    int rst;
                    const int kk = dec_unstuff_rule(i ? sc[i - 1] : 0, sc[i], i + 1 < dd.scan_len ? sc[i + 1] : 0, &rst);
                    if (rst) {
                        for (int p = 0; p < DEC_PAD; p++) ref.push_back(0xFF);
                        nr++;
                    } else if (kk) {
                        ref.push_back(sc[i]);
                    }
                }
                size_t mis = 0;
                while (mis < std::min(ref.size(), en.size()) && ref[mis] == en[mis]) mis++;
                fprintf(stderr, "[unstuff %d] scan %lld ntiles %d ent_len %u ref %zu nseg %u ref_rst %d nsub %u status %d first_mismatch %zu\n",
                        k, (long long)dd.scan_len, dd.ntiles, hs[k].ent_len, ref.size(), hs[k].nseg, nr, hs[k].nsub,
                        hs[k].status, mis);
            }
        }
        {
            Timed tm(c, "dec_init", stuffed);
            launch_dec_init(d_desc, d_state, Ps.p, Ps.total, S, warm_bits(S, bits), c->stream);
        }
        // ---- settle the subsequence entry states.  An image whose last sync
        // launch appended nothing to its worklist has settled (its worklists
        // stay empty); at each check the images that settled since the last one
        // run the rest of their decode on the aux stream while the others keep
        // relaxing here.  The relaxation's later launches re-walk the few long
        // chains of unsynchronised subsequences one link per launch and leave
        // most of the chip idle, so the settled images' write, DC, IDCT and
        // colour passes fill it.
        auto tail = [&](const std::vector<int>& ks, hipStream_t s, hipEvent_t wait_ev = nullptr,
                        hipEvent_t write_done = nullptr) -> icx_status {
            std::vector<int32_t> sid(ks.begin(), ks.end());
            std::vector<int64_t> a, b, r, q;
            int64_t stf = 0, tpx = 0;
            for (int k : ks) {
                a.push_back(cnt_pieces[k]);
                b.push_back(cnt_blk[k]);
                r.push_back(cnt_rows[k]);
                q.push_back(cnt_px[k]);
                stf += desc[k].scan_len;
                tpx += (int64_t)desc[k].w * desc[k].h;
            }
            const int n = (int)ks.size();
            const int32_t* d_sid = U.put(sid.data(), sid.size());
            const WPlan Ws = plan_of(U, a, d_sid), Wb = plan_of(U, b, d_sid), Wr = plan_of(U, r, d_sid),
                        Wp = plan_of(U, q, d_sid);
            if (icx_status st = U.flush()) return st;  // on c->stream, behind the launches that settled them
            if (s != c->stream) {
                hipError_t he2 = hipEventRecord(c->ev_dec_split, c->stream);
                if (he2 == hipSuccess) he2 = hipStreamWaitEvent(s, c->ev_dec_split, 0);
                if (he2 != hipSuccess) return hip_fail(c, he2, "decode stream split");
            }
            if (wait_ev) {  // the previous part's write pass (split tails, below)
                hipError_t he2 = hipStreamWaitEvent(s, wait_ev, 0);
                if (he2 != hipSuccess) return hip_fail(c, he2, "decode tail order");
            }
            launch_dec_offsets(d_desc, d_state, d_sid, n, s);
            {
                Timed tm(c, "dec_write", stf, false, s);
                launch_dec_write(d_desc, d_state, Ws.p, Ws.total, S, s);
            }
            if (write_done) {
                hipError_t he2 = hipEventRecord(write_done, s);
                if (he2 != hipSuccess) return hip_fail(c, he2, "decode tail order");
            }
            {
                Timed tm(c, "dec_dc", n, false, s);
                launch_dec_dc(d_desc, d_state, d_sid, n, s);
            }
            if (!coef_out) {
                {
                    Timed tm(c, "dec_idct", tpx, false, s);
                    launch_dec_idct(d_desc, d_state, Wb.p, Wb.total, s);
                }
                {
                    Timed tm(c, "dec_color", tpx, false, s);
                    launch_dec_luma_color_420(d_desc, d_state, Wr.p, Wr.total, s);
                    launch_dec_color(d_desc, d_state, Wp.p, Wp.total, s);
                }
            }
            return ICX_OK;
        };
        // tails of different checks go to different aux streams, so a check's
        // images need not wait behind the previous check's tail
        // A large tail (most of a big call's images settle at the first check)
        // goes in TAIL_SPLIT parts on as many aux streams, part p's write pass
        // after part p-1's: the latency-bound entropy write of one part runs
        // beside the bandwidth-bound pixel passes (DC, IDCT, colour) of the
        // part before it instead of after them.
        static const int TAIL_SPLIT = std::min(icx_ctx::DEC_AUX_MAX,
                                               std::max(1, getenv("ICX_DEC_TAIL_SPLIT") ? atoi(getenv("ICX_DEC_TAIL_SPLIT")) : 1));
        static const int NAUX = std::max(TAIL_SPLIT, std::min(icx_ctx::DEC_AUX_MAX,
                                         std::max(1, getenv("ICX_DEC_AUX") ? atoi(getenv("ICX_DEC_AUX")) : 1)));
        if (!c->ev_dec_split) {
            hipError_t he2 = hipEventCreateWithFlags(&c->ev_dec_split, hipEventDisableTiming);
            if (he2 != hipSuccess) return hip_fail(c, he2, "decode aux stream");
        }
        while (c->n_dec_aux < NAUX) {
            hipError_t he2 = hipStreamCreateWithFlags(&c->dec_aux[c->n_dec_aux], hipStreamNonBlocking);
            if (he2 == hipSuccess) he2 = hipEventCreateWithFlags(&c->ev_dec_aux[c->n_dec_aux], hipEventDisableTiming);
            if (he2 == hipSuccess) he2 = hipEventCreateWithFlags(&c->ev_dec_wr[c->n_dec_aux], hipEventDisableTiming);
            if (he2 != hipSuccess) return hip_fail(c, he2, "decode aux stream");
            c->n_dec_aux++;
        }
        uint32_t* h_wl = (uint32_t*)c->host.take((size_t)m * 4);
        if (!h_wl) return fail(c, ICX_E_NOMEM, "pinned staging exhausted");
        std::vector<char> tailed(m, 0);
        int aux_used = 0, aux_next = 0;  // aux streams used by this call (the first aux_used)
        int it = 0;
        static const char* const sync_names[] = {"dec_sync", "dec_sync_r1", "dec_sync_r2", "dec_sync_r3",
                                                 "dec_sync_r4", "dec_sync_r5", "dec_sync_r6", "dec_sync_r7+"};
        static const int SYNC_PER_CHECK = std::max(1, getenv("ICX_DEC_CHECK") ? atoi(getenv("ICX_DEC_CHECK")) : 2);
        for (;;) {
            for (int k = 0; k < SYNC_PER_CHECK && it < max_it; k++, it++) {
                Timed tm(c, sync_names[std::min(it, 7)], 0);
                launch_dec_sync(d_desc, d_state, Ps.p, Ps.total, S, it, m, d_changed + it, c->stream);
            }
            e = hipMemcpyAsync(h_changed, d_changed + it - 1, 4, hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(h_wl, d_wlcnt + (size_t)(it - 1) * m, (size_t)m * 4, hipMemcpyDeviceToHost,
                                   c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess) return hip_fail(c, e, "sync counter");
            if (*h_changed == 0) break;
            if (it >= max_it) return fail(c, ICX_E_DEVICE, "entropy decode did not settle");
            std::vector<int> early;
            for (int k = 0; k < m; k++)
                if (!tailed[k] && h_wl[k] == 0) early.push_back(k);
            if (!early.empty()) {
                for (int k : early) tailed[k] = 1;
                const int parts = (int)early.size() >= 32 * TAIL_SPLIT ? TAIL_SPLIT : 1;
                for (int q = 0; q < parts; q++) {
                    const size_t a = early.size() * q / parts, b = early.size() * (q + 1) / parts;
                    const std::vector<int> part(early.begin() + a, early.begin() + b);
                    const int sx = aux_next % NAUX, sp = (aux_next + NAUX - 1) % NAUX;
                    if (icx_status st = tail(part, c->dec_aux[sx], q ? c->ev_dec_wr[sp] : nullptr,
                                             parts > 1 ? c->ev_dec_wr[sx] : nullptr))
                        return st;
                    aux_next++;
                }
                aux_used = std::min(aux_next, NAUX);
            }
        }
        c->stats["dec_sync_iters"].launches += it;
        if (c->prof) {  // profiling: subsequences re-walked by each later launch (worklist sizes)
            std::vector<uint32_t> wl((size_t)m * it);
            e = hipMemcpy(wl.data(), d_wlcnt, wl.size() * 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) return hip_fail(c, e, "worklist counters");
            int64_t subs = 0;
            for (int k = 0; k < m; k++) subs += desc[k].nsub_max;
            c->stats["dec_sync_walks"].units += subs;
            for (size_t i = 0; i < (size_t)m * (it - 1); i++) c->stats["dec_sync_walks"].units += wl[i];  // launches 1..it-1
        }
        std::vector<int> rest;
        for (int k = 0; k < m; k++)
            if (!tailed[k]) rest.push_back(k);
        if (!rest.empty())
            if (icx_status st = tail(rest, c->stream)) return st;
        for (int k = 0; k < aux_used; k++) {  // the final download waits for the aux streams' images too
            e = hipEventRecord(c->ev_dec_aux[k], c->dec_aux[k]);
            if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_dec_aux[k], 0);
            if (e != hipSuccess) return hip_fail(c, e, "decode stream join");
        }
        DecState* h_state = (DecState*)c->host.take(sizeof(DecState) * m);
        if (!h_state) return fail(c, ICX_E_NOMEM, "pinned staging exhausted");
        e = hipMemcpyAsync(h_state, d_state, sizeof(DecState) * m, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "decode");
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(c, e, "decode launch");
        for (int k = 0; k < m; k++) {
            icx_decode_job& j = *sub[k]->job;
            if (j.status != ICX_OK) continue;
            if (h_state[k].status) {  // not the clean case: IJG 6b's recovery on a host thread
                recover.push_back(*sub[k]);
                continue;
            }
            if (coef_out) {
                const size_t nb = (size_t)desc[k].nblocks;
                if (nb * 64 > coef_cap) {
                    j.status = ICX_E_BUFFER;
                    continue;
                }
                std::vector<int32_t> dc(nb);
                if ((e = hipMemcpy(coef_out, desc[k].coefs, nb * 128, hipMemcpyDeviceToHost)) != hipSuccess ||
                    (e = hipMemcpy(dc.data(), desc[k].dc, nb * 4, hipMemcpyDeviceToHost)) != hipSuccess)
                    return hip_fail(c, e, "coefficient download");
                for (size_t b = 0; b < nb; b++) coef_out[b * 64] = (int16_t)dc[b];
                continue;
            }
            if (sub[k]->host_out) {
                e = hipMemcpyAsync(j.out, desc[k].out, j.out_len, hipMemcpyDeviceToHost, c->stream);
                if (e != hipSuccess) return hip_fail(c, e, "output download");
            }
        }
        e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "output download");
        resolve_profile(c);
    }
    if (!recover.empty()) {
        c->stats["dec_recovered"].units += (int64_t)recover.size();
        if (icx_status s = run_host_entropy(c, recover, coef_out, coef_cap)) return s;
    }
    return ICX_OK;
}

}  // namespace

extern "C" {

icx_status icx_jpeg_info(const uint8_t* data, size_t len, int32_t* width, int32_t* height, int32_t* ncomp)
{
    if (!data) return ICX_E_NULL;
    JpegHeader J;
    const icx_status s = parse_jpeg(data, len, len, J);
    if (width) *width = J.w;
    if (height) *height = J.h;
    if (ncomp) *ncomp = J.ncomp;
    return s;
}

icx_status icx_decode_jpg_batch(icx_ctx* ctx, icx_decode_job* jobs, int32_t n)
{
    if (!ctx || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    return run_decode(ctx, jobs, n, nullptr, 0);
}

icx_status icx_decode_jpg(icx_ctx* ctx, icx_decode_job* job)
{
    if (!ctx || !job) return ICX_E_NULL;
    const icx_status s = run_decode(ctx, job, 1, nullptr, 0);
    return s != ICX_OK ? s : job->status;
}

namespace {
icx_status pool_alloc(icx_ctx* ctx, DevPool& P, size_t bytes, void** ptr)
{
    if (!ctx || !ptr) return ICX_E_NULL;
    *ptr = nullptr;
    const size_t c = DevPool::cls(bytes);
    {
        std::lock_guard<std::mutex> lk(ctx->pool_mu);
        auto f = P.free_.find(c);
        if (f != P.free_.end() && !f->second.empty()) {
            *ptr = f->second.back();
            f->second.pop_back();
            P.cached -= c;
            P.live_[*ptr] = c;
            return ICX_OK;
        }
    }
    // a new buffer (or slab): allocated outside every lock (a pinned
    // allocation takes milliseconds; other threads keep taking cached buffers)
    bool slab = P.slabbed(c);
    size_t bytes_new = slab ? P.slab_bytes(c) : c;
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = P.host ? hipHostMalloc(ptr, bytes_new, hipHostMallocPortable) : hipMalloc(ptr, bytes_new);
    if (e != hipSuccess && slab) {
        // no room for a whole slab (16x the class on the device): the class
        // size alone may still fit - a tight device must not fail an
        // allocation a plain hipMalloc would serve
        (void)hipGetLastError();
        slab = false;
        bytes_new = c;
        e = P.host ? hipHostMalloc(ptr, bytes_new, hipHostMallocPortable) : hipMalloc(ptr, bytes_new);
    }
    if (e != hipSuccess) {
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);  // (no pool lock held: no lock-order inversion)
        return hip_fail(ctx, e, P.host ? "hipHostMalloc" : "hipMalloc");
    }
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    if (slab) {  // the first piece is this call's, the rest go to the free list
        P.slabs.push_back(*ptr);
        for (size_t o = 0; o < bytes_new; o += c) {
            void* p = (char*)*ptr + o;
            P.carved.insert(p);
            if (o) {
                P.free_[c].push_back(p);
                P.cached += c;
            }
        }
    }
    P.live_[*ptr] = c;
    return ICX_OK;
}

icx_status pool_free(icx_ctx* ctx, DevPool& P, void* ptr)
{
    if (!ctx) return ICX_E_NULL;
    if (!ptr) return ICX_OK;
    size_t c = 0;
    {
        std::lock_guard<std::mutex> lk(ctx->pool_mu);
        auto l = P.live_.find(ptr);
        if (l != P.live_.end()) {
            c = l->second;
            P.live_.erase(l);
            // Recycling needs no synchronisation because every call that uses a
            // pool buffer has finished its device work when it returns, on every
            // path (run_decode synchronises its streams after an error too): the
            // buffer's next use - a launch on this context's stream, or an
            // icx_upload / icx_stage_files copy on one of its copy streams - can
            // only come after that.  (Host buffers: likewise.)
            if (P.cached + c <= P.limit || P.carved.count(ptr)) {
                P.free_[c].push_back(ptr);
                P.cached += c;
                return ICX_OK;
            }
        }
    }
    if (!c) {
        std::lock_guard<std::recursive_mutex> lk(ctx->mu);
        return fail(ctx, ICX_E_INVALID, "free of a buffer this context did not allocate");
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = P.host ? hipHostFree(ptr) : hipFree(ptr);
    if (e == hipSuccess) return ICX_OK;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    return hip_fail(ctx, e, "free");
}
}  // namespace

icx_status icx_device_alloc(icx_ctx* ctx, size_t bytes, void** ptr)
{
    return ctx ? pool_alloc(ctx, ctx->pool, bytes, ptr) : ICX_E_NULL;
}

icx_status icx_device_free(icx_ctx* ctx, void* ptr) { return ctx ? pool_free(ctx, ctx->pool, ptr) : ICX_E_NULL; }

icx_status icx_host_alloc(icx_ctx* ctx, size_t bytes, void** ptr)
{
    return ctx ? pool_alloc(ctx, ctx->hpool, bytes, ptr) : ICX_E_NULL;
}

icx_status icx_host_free(icx_ctx* ctx, void* ptr) { return ctx ? pool_free(ctx, ctx->hpool, ptr) : ICX_E_NULL; }

icx_status icx_memcpy(icx_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (!ctx || ((!dst || !src) && bytes)) return ICX_E_NULL;
    if (!bytes) return ICX_OK;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? ICX_OK : hip_fail(ctx, e, "hipMemcpy");
}

icx_status icx_upload(icx_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (!ctx || ((!dst || !src) && bytes)) return ICX_E_NULL;
    if (!bytes) return ICX_OK;
    const int k = (int)(ctx->up_next.fetch_add(1, std::memory_order_relaxed) % icx_ctx::UP_STREAMS);
    hipError_t e;
    {
        std::lock_guard<std::mutex> lk(ctx->up_mu[k]);
        e = hipSetDevice(ctx->device);
        if (e == hipSuccess && !ctx->up_stream[k]) e = hipStreamCreateWithFlags(&ctx->up_stream[k], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->up_stream[k]);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->up_stream[k]);
    }
    if (e == hipSuccess) return ICX_OK;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    return hip_fail(ctx, e, "icx_upload");
}

icx_status icx_debug_decode_cmyk(icx_ctx* ctx, const uint8_t* data, size_t len, uint8_t* out, size_t cap)
{
    if (!ctx || !data || !out) return ICX_E_NULL;
    icx_decode_job j{};
    j.data = data;
    j.len = len;
    j.subsampling = 1;
    j.out = out;
    j.cap = cap;
    const icx_status s = run_decode(ctx, &j, 1, nullptr, 0, true);
    return s != ICX_OK ? s : j.status;
}

icx_status icx_debug_decode_coefs(icx_ctx* ctx, const uint8_t* data, size_t len, int16_t* coefs, size_t ncoefs)
{
    if (!ctx || !data || !coefs) return ICX_E_NULL;
    icx_decode_job j{};
    j.data = data;
    j.len = len;
    j.subsampling = 1;
    const icx_status s = run_decode(ctx, &j, 1, coefs, ncoefs);
    return s != ICX_OK ? s : j.status;
}

}  // extern "C"
