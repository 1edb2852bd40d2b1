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

#include <algorithm>
#include <cstdlib>
#include <cstring>
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

icx_status read_header(icx_ctx* c, const uint8_t* data, size_t len, bool dev, JpegHeader& J)
{
    if (!dev) return parse_jpeg(data, len, len, J);
    std::vector<uint8_t> tmp;
    size_t avail = std::min<size_t>(len, 64 << 10);
    for (;;) {
        tmp.resize(avail);
        hipError_t e = hipMemcpy(tmp.data(), data, avail, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail(c, e, "header download");
        icx_status s = parse_jpeg(tmp.data(), avail, len, J);
        if (s != ICX_E_BUFFER || avail >= len) return s;
        avail = std::min(len, avail * 4);
    }
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
    } else {  // non-interleaved single component: one block per MCU
        d.hs = d.vs = 1;
        d.nby = d.nbmcu = 1;
        d.mcux = (J.w + 7) / 8;
        d.mcuy = (J.h + 7) / 8;
    }
    d.nblocks = (int64_t)d.mcux * d.mcuy * d.nbmcu;
    for (int c = 0; c < 3; c++) d.pw[c] = d.ph[c] = d.cw[c] = d.ch[c] = 0;
    for (int c = 0; c < J.ncomp; c++) {
        const int hc = J.ncomp == 3 ? (c == 0 ? d.hs : 1) : 1, vc = J.ncomp == 3 ? (c == 0 ? d.vs : 1) : 1;
        d.cw[c] = (J.w * hc + d.hs - 1) / d.hs;  // downsampled_width
        d.ch[c] = (J.h * vc + d.vs - 1) / d.vs;
        d.pw[c] = (d.cw[c] + 7) / 8 * 8;
        d.ph[c] = (d.ch[c] + 7) / 8 * 8;
    }
    d.fancy = J.ncomp == 3 && d.hs == 2 && d.cw[1] > 2;  // do_fancy_upsampling && downsampled_width > 2
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
    // Long subsequences re-walk least (measured on 4K q95: 16384 beats 8192 for
    // smooth and noise content); shorter ones only when the batch would not
    // give the chip ~64k threads.
    uint32_t S = 16384;
    while (S > 2048 && total_bits / S < 65536) S /= 2;
    return S;
}

// Warm-up walk before each subsequence (k_dec_init): long enough for typical
// content to resynchronise, short against the subsequence.
uint32_t warm_bits(uint32_t sub_bits)
{
    if (const char* e = getenv("ICX_DEC_WARM")) return (uint32_t)atol(e);
    return std::min<uint32_t>(4096, sub_bits / 4);
}

struct WPlan {
    Plan p;
    int64_t total;
};

icx_status plan_of(icx_ctx* c, const std::vector<int64_t>& counts, const int32_t* d_ids, WPlan& out)
{
    std::vector<int64_t> pre(counts.size() + 1, 0);
    for (size_t i = 0; i < counts.size(); i++) pre[i + 1] = pre[i] + counts[i];
    int64_t* d_pre = (int64_t*)c->dev.take(pre.size() * 8);
    icx_status s = upload(c, d_pre, pre.data(), pre.size() * 8);
    if (s) return s;
    out.p.ids = d_ids;
    out.p.prefix = d_pre;
    out.p.m = (int32_t)counts.size();
    out.total = pre.back();
    return ICX_OK;
}

// mode 0: decode to pixels; mode 1: coefficients only (debug: natural order, DC in [0])
icx_status run_decode(icx_ctx* c, icx_decode_job* jobs, int n, int16_t* coef_out, size_t coef_cap)
{
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    hipError_t he = hipSetDevice(c->device);
    if (he != hipSuccess) return hip_fail(c, he, "hipSetDevice");
    std::vector<DecItem> items;
    items.reserve(n);
    // headers of device-resident files: one batched download of their first 64 KiB
    const size_t HEAD = 64 << 10;
    std::vector<char> dev_in(n, 0);
    std::vector<const uint8_t*> head(n, nullptr);
    {
        size_t total = 0;
        for (int i = 0; i < n; i++)
            if (jobs[i].data && is_device_ptr(jobs[i].data)) {
                dev_in[i] = 1;
                total += align_up(std::min(jobs[i].len, HEAD), 64);
            }
        if (total) {
            hipError_t e = c->host.reserve(std::max<size_t>(total + 4096, 64 << 20));
            if (e != hipSuccess) return hip_fail(c, e, "hipHostMalloc");
            c->host.used = 0;
            for (int i = 0; i < n; i++)
                if (dev_in[i]) {
                    uint8_t* h = (uint8_t*)c->host.take(std::min(jobs[i].len, HEAD));
                    e = hipMemcpyAsync(h, jobs[i].data, std::min(jobs[i].len, HEAD), hipMemcpyDeviceToHost, c->stream);
                    if (e != hipSuccess) return hip_fail(c, e, "header download");
                    head[i] = h;
                }
            e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess) return hip_fail(c, e, "header download");
        }
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
            j.status = parse_jpeg(head[i], std::min(j.len, HEAD), j.len, it.J);
            if (j.status == ICX_E_BUFFER) j.status = read_header(c, j.data, j.len, true, it.J);  // header > 64 KiB
        } else {
            j.status = parse_jpeg(j.data, j.len, j.len, it.J);
        }
        j.src_width = it.J.w;
        j.src_height = it.J.h;
        if (j.status != ICX_OK) continue;
        const int s = j.subsampling > 0 ? j.subsampling : icx_subsampling_factor(it.J.w, it.J.h);
        it.s = s;
        it.nch = it.J.ncomp == 3 ? 3 : 1;
        j.fmt = it.nch == 3 ? ICX_BGR24 : ICX_GRAY8;
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
        items.push_back(it);
    }
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
            const int64_t scan_len = (int64_t)(it.job->len - it.J.scan_off);
            const int64_t nmcu = (int64_t)d.mcux * d.mcuy;
            d.nseg_max = it.J.ri ? (int32_t)((nmcu + it.J.ri - 1) / it.J.ri) + 1 : 1;
            it.ent_cap = (size_t)scan_len + (size_t)(DEC_PAD - 2) * d.nseg_max + DEC_TAIL + 64;
            it.ntiles = (scan_len + DEC_TILE - 1) / DEC_TILE;
            it.nblocks = d.nblocks;
            size_t per = align_up(scan_len + 64, 256) + align_up(it.ent_cap, 256) + it.ntiles * 8 + 512 +
                         (size_t)d.nseg_max * 4 + (size_t)d.nblocks * (128 + 4) + sizeof(DecTab) + 4096;
            for (int k = 0; k < 3; k++) per += align_up((size_t)d.pw[k] * d.ph[k], 256);
            per += (size_t)(it.ent_cap * 8 / 2048 + 2) * (8 + 2 + 4 + 4);  // subsequence arrays at S >= 2048
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
        hipError_t e = c->dev.reserve(need + (size_t)m * 64 * 1024 + (16 << 20));
        if (e != hipSuccess) {
            for (DecItem* it : sub) it->job->status = ICX_E_NOMEM;
            (void)hipGetLastError();
            c->err = "device workspace allocation failed";
            continue;
        }
        c->dev.used = 0;
        size_t host_need = 64 << 20;
        for (DecItem* it : sub)
            if (!it->dev_in && !is_pinned_ptr(it->job->data)) host_need += align_up(it->job->len, 64);
        e = c->host.reserve(host_need);
        if (e != hipSuccess) return hip_fail(c, e, "hipHostMalloc");
        c->host.used = 0;

        std::vector<DecTab> tabs(m);
        std::vector<DecState> states(m);
        DecTab* d_tab = (DecTab*)c->dev.take(sizeof(DecTab) * m);
        int64_t max_nsub = 0;
        for (int k = 0; k < m; k++) {
            DecItem& it = *sub[k];
            DecDesc& d = desc[k];
            if (!build_dec_tab(it.J, tabs[k])) {
                it.job->status = ICX_E_CORRUPT;
                states[k].status = 6;
            }
            const int64_t scan_len = (int64_t)(it.job->len - it.J.scan_off);
            d.scan_len = scan_len;
            d.ntiles = (int32_t)it.ntiles;
            uint8_t* scan = (uint8_t*)c->dev.take(align_up(scan_len + 64, 256));
            e = hipMemsetAsync(scan + scan_len, 0, 64, c->stream);
            const uint8_t* src = it.job->data + it.J.scan_off;
            if (!it.dev_in && !is_pinned_ptr(it.job->data)) {  // pageable: via pinned staging (DMA at link speed)
                uint8_t* h = (uint8_t*)c->host.take(scan_len);
                if (h) {
                    memcpy(h, src, scan_len);
                    src = h;
                }
            }
            if (e == hipSuccess)
                e = hipMemcpyAsync(scan, src, scan_len, it.dev_in ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                   c->stream);
            if (e != hipSuccess) return hip_fail(c, e, "scan upload");
            d.scan = scan;
            d.ent = (uint8_t*)c->dev.take(align_up(it.ent_cap, 256));
            d.ent_cap = (int64_t)it.ent_cap;
            d.tile_cnt = (uint32_t*)c->dev.take(it.ntiles * 4 + 4);
            d.tile_rst = (uint32_t*)c->dev.take(it.ntiles * 4 + 4);
            d.seg = (uint32_t*)c->dev.take((size_t)d.nseg_max * 4);
            d.nsub_max = (int32_t)((it.ent_cap * 8 + S - 1) / S);
            max_nsub = std::max<int64_t>(max_nsub, d.nsub_max);
            d.est = (uint64_t*)c->dev.take((size_t)(d.nsub_max + 1) * 8);
            d.wl[0] = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.wl[1] = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.ncnt = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.boff = (uint32_t*)c->dev.take((size_t)(d.nsub_max + 1) * 4);
            d.coefs = (int16_t*)c->dev.take((size_t)d.nblocks * 128);
            d.dc = (int32_t*)c->dev.take((size_t)d.nblocks * 4);
            if (!coef_out) {
                for (int q = 0; q < d.ncomp; q++) d.plane[q] = (uint8_t*)c->dev.take((size_t)d.pw[q] * d.ph[q]);
                it.host_out = !is_device_ptr(it.job->out);
                d.out = it.host_out ? (uint8_t*)c->dev.take(it.job->out_len) : it.job->out;
                d.ostride = d.ow * it.nch;
            }
            d.tab = d_tab + k;
            states[k].end = scan_len;  // coefficients need no clearing: the write pass stores whole blocks
        }
        DecDesc* d_desc = (DecDesc*)c->dev.take(sizeof(DecDesc) * m);
        DecState* d_state = (DecState*)c->dev.take(sizeof(DecState) * m);
        const int max_it = (int)max_nsub + 8;  // each launch settles at least one more subsequence
        uint32_t* d_changed = (uint32_t*)c->dev.take((size_t)max_it * 4);
        uint32_t* d_wlcnt = (uint32_t*)c->dev.take((size_t)m * max_it * 4);
        for (int k = 0; k < m; k++) desc[k].wl_cnt = d_wlcnt;
        uint32_t* h_changed = (uint32_t*)c->host.take(4);
        int32_t* d_ids = (int32_t*)c->dev.take((size_t)m * 4);
        std::vector<int32_t> ids(m);
        for (int k = 0; k < m; k++) ids[k] = k;
        icx_status st;
        if ((st = upload(c, d_tab, tabs.data(), sizeof(DecTab) * m)) ||
            (st = upload(c, d_desc, desc.data(), sizeof(DecDesc) * m)) ||
            (st = upload(c, d_state, states.data(), sizeof(DecState) * m)) ||
            (st = upload(c, d_ids, ids.data(), (size_t)m * 4)))
            return st;
        e = hipMemsetAsync(d_changed, 0, (size_t)max_it * 4, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(d_wlcnt, 0, (size_t)m * max_it * 4, c->stream);
        if (e != hipSuccess) return hip_fail(c, e, "counter clear");

        std::vector<int64_t> cnt_tiles(m), cnt_subs(m), cnt_blk(m), cnt_px(m), cnt_rows(m);
        int64_t stuffed = 0;
        for (int k = 0; k < m; k++) {
            cnt_tiles[k] = sub[k]->ntiles;
            cnt_subs[k] = (desc[k].nsub_max + 1 + 255) / 256;
            cnt_blk[k] = (desc[k].nblocks + 31) / 32;
            // colour: the row-pair kernel for s == 1 4:2:0 fancy, the per-pixel gather kernel otherwise
            const bool rows = desc[k].s == 1 && desc[k].ncomp == 3 && desc[k].hs == 2 && desc[k].vs == 2 &&
                              desc[k].fancy;
            cnt_px[k] = rows ? 0 : ((int64_t)desc[k].oh * ((desc[k].ow + 3) / 4) + 255) / 256;
            cnt_rows[k] = rows ? (int64_t)((desc[k].oh + 1) / 2) * ((desc[k].ow + 1023) / 1024) : 0;
            stuffed += desc[k].scan_len;
        }
        WPlan Pt, Ps, Pb, Pp, Pr;
        if ((st = plan_of(c, cnt_tiles, d_ids, Pt)) || (st = plan_of(c, cnt_subs, d_ids, Ps)) ||
            (st = plan_of(c, cnt_blk, d_ids, Pb)) || (st = plan_of(c, cnt_px, d_ids, Pp)) ||
            (st = plan_of(c, cnt_rows, d_ids, Pr)))
            return st;
        {
            Timed tm(c, "dec_unstuff", stuffed);
            launch_unstuff(d_desc, d_state, Pt.p, Pt.total, d_ids, m, S, c->stream);
        }
        {
            Timed tm(c, "dec_init", stuffed);
            launch_dec_init(d_desc, d_state, Ps.p, Ps.total, S, warm_bits(S), c->stream);
        }
        // ---- settle the subsequence entry states
        int it = 0;
        for (;;) {
            for (int k = 0; k < 4 && it < max_it; k++, it++) {
                Timed tm(c, "dec_sync", 0);
                launch_dec_sync(d_desc, d_state, Ps.p, Ps.total, S, it, max_it, d_changed + it, c->stream);
            }
            e = hipMemcpyAsync(h_changed, d_changed + it - 1, 4, hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess) return hip_fail(c, e, "sync counter");
            if (*h_changed == 0) break;
            if (it >= max_it) return fail(c, ICX_E_DEVICE, "entropy decode did not settle");
        }
        c->stats["dec_sync_iters"].launches += it;
        launch_dec_offsets(d_desc, d_state, d_ids, m, c->stream);
        {
            Timed tm(c, "dec_write", stuffed);
            launch_dec_write(d_desc, d_state, Ps.p, Ps.total, S, c->stream);
        }
        {
            Timed tm(c, "dec_dc", m);
            launch_dec_dc(d_desc, d_state, d_ids, m, c->stream);
        }
        int64_t px = 0;
        for (int k = 0; k < m; k++) px += (int64_t)desc[k].w * desc[k].h;
        if (!coef_out) {
            {
                Timed tm(c, "dec_idct", px);
                launch_dec_idct(d_desc, d_state, Pb.p, Pb.total, c->stream);
            }
            {
                Timed tm(c, "dec_color", px);
                launch_dec_color_420(d_desc, d_state, Pr.p, Pr.total, c->stream);
                launch_dec_color(d_desc, d_state, Pp.p, Pp.total, c->stream);
            }
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
            if (h_state[k].status) {
                j.status = ICX_E_CORRUPT;
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
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    const size_t c = DevPool::cls(bytes);
    auto f = P.free_.find(c);
    if (f != P.free_.end() && !f->second.empty()) {
        *ptr = f->second.back();
        f->second.pop_back();
        P.cached -= c;
    } else {
        hipError_t e = hipSetDevice(ctx->device);
        if (e == hipSuccess) e = P.host ? hipHostMalloc(ptr, c, hipHostMallocPortable) : hipMalloc(ptr, c);
        if (e != hipSuccess) return hip_fail(ctx, e, P.host ? "hipHostMalloc" : "hipMalloc");
    }
    P.live_[*ptr] = c;
    return ICX_OK;
}

icx_status pool_free(icx_ctx* ctx, DevPool& P, void* ptr)
{
    if (!ctx) return ICX_E_NULL;
    if (!ptr) return ICX_OK;
    std::lock_guard<std::recursive_mutex> lk(ctx->mu);
    auto l = P.live_.find(ptr);
    if (l == P.live_.end()) return fail(ctx, ICX_E_INVALID, "free of a buffer this context did not allocate");
    const size_t c = l->second;
    P.live_.erase(l);
    // A recycled buffer's next use is a copy or launch on this context's
    // stream, ordered after every launch that used it before, so recycling
    // needs no synchronisation.  (Host buffers: every call that reads one
    // synchronises before returning.)
    if (P.cached + c <= P.limit) {
        P.free_[c].push_back(ptr);
        P.cached += c;
        return ICX_OK;
    }
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess) e = P.host ? hipHostFree(ptr) : hipFree(ptr);
    return e == hipSuccess ? ICX_OK : hip_fail(ctx, e, "free");
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
