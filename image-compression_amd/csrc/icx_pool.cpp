// icx_pool.cpp — one handle over several GPUs for a single host process.
//
// The reference runs CompressionBatch's tasks on availableProcessors() threads
// of one JVM (CompressionBatch.java:64-88); a JNI host therefore needs every
// GPU of the node behind one handle.  A pool owns one context per device and
// splits each batched call into per-device shares, balanced by pixel count
// (largest first onto the least-loaded device: the same LPT rule as
// icx.pipeline.shard), runs the shares on one host thread per device and
// merges the per-job results back.  Jobs are independent (no data-path
// exchange between GPUs), so the shares need no collective; the learned
// cache stays on the caller's side as for a single context (icx_fit_job
// carries the caller's cache.get and returns what it would cache.put).
//
// Buffers of pool calls must be host memory: which device runs a job is
// decided here, so device-resident data belongs with icx_pool_context(i); a
// job with a device pointer gets ICX_E_INVALID and is not run.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <thread>
#include <vector>

#include "../../include/icx.h"
#include "icx_context.h"

struct icx_pool {
    std::vector<icx_ctx*> ctx;
};

namespace {

// Per-device job lists: indices into the caller's array, LPT by weight.
std::vector<std::vector<int>> shares(const std::vector<double>& weight, int ndev)
{
    std::vector<int> order(weight.size());
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return weight[a] > weight[b]; });
    std::vector<std::vector<int>> out(ndev);
    std::vector<double> load(ndev, 0.0);
    for (int i : order) {
        const int d = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        out[d].push_back(i);
        load[d] += weight[i];
    }
    for (auto& s : out) std::sort(s.begin(), s.end());  // keep the caller's order within a device
    return out;
}

bool host_only(const icx_fit_job& j) { return !icx::is_device_ptr(j.img.px) && !icx::is_device_ptr(j.out); }
bool host_only(const icx_decode_job& j) { return !icx::is_device_ptr(j.data) && !icx::is_device_ptr(j.out); }
bool host_only(const icx_png_fit_job& j) { return !icx::is_device_ptr(j.src.px) && !icx::is_device_ptr(j.dst); }

// Runs fn(ctx, jobs, n) on every device's share of `jobs` in parallel.
template <class Job, class Fn>
icx_status run_shares(icx_pool* p, Job* jobs, int32_t n, std::vector<double> weight, Fn fn)
{
    if (!p || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    const int ndev = (int)p->ctx.size();
    std::vector<char> run(n, 1);
    for (int i = 0; i < n; i++)
        if (!host_only(jobs[i])) {
            jobs[i].status = ICX_E_INVALID;
            run[i] = 0;
            weight[i] = -1.0;  // sorted last, dropped below
        }
    std::vector<std::vector<int>> sh = shares(weight, ndev);
    for (auto& s : sh) s.erase(std::remove_if(s.begin(), s.end(), [&](int i) { return !run[i]; }), s.end());
    std::vector<std::vector<Job>> part(ndev);
    std::vector<icx_status> st(ndev, ICX_OK);
    for (int d = 0; d < ndev; d++)
        for (int i : sh[d]) part[d].push_back(jobs[i]);
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; d++) {
        if (part[d].empty()) continue;
        th.emplace_back([&, d]() { st[d] = fn(p->ctx[d], part[d].data(), (int32_t)part[d].size()); });
    }
    for (auto& t : th) t.join();
    for (int d = 0; d < ndev; d++)
        for (size_t k = 0; k < sh[d].size(); k++) jobs[sh[d][k]] = part[d][k];
    for (icx_status s : st)
        if (s != ICX_OK) return s;
    return ICX_OK;
}

}  // namespace

extern "C" {

icx_status icx_pool_create(const int32_t* devices, int32_t ndev, icx_pool** out)
{
    if (!out || (!devices && ndev > 0)) return ICX_E_NULL;
    *out = nullptr;
    if (ndev <= 0) return ICX_E_INVALID;
    icx_pool* p = new icx_pool;
    for (int i = 0; i < ndev; i++) {
        icx_ctx* c = nullptr;
        const icx_status s = icx_create(devices[i], &c);
        if (s != ICX_OK) {
            for (icx_ctx* q : p->ctx) icx_destroy(q);
            delete p;
            return s;
        }
        p->ctx.push_back(c);
    }
    *out = p;
    return ICX_OK;
}

void icx_pool_destroy(icx_pool* pool)
{
    if (!pool) return;
    for (icx_ctx* c : pool->ctx) icx_destroy(c);
    delete pool;
}

int32_t icx_pool_size(const icx_pool* pool) { return pool ? (int32_t)pool->ctx.size() : 0; }

icx_ctx* icx_pool_context(icx_pool* pool, int32_t i)
{
    return pool && i >= 0 && i < (int32_t)pool->ctx.size() ? pool->ctx[i] : nullptr;
}

icx_status icx_pool_compress_jpg_batch(icx_pool* pool, icx_fit_job* jobs, int32_t n)
{
    if (!pool || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    std::vector<double> w(n);
    for (int i = 0; i < n; i++) w[i] = (double)jobs[i].img.width * jobs[i].img.height;
    return run_shares(pool, jobs, n, w, icx_compress_jpg_batch);
}

icx_status icx_pool_decode_jpg_batch(icx_pool* pool, icx_decode_job* jobs, int32_t n)
{
    if (!pool || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    std::vector<double> w(n);
    for (int i = 0; i < n; i++) w[i] = (double)jobs[i].len;  // compressed bytes: the entropy decode's work
    return run_shares(pool, jobs, n, w, icx_decode_jpg_batch);
}

icx_status icx_pool_png_fit_batch(icx_pool* pool, icx_png_fit_job* jobs, int32_t n)
{
    if (!pool || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    std::vector<double> w(n);
    for (int i = 0; i < n; i++) w[i] = (double)jobs[i].src.width * jobs[i].src.height;
    return run_shares(pool, jobs, n, w, icx_png_fit_batch);
}

}  // extern "C"
