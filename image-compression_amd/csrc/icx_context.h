// icx_context.h — per-context state shared by the encode and decode drivers
// (one HIP stream, device workspace arena, pinned staging arena, per-kernel
// HIP-event timing) and the small helpers around it.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>

#include <algorithm>
#include <cstring>
#include <map>
#include <atomic>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/icx.h"
#include "icx_internal.h"

namespace icx {

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ------------------------------------------------------------ arenas
struct DevArena {
    uint8_t* base = nullptr;
    size_t cap = 0, used = 0;
    hipError_t reserve(size_t bytes)
    {
        if (bytes <= cap) return hipSuccess;
        if (base) hipFree(base);
        base = nullptr;
        cap = 0;
        size_t want = std::max(bytes, cap * 3 / 2);
        hipError_t e = hipMalloc(&base, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            e = hipMalloc(&base, bytes);
            if (e != hipSuccess) return e;
            want = bytes;
        }
        cap = want;
        return hipSuccess;
    }
    void* take(size_t n)
    {
        used = align_up(used, 256);
        void* p = base + used;
        used += n;
        if (used > cap) overflow = true;  // a sizing bug: callers fail the call before any launch
        return p;
    }
    bool overflow = false;
    ~DevArena() { if (base) hipFree(base); }
};

struct HostArena {
    uint8_t* base = nullptr;
    size_t cap = 0, used = 0;
    hipError_t reserve(size_t bytes)
    {
        if (bytes <= cap) return hipSuccess;
        if (base) hipHostFree(base);
        base = nullptr;
        size_t want = std::max(bytes, cap * 2);
        hipError_t e = hipHostMalloc((void**)&base, want, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        cap = want;
        return hipSuccess;
    }
    void* take(size_t n)
    {
        used = align_up(used, 64);
        if (used + n > cap) return nullptr;
        void* p = base + used;
        used += n;
        return p;
    }
    ~HostArena() { if (base) hipHostFree(base); }
};

struct Pending {
    std::string name;
    hipEvent_t a, b;
    int64_t units;
};

struct KStat {
    int64_t launches = 0, units = 0;
    double ms = 0;
};


// Device or host buffer?  hipPointerGetAttributes costs ~0.25 us and the
// drivers ask per image several times a call, so device allocation ranges
// (hipMemGetAddressRange of a pointer found to be device memory) are kept in
// a process-wide map and later pointers inside one are answered without a
// HIP call.  Device virtual ranges stay reserved by the runtime after a free,
// so a cached range never holds a host pointer.
inline bool is_device_ptr(const void* p)
{
    if (!p) return false;
    static std::mutex mu;
    static std::map<uintptr_t, uintptr_t> ranges;  // base -> end
    const uintptr_t a = (uintptr_t)p;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = ranges.upper_bound(a);
        if (it != ranges.begin() && a < (--it)->second) return true;
    }
    hipPointerAttribute_t at;
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const bool dev = at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
    if (dev) {
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && base && size) {
            std::lock_guard<std::mutex> g(mu);
            ranges[(uintptr_t)base] = (uintptr_t)base + size;
        } else {
            (void)hipGetLastError();
        }
    }
    return dev;
}


}  // namespace icx

// ============================================================ context
// Caching allocator behind icx_device_alloc/free: freed buffers are kept by
// size class (power of two) and handed out again, so a pipeline that
// allocates a frame buffer per image never pays hipMalloc/hipFree (which
// synchronise the device) after warm-up.
struct DevPool {
    std::map<size_t, std::vector<void*>> free_;
    std::map<void*, size_t> live_;
    size_t cached = 0, limit = (size_t)16 << 30;
    static size_t cls(size_t n)
    {
        size_t c = 1 << 16;
        while (c < n) c <<= 1;
        return c;
    }
    bool host = false;  // pinned host pool (hipHostMalloc) instead of device memory
    // pinned buffers below kSlabMax are carved from slabs of >= kSlab bytes:
    // one hipHostMalloc per slab (a pinned allocation costs milliseconds and
    // the runtime serialises them: a batch's first run read files at 2 GB/s
    // with one allocation per file); carved buffers always return to the free
    // lists, the slabs are released with the pool
    static constexpr size_t kSlab = (size_t)64 << 20, kSlabMax = (size_t)16 << 20;
    // device buffers of 1-32 MiB (staged files, decoded 4K frames) likewise,
    // 16 per slab: a first files -> files run staged ~500 files and decoded
    // as many frames with one hipMalloc each (round 5)
    static constexpr size_t kDevSlabMin = (size_t)1 << 20, kDevSlabMax = (size_t)32 << 20;
    bool slabbed(size_t c) const { return host ? c <= kSlabMax : c >= kDevSlabMin && c <= kDevSlabMax; }
    size_t slab_bytes(size_t c) const { return host ? (c > kSlab ? c : kSlab) : 16 * c; }
    std::vector<void*> slabs;
    std::set<void*> carved;
    ~DevPool()
    {
        for (auto& kv : free_)
            for (void* p : kv.second)
                if (!carved.count(p)) (void)(host ? hipHostFree(p) : hipFree(p));
        for (auto& kv : live_)
            if (!carved.count(kv.first)) (void)(host ? hipHostFree(kv.first) : hipFree(kv.first));
        for (void* s : slabs) (void)(host ? hipHostFree(s) : hipFree(s));
    }
};

inline bool is_pinned_ptr(const void* p)
{
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

struct icx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::recursive_mutex mu;
    std::string err;
    icx::DevArena dev;
    icx::HostArena host;
    bool prof = false;
    std::vector<icx::Pending> pending;
    std::vector<hipEvent_t> evpool;
    std::map<std::string, icx::KStat> stats;
    size_t budget = 0;  // device workspace budget per sub-batch
    int table_layout = 0;  // ICX_TABLES_SEPARATE / ICX_TABLES_GROUPED (icx_set_table_layout)
    // inverse colour maps of the default TYPE_BYTE_INDEXED [0] / TYPE_BYTE_BINARY
    // [1] maps (32x32x32, device), built at the first palette resize
    uint8_t* d_inv[2] = {nullptr, nullptr};
    int inv_prims[2] = {0, 0};
    DevPool pool;
    DevPool hpool;  // pinned host buffers (hpool.host = true)
    // the pools' own lock: host threads reading files into pinned buffers must
    // not wait for a batch call, which holds `mu` for its whole run
    std::mutex pool_mu;
    // Host-buffer batches: inputs are uploaded (io_up) into one of two staging
    // arenas while the previous sub-batch computes, outputs leave (io_down)
    // while the next one computes; created on first use.
    hipStream_t io_up = nullptr, io_down = nullptr;
    // decoder: images whose entry states settled early finish on the dec_aux
    // streams (one per settling check, round robin) while the others keep
    // relaxing on `stream` (created at the first decode)
    static constexpr int DEC_AUX_MAX = 4;
    int n_dec_aux = 0;
    hipStream_t dec_aux[DEC_AUX_MAX] = {};
    hipEvent_t ev_dec_split = nullptr, ev_dec_aux[DEC_AUX_MAX] = {};
    hipEvent_t ev_dec_wr[DEC_AUX_MAX] = {};  // an aux stream's last write pass (split tails)
    icx::DevArena stage[2];
    hipEvent_t ev_up[2] = {nullptr, nullptr}, ev_down[2] = {nullptr, nullptr}, ev_done = nullptr;
    // icx_upload: host threads push file bytes to HBM on their own copy
    // streams, without `mu`, while a batch call runs its kernels on `stream`
    static constexpr int UP_STREAMS = 4;
    std::mutex up_mu[UP_STREAMS];
    hipStream_t up_stream[UP_STREAMS] = {};
    std::atomic<unsigned> up_next{0};
};

namespace icx {

inline icx_status fail(icx_ctx* c, icx_status s, const char* msg)
{
    if (c) c->err = msg;
    return s;
}

inline icx_status hip_fail(icx_ctx* c, hipError_t e, const char* where)
{
    if (c) c->err = std::string(where) + ": " + hipGetErrorString(e);
    (void)hipGetLastError();
    return e == hipErrorOutOfMemory ? ICX_E_NOMEM : ICX_E_DEVICE;
}

inline hipEvent_t get_event(icx_ctx* c)
{
    if (!c->evpool.empty()) {
        hipEvent_t e = c->evpool.back();
        c->evpool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

// Times one launch when profiling is on: its events go to the launch
// wrapper (g_launch_timing), which records them in the dispatch itself; a
// region whose wrapper launched nothing returns them unused
// (ext).  Without ext, events are recorded on the stream around the region.
struct Timed {
    icx_ctx* c;
    Pending p;
    bool on, ext;
    hipStream_t st;  // the stream the region's launches go to (default: the context's)
    Timed(icx_ctx* ctx, const char* name, int64_t units, bool ext_launch = false, hipStream_t stream = nullptr)
        : c(ctx), on(ctx->prof), ext(ext_launch), st(stream ? stream : ctx->stream)
    {
        if (!on) return;
        p.name = name;
        p.units = units;
        p.a = get_event(c);
        p.b = get_event(c);
        if (ext) g_launch_timing = LaunchTiming{p.a, p.b, false};
        else hipEventRecord(p.a, st);
    }
    ~Timed()
    {
        if (!on) return;
        if (!ext) {
            hipEventRecord(p.b, st);
            c->pending.push_back(p);
            return;
        }
        const bool used = g_launch_timing.used;
        g_launch_timing = LaunchTiming{};
        if (used) {
            c->pending.push_back(p);
        } else {
            c->evpool.push_back(p.a);
            c->evpool.push_back(p.b);
        }
    }
};

// Host wall time of a region into the profile (name: "host.*"), when profiling.
struct HostSpan {
    icx_ctx* c;
    const char* name;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~HostSpan()
    {
        if (!c->prof) return;
        KStat& k = c->stats[name];
        k.launches++;
        k.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
};

inline void resolve_profile(icx_ctx* c)  // call after a stream synchronisation
{
    for (auto& p : c->pending) {
        float ms = 0;
        hipEventElapsedTime(&ms, p.a, p.b);
        KStat& s = c->stats[p.name];
        s.launches++;
        s.ms += ms;
        s.units += p.units;
        c->evpool.push_back(p.a);
        c->evpool.push_back(p.b);
    }
    c->pending.clear();
}

inline icx_status upload(icx_ctx* c, void* dst, const void* src, size_t n)
{
    void* h = c->host.take(n);
    if (!h) return fail(c, ICX_E_NOMEM, "pinned staging exhausted");
    memcpy(h, src, n);
    hipError_t e = hipMemcpyAsync(dst, h, n, hipMemcpyHostToDevice, c->stream);
    return e == hipSuccess ? ICX_OK : hip_fail(c, e, "hipMemcpyAsync(H2D)");
}

// Packs a launch's small host->device arguments (descriptors, tables, work
// plans) into one pinned block and one copy.  alloc() hands out the device
// address at once (so descriptors can point at each other) and the host slot
// to fill before flush().
struct Uploader {
    icx_ctx* c;
    uint8_t *h = nullptr, *d = nullptr;
    size_t cap = 0, used = 0, flushed = 0;
    bool overflow = false;
    Uploader(icx_ctx* ctx, size_t bytes) : c(ctx), cap(bytes)
    {
        h = (uint8_t*)c->host.take(bytes);
        d = (uint8_t*)c->dev.take(bytes);
    }
    template <class T>
    T* alloc(size_t count, T** host)
    {
        used = align_up(used, 64);
        const size_t n = sizeof(T) * count;
        if (!h || used + n > cap) {
            overflow = true;
            *host = nullptr;
            return nullptr;
        }
        *host = (T*)(h + used);
        T* p = (T*)(d + used);
        used += n;
        return p;
    }
    template <class T>
    T* put(const T* src, size_t count)
    {
        T* hp;
        T* p = alloc<T>(count, &hp);
        if (hp) memcpy((void*)hp, (const void*)src, sizeof(T) * count);
        return p;
    }
    // Bytes to reserve for `count` objects of T (with the 64-byte alignment).
    template <class T>
    static size_t need(size_t count) { return align_up(sizeof(T) * count, 64); }
    // Copies what was put since the last flush (one copy); puts may follow.
    icx_status flush()
    {
        if (overflow) return fail(c, ICX_E_NOMEM, "upload staging exhausted");
        if (used == flushed) return ICX_OK;
        hipError_t e = hipMemcpyAsync(d + flushed, h + flushed, used - flushed, hipMemcpyHostToDevice, c->stream);
        flushed = used;
        return e == hipSuccess ? ICX_OK : hip_fail(c, e, "hipMemcpyAsync(H2D)");
    }
};

}  // namespace icx
