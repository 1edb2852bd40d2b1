// FETCH_SIZE calibration for k_huff's access pattern (rocprofv3 PMC).
//
// MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a wide
// coalesced streaming read; other access shapes are uncalibrated.  k_huff
// reads candidate lists the way `gather_lists` below does - one thread per
// scan block, the block's list offset (4 B) and length (1 B), then 16-B
// groups of its list (packed per MCU of 6 blocks in 1536-B regions) - so
// this program runs kernels with known byte counts under `rocprofv3 --pmc
// FETCH_SIZE` and prints each kernel's algorithmic bytes:
//   stream16        16 B per lane, contiguous (the guide's calibrated shape)
//   gather_noise    lists of a uniform-noise 4K frame's length mix (~16 entries)
//   gather_smooth   lists of a smooth frame's mix (~5 entries)
// Buffers are 4 GiB, well past the 256 MiB Infinity Cache, and a 1 GiB
// store sweep runs between the kernels, so every read comes from HBM.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/calib_fetch.hip -o image-compression_amd/lib/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                                                     \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                 \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

__global__ void stream16(const uint4* __restrict__ src, size_t n, uint32_t* __restrict__ sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // never true for this data; keeps the loads
}

// k_huff's list read: thread = block; meta loads, then 16-B groups j < cnt.
__global__ __launch_bounds__(256) void gather_lists(const uint32_t* __restrict__ coefs,
                                                    const uint32_t* __restrict__ coff,
                                                    const uint8_t* __restrict__ ncoef, int64_t nblocks,
                                                    uint32_t* __restrict__ sink)
{
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= nblocks) return;
    const int cnt = ncoef[b];
    const uint4* lst = (const uint4*)(coefs + 4 * (size_t)coff[b]);
    uint32_t acc = 0;
    for (int j = 0; j < cnt; j += 4) {
        const uint4 v = lst[j / 4];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void sweep(uint4* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main()
{
    const size_t kBytes = (size_t)4 << 30;
    uint4* big = nullptr;
    uint4* flush = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&big, kBytes));
    CHECK(hipMalloc(&flush, (size_t)1 << 30));
    CHECK(hipMalloc(&sink, 64));
    const size_t n16 = kBytes / 16;
    hipLaunchKernelGGL(sweep, dim3(8192), dim3(256), 0, 0, big, n16);
    CHECK(hipDeviceSynchronize());
    auto flush_caches = [&] {
        hipLaunchKernelGGL(sweep, dim3(8192), dim3(256), 0, 0, flush, ((size_t)1 << 30) / 16);
        CHECK(hipDeviceSynchronize());
    };
    flush_caches();
    hipLaunchKernelGGL(stream16, dim3(16384), dim3(256), 0, 0, big, n16, sink);
    CHECK(hipDeviceSynchronize());
    printf("stream16 algorithmic_bytes %zu\n", kBytes);

    // Lists: MCUs of 6 blocks (Y0 Y1 Y2 Y3 Cb Cr), each block's list padded
    // to 4 entries, packed from the start of the MCU's 384-entry region.
    std::mt19937 rng(7);
    for (int kind = 0; kind < 2; kind++) {
        // length distributions (entries incl. DC) close to the headline's
        std::normal_distribution<double> luma(kind == 0 ? 19.0 : 6.0, kind == 0 ? 5.0 : 2.5);
        std::normal_distribution<double> chroma(kind == 0 ? 9.0 : 2.0, kind == 0 ? 3.0 : 1.0);
        const int64_t nmcu = (int64_t)(kBytes / (384 * 4)) - 1;
        const int64_t nblocks = nmcu * 6;
        std::vector<uint32_t> off((size_t)nblocks);
        std::vector<uint8_t> len((size_t)nblocks);
        size_t algo = 0;
        for (int64_t m = 0; m < nmcu; m++) {
            uint32_t pos = (uint32_t)(m * 384);
            for (int k = 0; k < 6; k++) {
                const double v = k < 4 ? luma(rng) : chroma(rng);
                const int l = std::min(64, std::max(1, (int)(v + 0.5)));
                off[(size_t)(m * 6 + k)] = pos / 4;
                len[(size_t)(m * 6 + k)] = (uint8_t)l;
                const int padded = (l + 3) & ~3;
                pos += padded;
                algo += (size_t)padded * 4 + 5;
            }
        }
        uint32_t* doff = nullptr;
        uint8_t* dlen = nullptr;
        CHECK(hipMalloc(&doff, off.size() * 4));
        CHECK(hipMalloc(&dlen, len.size()));
        CHECK(hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dlen, len.data(), len.size(), hipMemcpyHostToDevice));
        flush_caches();
        hipLaunchKernelGGL(gather_lists, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, 0,
                           (const uint32_t*)big, doff, dlen, nblocks, sink);
        CHECK(hipDeviceSynchronize());
        printf("%s algorithmic_bytes %zu blocks %lld mean_padded_entries %.2f\n",
               kind == 0 ? "gather_noise" : "gather_smooth", algo, (long long)nblocks,
               (double)(algo - 5 * (size_t)nblocks) / 4.0 / (double)nblocks);
        CHECK(hipFree(doff));
        CHECK(hipFree(dlen));
    }
    CHECK(hipFree(big));
    CHECK(hipFree(flush));
    CHECK(hipFree(sink));
    return 0;
}
