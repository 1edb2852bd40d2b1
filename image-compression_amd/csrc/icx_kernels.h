// icx_kernels.h — launch wrappers of the gfx950 kernels (icx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "icx_internal.h"

namespace icx {

// Digest of the encoder's constant tables: on the device (from its symbols,
// into *out) and on the host (from the tables upload_constants takes).
void launch_const_digest(uint64_t* out, hipStream_t st);
uint64_t const_digest_host(const uint8_t nat_to_zz[64], const uint8_t zz_to_nat[64], const uint32_t dc[2][16],
                           const uint32_t ac[2][256], const uint8_t hdr[4][HDR_COLOR], const int8_t dith[3][64]);
hipError_t upload_constants(const uint8_t nat_to_zz[64], const uint8_t zz_to_nat[64],
                            const uint32_t dc[2][16], const uint32_t ac[2][256],
                            const uint8_t hdr[4][HDR_COLOR], const int8_t dith[3][64]);

// kind: 0 = BGR24, 1 = RGB24, 2 = GRAY8
// ImgState::list_entries of a plan's images after their FDCT (byte accounting)
void launch_list_count(const ImgDesc* d, ImgState* s, const Plan& p, hipStream_t st);
void launch_fdct(const ImgDesc* d, ImgState* s, const QNode* n, const Plan& p, int64_t tiles, int kind,
                 hipStream_t st);
void launch_huff(const ImgDesc* d, const ImgState* s, const QNode* n, const Plan& p, int64_t chunks, bool rev,
                 hipStream_t st);
// k_scan: the trial's offsets, exact file size and one binary-search step (decide)
void launch_scan(const ImgDesc* d, ImgState* s, const QNode* n, const Plan& p, hipStream_t st);
void launch_ffscan(const ImgDesc* d, ImgState* s, const Plan& p, hipStream_t st);
void launch_stuff(const ImgDesc* d, const ImgState* s, const QNode* n, const Plan& p, int64_t chunks,
                  hipStream_t st);
void launch_resize(const uint8_t* src, int sw, int sh, int sstride, int fmt, uint8_t* dst, int dw,
                   int dh, int dstride, hipStream_t st);
// Batched resize (icx_png_fit_batch): m descriptors of one pixel format in
// device memory, prefix = exclusive tile counts (prefix[m] = tiles), uniform
// = tiles per image when every image has as many (2-D grid), else 0.
struct ResizeArgs {
    const uint8_t* src;
    uint8_t* dst;
    int32_t sw, sh, sstride, fmt;
    int32_t dw, dh, dstride, tiles_x;
    int64_t x0l, dxl, y0l, dyl;  // inverse scale (32.32) and the first pixel centre's source position
    // ICX_INDEXED8 / ICX_BINARY1: the source's colour map (device, 256 entries)
    // and the inverse map of the destination's default one (device, 32x32x32)
    const uint32_t* pal = nullptr;
    const uint8_t* inv = nullptr;
    int32_t prims = 0;  // the destination map represents the primaries (no dither for them)
};
ResizeArgs resize_args(const uint8_t* src, int sw, int sh, int sstride, int fmt, uint8_t* dst, int dw, int dh,
                       int dstride);
int64_t resize_tiles(int dw, int dh);
void launch_resize_one(const ResizeArgs& a, hipStream_t st);
void launch_resize_batch(int fmt, const ResizeArgs* descs, const int64_t* prefix, int m, int64_t tiles,
                         int64_t uniform, hipStream_t st);

}  // namespace icx
