// icx_kernels.h — launch wrappers of the gfx950 kernels (icx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "icx_internal.h"

namespace icx {

hipError_t upload_constants(const uint8_t nat_to_zz[64], const uint8_t zz_to_nat[64],
                            const uint32_t dc[2][16], const uint32_t ac[2][256],
                            const uint8_t hdr[2][HDR_COLOR]);

// kind: 0 = BGR24, 1 = RGB24, 2 = GRAY8
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

}  // namespace icx
