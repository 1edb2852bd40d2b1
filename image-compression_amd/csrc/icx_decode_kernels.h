// icx_decode_kernels.h — launch wrappers of the device JPEG decoder (icx_decode.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "icx_decode.h"
#include "icx_internal.h"

namespace icx {

// tiles: per job ceil(dst_len / STAGE_TILE) workgroups (Plan.ids unused)
void launch_stage(const StageJob* jobs, const Plan& tiles, int64_t nwg, hipStream_t st);
// cnt / tiles: per image ceil(ntiles / DEC_UNSTUFF_TILES) / ceil(ntiles / DEC_SCATTER_TILES) work items (4 KiB stuffed tiles)
void launch_unstuff(const DecDesc* d, DecState* s, const Plan& cnt, int64_t ncnt, const Plan& tiles, int64_t ntiles,
                    const int32_t* ids, int m, uint32_t sub_bits, hipStream_t st);
// subs: per image ceil((nsub_max + 1) / 256) workgroups
// warm: bits decoded before each subsequence start to estimate its entry state
void launch_dec_init(const DecDesc* d, const DecState* s, const Plan& subs, int64_t nwg, uint32_t sub_bits,
                     uint32_t warm, hipStream_t st);
// iter 0 walks every subsequence, iter r > 0 the worklist built by iter r-1;
// wl_cnt holds nimg counters per launch (wl_cnt[r * nimg + image], zeroed before iter 0)
void launch_dec_sync(const DecDesc* d, const DecState* s, const Plan& subs, int64_t nwg, uint32_t sub_bits,
                     int iter, int nimg, uint32_t* changed, hipStream_t st);
void launch_dec_offsets(const DecDesc* d, DecState* s, const int32_t* ids, int m, hipStream_t st);
void launch_dec_write(const DecDesc* d, DecState* s, const Plan& subs, int64_t nwg, uint32_t sub_bits,
                      hipStream_t st);
void launch_dec_dc(const DecDesc* d, const DecState* s, const int32_t* ids, int m, hipStream_t st);
// blocks: per image ceil(nblocks / 32) workgroups (fuse420 images: ceil(2 * mcux * mcuy / 32))
void launch_dec_idct(const DecDesc* d, const DecState* s, const Plan& blocks, int64_t nwg, hipStream_t st);
// px: per image ceil(oh * ceil(ow / 4) / 256) workgroups (any source subsampling)
void launch_dec_color(const DecDesc* d, const DecState* s, const Plan& px, int64_t nwg, hipStream_t st);
// tiles: per image mcuy * ceil(mcux / 8) workgroups (fuse420 images only)
void launch_dec_luma_color_420(const DecDesc* d, const DecState* s, const Plan& tiles, int64_t nwg, hipStream_t st);

}  // namespace icx
