// icx_io.cpp — native reader side of the files -> files path (icx_stage_files).
//
// The reference's CompressionBatch runs processImage on availableProcessors()
// threads (CompressionBatch.java:64-88); each task stats the file, reads it
// and hands the bytes to the ImageIO reader (ImageCompression.java:53-76,
// 113-126).  Here the host threads only stage: per file the existence /
// readability check, the size (the -s gate is the caller's), one read into
// pinned memory, the JPEG header parse (icx_jpeg_info's rules) with the
// dimensions gate, and for a JPEG the device decoder will take, one copy to
// HBM on a copy stream of the context's own (icx_upload) - all without the
// Python interpreter lock, so a Python caller's reader threads overlap fully
// (DESIGN.md §9).  The caller decides every result (skip, format fallback,
// decode) from the staged facts, in the reference's order.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "../../include/icx.h"
#include "icx_context.h"
#include "icx_jpeg_parse.h"

using namespace icx;

static_assert(sizeof(icx_stage_job) == 80, "icx_stage_job layout (icx/_native.py StageJob)");

namespace {

// read the whole file (n bytes) at dst; 0 or an errno
int read_all(int fd, uint8_t* dst, size_t n)
{
    size_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, dst + got, n - got, (off_t)got);
        if (r < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (r == 0) return EIO;  // the file shrank under us
        got += (size_t)r;
    }
    return 0;
}

}  // namespace

extern "C" {

icx_status icx_stage_files(icx_ctx* ctx, icx_stage_job* jobs, int32_t n)
{
    if (!ctx || (!jobs && n > 0)) return ICX_E_NULL;
    if (n < 0) return ICX_E_INVALID;
    // pass 1: existence, readability, size (ImageCompression.java:55-59)
    int64_t biggest = 0;
    for (int i = 0; i < n; i++) {
        icx_stage_job& j = jobs[i];
        j.exists = 0;
        j.size = 0;
        j.read_errno = 0;
        j.jpeg_status = -1;
        j.width = j.height = j.ncomp = 0;
        j.dev = nullptr;
        j.status = ICX_OK;
        if (!j.path) {
            j.status = ICX_E_NULL;
            continue;
        }
        struct stat sb;
        if (stat(j.path, &sb) != 0 || access(j.path, R_OK) != 0) continue;
        j.exists = 1;
        j.size = (int64_t)sb.st_size;
        if (j.size > j.min_size) biggest = std::max(biggest, j.size);
    }
    if (biggest == 0) return ICX_OK;
    void* hbuf = nullptr;
    if (icx_status s = icx_host_alloc(ctx, (size_t)biggest, &hbuf)) return s;
    uint8_t* buf = (uint8_t*)hbuf;
    icx_status ret = ICX_OK;
    // pass 2: read, parse, gate, upload
    for (int i = 0; i < n && ret == ICX_OK; i++) {
        icx_stage_job& j = jobs[i];
        if (!j.exists || j.status != ICX_OK || j.size <= j.min_size) continue;
        const int fd = open(j.path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
            j.read_errno = errno;
            continue;
        }
        const int err = read_all(fd, buf, (size_t)j.size);
        close(fd);
        if (err) {
            j.read_errno = err;
            continue;
        }
        if (j.size < 2 || buf[0] != 0xFF || buf[1] != 0xD8) continue;  // not a JPEG: the caller's readers
        int32_t w = 0, h = 0, nc = 0;
        j.jpeg_status = icx_jpeg_info(buf, (size_t)j.size, &w, &h, &nc);
        j.width = w;
        j.height = h;
        j.ncomp = nc;
        if (j.jpeg_status != ICX_OK) continue;
        if (w <= j.min_width || h <= j.min_height) continue;  // ImageCompression.java:131: not decoded
        void* dev = nullptr;
        icx_status s = icx_device_alloc(ctx, (size_t)j.size, &dev);
        if (s == ICX_OK) s = icx_upload(ctx, dev, buf, (size_t)j.size);
        if (s != ICX_OK) {
            if (dev) icx_device_free(ctx, dev);
            j.status = s;
            if (s != ICX_E_NOMEM) ret = s;  // a device failure ends the call (the rest keep dev = NULL)
            continue;
        }
        j.dev = dev;
    }
    icx_host_free(ctx, hbuf);
    return ret;
}

}  // extern "C"
