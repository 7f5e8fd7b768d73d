// dcr_writer.h — kernel arguments of the device record writer
// (dcr_writer.hip); not part of the C-ABI (include/dcr.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dcr.h"

namespace dcrw {

struct FmtArgs {
    dcr_out ss, ds;                 // device kernel outputs
    const int32_t *sub_off;         // [4F+1]
    const uint8_t *read_mapq;
    const int64_t *ss_col_off, *ds_col_off;
    const dcr_read_info *info;      // per-read preprocessing status
    const char *names;
    const int64_t *fam_code, *fam_rx;
    const int32_t *fam_tid;
    int32_t n_fam;
    int32_t *fam_fail;              // [F] DCR_FAIL_* | which << 8
    int32_t *ds_len_out;            // [2F]
    int64_t *rec_size;              // [2F+1] (the last one 0: the scan's total)
    int64_t *rec_off;               // [2F+1]
    uint8_t *stream;                // formatted records
};

#ifndef DFL_CLAIM
#define DFL_CLAIM 1   // pipeline k_deflate: blocks claimed from a counter (0: workgroup w takes w, w + grid, ...)
#endif
struct DflArgs {
    const uint8_t *stream;
    const int64_t *stream_bytes;    // device scalar (rec_off[2F])
    uint8_t *slots;                 // 64 KiB per block
    int64_t *sizes;                 // per block (0 past the last block)
    uint32_t *tok;                  // dfl::kTokWords per workgroup of the grid
    unsigned long long *stamps;     // diagnostic (dcr_deflate_probe): s_memtime cycles per phase, or null
    unsigned long long *claim;      // zeroed block counter: workgroups claim blocks from it (null: a fixed stride)
};

struct CompactArgs {
    const uint8_t *slots;
    const int64_t *sizes;
    const int64_t *offs;            // exclusive scan of sizes
    const int64_t *stream_bytes;
    uint8_t *out;
    int64_t *totals;                // [3] compressed bytes, formatted bytes, blocks
};

__global__ void k_famfail(FmtArgs A);
__global__ void k_fmt_size(FmtArgs A);
__global__ void k_fmt_write(FmtArgs A);
__global__ void k_deflate(DflArgs D);
__global__ void k_compact(CompactArgs C);

// exclusive prefix sum out[i] = in[0] + .. + in[i-1] (in != out), tmp of
// scan_tmp_bytes(n) bytes; launches on s
size_t scan_tmp_bytes(int n);
hipError_t scan_excl_i64(const int64_t *in, int64_t *out, int n, int64_t *tmp, hipStream_t s);

}  // namespace dcrw
