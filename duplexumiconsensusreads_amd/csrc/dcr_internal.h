// dcr_internal.h — types shared by dcr_kernels.hip and dcr_capi.hip (not part
// of the C-ABI; include/dcr.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/dcr.h"

namespace dcr {

// sets dcr_last_error() (dcr_capi.hip) and returns code
int set_error(int code, const std::string &msg);

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kRecmetaWaves = 16;   // k_recmeta: waves per block (one list atomic per block), at most
// k_recmeta's dynamic LDS for a block of nw waves: RecAgg[nw][64], int[nw][64], int[3][nw]
inline size_t recmeta_lds_bytes(int nw) { return (size_t)nw * (48 * 64 + 4 * 64 + 12); }
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kFastWaves = 4;               // k_consensus_fast: five 4-wave blocks per CU (5 waves per SIMD)
constexpr int kFastBlock = kWave * kFastWaves;
constexpr int kDeepReads = 64;              // k_decide: single-strand records of this many reads go to k_decide_deep
constexpr int kDeepWaves = 8;               // k_decide_deep: waves per record (one 512-thread block, two per CU)

// Per-record launch metadata written by k_recmeta for the fast kernel, in
// fast-list order (one scalar 32-byte load per record).
struct RecMeta {
    uint32_t base_al;   // 16-aligned byte offset of the record's kept bases/quals (< 2^32 - 4096)
    int32_t d0;         // pos of the record's first read - min_pos (< 2^16) | MAPQ << 16
    int64_t off;        // output column offset (ss_col_off / ds_col_off)
    int32_t rec;        // record index
    int32_t g0;         // index of its first read in the read-meta array
    int32_t minpos;     // min_pos (:458)
    uint32_t w;         // R | T << 7 | staged dwords << 15
};
static_assert(sizeof(RecMeta) == 32, "RecMeta is one s_load_dwordx8");

#ifndef DCR_LAYOUT_KERNEL
#define DCR_LAYOUT_KERNEL 1   // insertion layouts by events in k_ins_layout (0: the general kernel steps columns)
#endif

struct Workspace {
    dcr_read_info *info;    // [n_reads]
    uint32_t *norm_cig;     // [n_cigar] normalised runs (M/I/D)
    int32_t *cons;          // [cols] consensus char | quality << 8 (T > kColsLds)
    double *et;             // [cols] e/d per kept column        (T > kColsLds)
    uint8_t *insflag;       // [ss cols] insertion-column flags (R > 64 layout)
    int4 *state;            // [n_reads] layout state (R > 64)
    int *err;               // [1] capacity error flag
    int *ovf;               // [n_rec] records for the general kernel
    int *ovf_count;         // [2] single-strand / duplex general-list lengths
    int *fast_count;        // [2] single-strand / duplex fast-list lengths
    int *xcount;            // [2] single-strand / duplex exact-queue lengths
    int *gen_next;          // [2] next general-list entry to claim (k_consensus_general)
    int *deep;              // [n_rec] general-list indices of deep single-strand records (k_decide_deep)
    int *deep_count;        // [1] their number
    int *lay_next;          // [2] next general-list entry to claim (k_ins_layout)
    int *xlist;             // [n_rec] exact queue: fast-list indices (k_consensus_fast<., true>)
    unsigned long long *stamps;   // [32] diagnostic phase cycles (DCR_STAMP builds only)
    RecMeta *meta;          // [n_rec] fast list
    uint4 *rows;            // [n_rec] per fast-list entry: the record's scalars as k_consensus_fast
                            // decided them (pos, T | D << 8 | M << 16 | MAPQ << 24, mean numerator
                            // or 0, kind), expanded into dcr_out by k_fast_rows; kind 0 = not decided
    uint2 *rmeta;           // [max(n_reads, 4F)] per read: len | mapq << 8 | (pos - pos of the record's
                            // first read) << 16 (int16), seq_start (low 32 bits)
    // insertion layouts by events (k_ins_layout), per general-list record of
    // either strand (single-strand 4F, then duplex 2F): 1 when laid out, -1
    // when the general kernel lays it out itself; its insertion-column mask;
    // its element codes, kLayRow per read at a fixed place (single-strand:
    // from sub_off[rec] * kLayRow; duplex record p: from (n_reads + 2p) *
    // kLayRow; a same-counter atomic per record cost milliseconds), tile-major
    // ([32-column tile][read][32]): a tile of every read is one contiguous
    // block, copied into the general kernel's LDS tile with 16-byte loads
    int *lay_base;          // [6F]
    uint64_t *lay_mask;     // [6F][4]
    uint16_t *lay;          // [(n_reads + 4F) * kLayRow]
};
constexpr int kLayRow = 256;        // columns per laid-out row (records of T <= 256)

struct Args {
    dcr_batch in;
    const dcr_params *P;
    Workspace ws;
    dcr_out ss;
    dcr_out ds;
    int64_t n_rec;
    int fast_ok;            // fast_allowed() (dcr_capi.hip): the fast kernel may take records
    int rpw;                // k_recmeta: records per wave (a power of two <= 64; fewer for deep records)
    int t16;                // decision margin in 1/16 nat (fast_constants)
    const uint32_t *wtab;   // [DCR_LUT_N] per LUT row: LLR term | -ln(p'/5) bound << 16 | not-a-call-row << 31
};

// the fast kernel's compact arguments (one strand; fewer scalar registers than Args)
struct FastArgs {
    const uint8_t *gb, *gq;         // staged bytes: input reads (single-strand) or single-strand consensus (duplex)
    int64_t nbytes;                 // length of gb / gq (buffer-load range check)
    const RecMeta *meta;            // fast list descriptors
    uint4 *rows;                    // per fast-list entry: decided scalars (Workspace::rows)
    const uint2 *rmeta;             // per-read words
    const int *fast_count;          // fast-list length
    dcr_read_info *info;            // single-strand: read info of the fast records' reads
    uint32_t *norm_cig;             // single-strand: runs of records handed to the general kernel
    const int32_t *cig_off;         // single-strand: batch cig_off
    int *ovf;                       // general list of this strand
    int *ovf_count;
    int *xlist;                     // exact queue (fast-list indices) and its length
    int *xcount;
    dcr_out O;                      // this strand's outputs
    const dcr_params *P;
    unsigned long long *stamps;     // diagnostic builds
    uint32_t kq;                    // bytes 255 - min_base_quality
    uint32_t kqlo;                  // bytes 0x80 - fast_qlo (lowest quality with 1-p' >= p'/5 upward)
    int maxq;
    int t16;                        // decision margin in 1/16 nat (dcr_capi.hip: fast_constants)
    int r_safe;                     // most reads for which no decided column's L_b can underflow
    int minbq;                      // single-strand: min_base_quality (masked rows in the table); duplex: -1
    int lo_check;                   // some unmasked quality may lie below fast_qlo: check the bytes
    const uint16_t *llr16;          // [123] per-quality LLR term, 1/16 nat, rounded down (EXACT's wide rows)
    const uint16_t *llr8;           // [123] the same in 1/u nat, u = 16, 8 or 4 (the common instantiation's narrow rows)
    const uint32_t *r2tab;          // [5 * 128 * 5 * 128] two-read column outcomes (k_r2_table), EXACT
    int t8;                         // decision margin in 1/u nat
    int narrow;                     // llr8 fits the narrow rows (else the common kernel queues every record)
    const double *e1000;            // [1001] k / 1000 correctly rounded (numpy round(x, 3) = rint(1000 x) / 1000)
    // record scalars (pos, mapq, len, n_cig, n_de, D, M, E lo, E hi, cigar):
    // the lowest of the ten arrays and each one's byte offset from it, when
    // every store lies within 4 GiB above it (else sbase = null: 64-bit addresses)
    uint8_t *sbase;
    uint32_t sofs[10];
    int want_info;                  // single-strand: write every read's dcr_read_info (DCR_OPT_READ_INFO)
    int direct_r;                   // single-strand records of at most this many reads go to the exact queue unstaged
};

template <bool DUPLEX> __global__ void k_recmeta(Args a);
__global__ void k_prep_big(Args a);
template <bool DUPLEX, bool EXACT> __global__ void k_consensus_fast(FastArgs a);
__global__ void k_fast_rows(FastArgs a);
__global__ void k_r2_table(const dcr_params *P, uint32_t *tab);
constexpr int kR2Entries = 5 * 128 * 5 * 128;
template <bool DUPLEX> __global__ void k_consensus_general(Args a);
template <bool DUPLEX> __global__ void k_decide(Args a);
template <bool DUPLEX> __global__ void k_ins_layout(Args a);
__global__ void k_decide_deep(Args a);

}  // namespace dcr
