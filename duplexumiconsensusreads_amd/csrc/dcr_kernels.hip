// dcr_kernels.hip — gfx950 (MI355X) kernels of the duplex-consensus hot path.
//
// Reference: /root/reference/DuplexUMIConsensusReads.py (":line" below).
//
//   k_recmeta    one lane per record: classifies it (fast list / general list /
//                status); prep_read (remove_clipping / mask / trim_3prime_N,
//                :191-325) for the reads of general records.
//   k_consensus_fast / _general
//                one wavefront per consensus record (single-strand: one
//                subfamily; duplex: one A1+B2 / B1+A2 pair).  Phases:
//                  0. stage the record's bases/quals from HBM into LDS as
//                     16-bit element codes (wide coalesced loads, one trip)
//                  1. column layout of reconstruct_alignment (:430-547)
//                  2. per-column likelihood products in read order + posterior,
//                     masking and output quality (:550-712)
//                  3. field layout: trims, CIGAR, seq/qual (:716-871),
//                     depth/errors and their pairwise mean (:970-1021), MAPQ
//                     (:874-889).
// All arithmetic is IEEE binary64 in the reference's operation order; build
// with -ffp-contract=off (no FMA contraction).  No transcendental runs on the
// device: p', thresholds and phred rounding boundaries are host tables.
//
// Likelihood "slots" (phase 2).  The reference keeps six products per column
// (:590-600).  Every class that has not yet appeared in the column receives
// the same factor p'/5 from every read, so all unseen classes hold the SAME
// double — one chain U.  A class seen for the first time at read r starts
// from U (its value so far, bit for bit) times (1 - p').  So a lane keeps U
// plus one chain per distinct class actually observed, and the wave pays only
// for the largest number of distinct classes among its 64 columns (usually
// one or two) instead of six.  Results are bit-identical to the six chains.
#include <type_traits>

#include "dcr_internal.h"

#ifndef DCR_STAMP
#define DCR_STAMP 0   // diagnostic builds only (tools/stamps.py): per-phase s_memtime cycle totals
#endif
#ifndef DCR_GSTAMP
#define DCR_GSTAMP 0  // diagnostic builds only (tools/gstamps.py): per-phase s_memtime cycles of the general kernel
#endif
#ifndef DCR_LAYHOIST
#define DCR_LAYHOIST 1  // k_ins_layout: a record of <= 64 reads builds its read table once
#endif
#ifndef DCR_LAYU
#define DCR_LAYU 2    // k_ins_layout: reads whose byte loads are in flight together (2: 5 waves per SIMD; 4: 4, slower)
#endif
#ifndef DCR_LAYCLAIM
#define DCR_LAYCLAIM 1  // k_ins_layout: records claimed one at a time past the first (0: fixed stride)
#endif
#ifndef DCR_LAYOCC
#define DCR_LAYOCC 1  // k_ins_layout: waves per SIMD its launch bounds ask for
#endif
#ifndef DCR_FAST_OCC
#define DCR_FAST_OCC 7   // fast kernel (common instantiation): waves per SIMD the launch bounds ask for
#endif
#ifndef DCR_EXACT_OCC
#define DCR_EXACT_OCC 4  // fast kernel (EXACT instantiation): waves per SIMD the launch bounds ask for
#endif
#ifndef DCR_TRIM2
#define DCR_TRIM2 1   // fast kernel: the 3' trim of C2-shaped records checked from the evidence counts
#endif
#ifndef DCR_ROWS
#define DCR_ROWS 1    // fast kernel: decided scalars as one 16-byte row per record, expanded by k_fast_rows
#endif
#ifndef DCR_DEFER
#define DCR_DEFER 1   // fast kernel: a record's row stored after the next record's staging (its vmcnt(0) does not wait
                      // for it; deferring the column stores too held registers across the loop and was slower)
#endif
#ifndef DCR_LCPOL
#define DCR_LCPOL 0   // fast kernel: cache policy of the staging loads (gfx950 aux bits: 2 = nt)
#endif
#ifndef DCR_SCPOL
#define DCR_SCPOL 0   // fast kernel: cache policy of the column stores
#endif
#ifndef DCR_VMPAD
#define DCR_VMPAD 0   // fast kernel: range-checked-out stores after the prefetch (see the record loop)
#endif
#ifndef DCR_STRIDE
#define DCR_STRIDE 1  // fast kernel: evenly spaced reads' codes addressed by a stepped VGPR (no per-read readlane)
#endif
#ifndef DCR_ST4
#define DCR_ST4 0     // fast kernel (common instantiation): column stores four columns per lane through the free stage
                      // (4 stores per record instead of 4 per tile: measured level, profiles/r06h)
#endif
#ifndef DCR_ABL
#define DCR_ABL 0   // diagnostic builds only (tools/ablate.py); fast kernel: 1 staging only, 2 +products,
                    // 4 always the exact pairwise mean, 5 no per-column stores, 6 every single-strand record
                    // staged from the fast list's first record's bytes (cache-resident: the kernel without its
                    // HBM reads), 7 column stores cache-resident (DCR_RSRC_*), 8 column stores at
                    // 64-column-aligned offsets (records overlap: timing only)
#endif

#define DCR_STR_(x) #x
#define DCR_STR(x) DCR_STR_(x)
namespace dcr {

constexpr int kStageElems = 2048;        // per-wave LDS staging (16-bit codes)
constexpr int kTileIns = 32;             // column tile of the insertion layout
constexpr int kFastMaxT = 240;           // pairwise_small: both halves <= 128
constexpr int kFastMaxR = 63;            // fast kernel: 6-bit class counters
constexpr int kColsLds = 256;            // per-wave LDS column scratch

// element code: bits 0..8 LUT row (quality 0..255, 256 '+', 257 '-'), bits 9..11 class
// class: 0 A, 1 T, 2 C, 3 G, 4 '+', 5 '-', 6 N/n, 7 invalid character (:580-591)
constexpr uint32_t kPad = (6u << 9) | 2u;          // 'N' with quality 2 (:509-510, :543-544)
constexpr uint32_t kPlus = (4u << 9) | DCR_LUT_PLUS;
constexpr uint32_t kDel = (5u << 9) | DCR_LUT_DEL;

struct WaveLds {
    uint16_t pad_code[4];                  // [0] = kPad: sentinel the fast layout loads outside a read (8 B keeps stage 8-aligned)
    uint16_t stage[kStageElems];           // element codes of the record's bytes (records that fit)
    uint16_t tile[kWave][kTileIns];        // insertion layout: 64 reads x 32 columns
    int32_t cons[kColsLds];
    double et[kColsLds];
    // uniform stack of the pairwise-sum walk (phase 3)
    int stk_off[24], stk_n[24], stk_stage[24];
    double stk_left[24];
};

// class of an input base (A/T/C/G/N; anything else is invalid, :580-585)
__device__ __forceinline__ uint32_t base_class(uint32_t b) {
    // 4-bit class per letter 'A'..'Z' packed in two 64-bit words; 7 = invalid
    constexpr uint64_t lo = 0x7777777777777777ull & ~(0xfull << 0) & ~(0xfull << 8) & ~(0xfull << 24)
                            & ~(0xfull << 52);
    // letters: A=0 ('A'-'A'=0), C=2, G=6, N=13, T=19
    const uint64_t tab_lo = (lo | (0ull << 0) | (2ull << 8) | (3ull << 24) | (6ull << 52));
    constexpr uint64_t tab_hi = (0x7777777777777777ull & ~(0xfull << 12)) | (1ull << 12);
    const uint32_t i = b - 'A';
    if (i >= 32u) return 7;
    const uint64_t t = i < 16 ? tab_lo : tab_hi;
    return (uint32_t)(t >> ((i & 15) * 4)) & 15u;
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// wave64 reductions on the VALU with DPP (quad_perm, half-row and row mirrors,
// row_bcast15/31; gfx9 encodings), result read from lane 63 into an SGPR —
// no LDS round trips (a ds_bpermute butterfly costs 6 dependent LDS latencies)
template <class F>
__device__ __forceinline__ int wave_reduce(int v, int ident, F op) {
    v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x140, 0xF, 0xF, false));  // row_mirror
    v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min(int v) {
    return wave_reduce(v, 0x7fffffff, [](int x, int y) { return min(x, y); });
}
__device__ __forceinline__ int wave_max(int v) {
    return wave_reduce(v, -0x7fffffff - 1, [](int x, int y) { return max(x, y); });
}
__device__ __forceinline__ int wave_sum(int v) {
    return wave_reduce(v, 0, [](int x, int y) { return x + y; });
}
__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// wave-local ordering of global/LDS traffic between phases of one wavefront
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// wave-local LDS ordering: a wave's DS instructions execute in order, so only
// the compiler must be kept from reordering (no vmcnt drain of prefetches)
__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ prep_read
// remove_clipping (:191-265): drop H; drop S with its bases (5'/3' ends);
// mask_low_quality_bases (:268-289): base -> 'N' if qual < min_base_quality
// (applied by the consumer); trim_3prime_N (:292-325): drop trailing 'N' and
// cut as many entries from the END of the expanded CIGAR.
__device__ __forceinline__ void prep_read(const dcr_batch &in, const dcr_params *P, const Workspace &ws, int64_t i) {
    const int minbq = P->min_base_quality;
    const uint32_t *cig = in.cigar + in.cig_off[i];
    const int n = in.cig_n[i];
    int sc5 = 0, sc3 = 0;
    bool inseq = false, modified = false;
    int64_t E = 0;
    for (int j = 0; j < n; ++j) {
        const uint32_t v = cig[j];
        const int op = v & 15, ln = v >> 4;
        if (op == 5) {
            modified = true;
        } else if (op == 4) {
            modified = true;
            if (!inseq) sc5 = ln; else sc3 = ln;
        } else {
            inseq = true;
            E += ln;
        }
    }
    int len = in.seq_len[i];
    int start = 0;
    if (modified) {
        start = sc5;
        len -= sc5 + sc3;
    }
    dcr_read_info inf;
    inf.seq_start = in.seq_off[i] + start;
    inf.len = 0;
    inf.n_cig = 0;
    inf.status = DCR_ST_OK;
    inf.has_ins = 0;
    if (len <= 0) {                      // empty sequence: enumerate(None) at :279
        inf.status = DCR_ST_TYPE_ERROR;
        ws.info[i] = inf;
        return;
    }
    const uint8_t *s = in.bases + inf.seq_start;
    const uint8_t *q = in.quals + inf.seq_start;
    int tl = len;
    while (tl > 0 && (s[tl - 1] == 'N' || (int)q[tl - 1] < minbq)) --tl;
    int64_t keep = E - (len - tl);
    if (keep <= 0) {                     // compress_cigarlist([]) at :740 via :322
        inf.status = DCR_ST_INDEX_ERROR;
        ws.info[i] = inf;
        return;
    }
    uint32_t *out = ws.norm_cig + in.cig_off[i];
    int nout = 0, last = -1, has_ins = 0;
    for (int j = 0; j < n && keep > 0; ++j) {
        const uint32_t v = cig[j];
        int op = v & 15;
        const int64_t ln = v >> 4;
        if (op == 4 || op == 5) continue;
        if (op == 7 || op == 8) op = 0;  // change_match_mismatch_operations (:361-377)
        const int64_t take = ln < keep ? ln : keep;
        keep -= take;
        if (take == 0) continue;
        has_ins |= (op == 1);
        if (op == last) out[nout - 1] += (uint32_t)take << 4;
        else out[nout++] = ((uint32_t)take << 4) | (uint32_t)op;
        last = op;
    }
    inf.len = tl;
    inf.n_cig = nout;
    inf.has_ins = has_ins;
    ws.info[i] = inf;
}

// Clip-only view of a read (remove_clipping :191-265 without the 3' N trim,
// which needs the bases): kept window and whether the read is one M-like run
// (=/X become M, :361-377) whose length matches the kept sequence.
struct ClipView {
    int64_t seq_start;
    int len;          // kept length before trim_3prime_N
    bool single_m;
};

__device__ __forceinline__ ClipView clip_view(const dcr_batch &in, int64_t i) {
    const uint32_t *cig = in.cigar + in.cig_off[i];
    const int n = in.cig_n[i];
    int sc5 = 0, sc3 = 0, nm = 0, other = 0;
    bool inseq = false, modified = false;
    int64_t E = 0;
    for (int j = 0; j < n; ++j) {
        const uint32_t v = cig[j];
        const int op = v & 15, ln = v >> 4;
        if (op == 5) {
            modified = true;
        } else if (op == 4) {
            modified = true;
            if (!inseq) sc5 = ln; else sc3 = ln;
        } else {
            inseq = true;
            E += ln;
            if (op == 0 || op == 7 || op == 8) ++nm; else ++other;
        }
    }
    ClipView cv;
    int len = in.seq_len[i];
    int start = 0;
    if (modified) {
        start = sc5;
        len -= sc5 + sc3;
    }
    cv.seq_start = in.seq_off[i] + start;
    cv.len = len;
    cv.single_m = other == 0 && nm > 0 && E == (int64_t)len;
    return cv;
}

// ------------------------------------------------------------ read access
struct ReadRef {
    int pos, len, ncig, mapq, status;
    const uint32_t *cig;
    const uint8_t *seq, *qual;
    int64_t seq_start;     // offset of the first kept base in its byte array
};

template <bool DUPLEX>
__device__ __forceinline__ ReadRef get_read(const Args &a, int64_t rec, int r) {
    ReadRef rd;
    if (!DUPLEX) {
        const int gr = a.in.sub_off[rec] + r;
        const dcr_read_info inf = a.ws.info[gr];
        rd.pos = a.in.read_pos[gr];
        rd.len = inf.len;
        rd.ncig = inf.n_cig;
        rd.mapq = a.in.read_mapq[gr];
        rd.status = inf.status;
        rd.cig = a.ws.norm_cig + a.in.cig_off[gr];
        rd.seq_start = inf.seq_start;
        rd.seq = a.in.bases + inf.seq_start;
        rd.qual = a.in.quals + inf.seq_start;
    } else {
        // pair p = 2f + j uses single-strand records 4f + 2j (+1)  (:1575-1576)
        const int64_t s = 2 * rec + r;
        const int64_t off = a.in.ss_col_off[s];
        rd.pos = a.ss.pos[s];
        rd.len = a.ss.len[s];
        rd.ncig = a.ss.n_cig[s];
        rd.mapq = a.ss.mapq[s];
        rd.status = a.ss.status[s];
        rd.cig = a.ss.cigar + off;
        rd.seq_start = off;
        rd.seq = a.ss.seq + off;
        rd.qual = a.ss.qual + off;
    }
    return rd;
}

// element code of a base with its quality; masking only for single-strand
// input reads (mask_low_quality_bases :280)
template <bool DUPLEX>
__device__ __forceinline__ uint32_t make_code(uint32_t b, uint32_t q, int minbq) {
    uint32_t cls = base_class(b);
    if (!DUPLEX && (int)q < minbq) cls = 6;
    return (cls << 9) | q;
}

template <bool DUPLEX>
__device__ __forceinline__ uint32_t base_elem(const ReadRef &rd, int is, int minbq) {
    return make_code<DUPLEX>(rd.seq[is], rd.qual[is], minbq);
}

// ------------------------------------------------ reconstruct_alignment state
// lane = read.  Mirrors idx_cigar / idx_seq (:465-466) with run-length CIGAR.
struct Sim {
    int k, o, is, curop, curlen;
    uint32_t nxt;         // run k + 1, loaded one transition ahead (0: none)
};

__device__ __forceinline__ void sim_set_run(Sim &s, const ReadRef &rd, uint32_t v) {
    if (s.k < rd.ncig) {
        s.curop = v & 15;
        s.curlen = v >> 4;
    } else {
        s.curop = -1;     // exhausted: get_current_CIGAR_operations reports 0 (:424-425)
        s.curlen = 0;
    }
    s.nxt = s.k + 1 < rd.ncig ? rd.cig[s.k + 1] : 0u;
}
__device__ __forceinline__ void sim_load_run(Sim &s, const ReadRef &rd) {
    sim_set_run(s, rd, s.k < rd.ncig ? rd.cig[s.k] : 0u);
}
// the next run comes from the register loaded at the previous transition, so a
// column step never waits on HBM for it
__device__ __forceinline__ void sim_advance(Sim &s, const ReadRef &rd) {
    if (++s.o == s.curlen) {
        ++s.k;
        s.o = 0;
        sim_set_run(s, rd, s.nxt);
    }
}

// one column of :473-545 for one read; returns the element code.  `elem(is)`
// gives the code of the read's base is (from HBM, or from the LDS stage)
template <bool DUPLEX, class Elem>
__device__ __forceinline__ uint32_t sim_step_e(Sim &s, const ReadRef &rd, int p, bool ins_col, bool &idx_err,
                                               const Elem &elem) {
    uint32_t e;
    if (ins_col) {                                   // :478-499
        if (s.curop == 1) {
            if (s.is >= rd.len) { idx_err = true; return kPad; }
            e = elem(s.is);
            ++s.is;
            sim_advance(s, rd);
        } else {
            e = kPlus;
        }
    } else if (p < rd.pos) {                         // :506-510
        e = kPad;
    } else if (s.is < rd.len) {                      // :514-535
        if (s.curop < 0) { idx_err = true; return kPad; }
        if (s.curop == 2) {
            e = kDel;
        } else {
            e = elem(s.is);
            ++s.is;
        }
        sim_advance(s, rd);
    } else {                                         // :540-544
        e = kPad;
    }
    return e;
}
template <bool DUPLEX>
__device__ __forceinline__ uint32_t sim_step(Sim &s, const ReadRef &rd, int p, bool ins_col,
                                             int minbq, bool &idx_err) {
    return sim_step_e<DUPLEX>(s, rd, p, ins_col, idx_err,
                              [&](int is) { return base_elem<DUPLEX>(rd, is, minbq); });
}

// position of op index j of a read without I ops: (op, seq index), or pad.
// The seq index is the number of M ops before j; once it reaches len the
// read pads for good (:514, :540).
__device__ __forceinline__ bool walk_runs(const uint32_t *cig, int ncig, int j, int len, int &is, bool &del) {
    int acc = 0, accis = 0;
    int op = -1;
    is = 0;
    for (int k = 0; k < ncig; ++k) {
        const uint32_t v = cig[k];
        const int ln = v >> 4, o = v & 15;
        if (op < 0 && j < acc + ln) {
            op = o;
            is = accis + (o == 0 ? j - acc : 0);
        }
        acc += ln;
        if (o == 0) accis += ln;
    }
    if (op < 0 || is >= len) return false;
    del = op == 2;
    return true;
}

// ------------------------------------------ insertion layout by events
// (k_ins_layout; tests/fil_model.py is its host model, checked against the
// oracle's column-by-column reconstruct_alignment, :430-547).  A column is an
// insertion column when a read's current op is I (:476-478): only reads that
// hold an I run make one, and between insertion blocks every started read
// advances one op per column (:506-535).  So the blocks follow from each I
// read's run start counted in normal columns (phase A, event by event: reads
// whose runs start at the same column make one block, as long as its longest
// run), and a read's element at column t from N(t), the normal columns before
// t: op index N(t) - N(s_r) (+ its I run once past), then the op and the read's
// bases before it (phase B, lane = column).

// the op at expanded index j of a read's runs (<= 4; I and M consume bases,
// D not) and the read's bases before it (all its bases past the last op)
struct RunPos {
    int op, is;
};
__device__ __forceinline__ RunPos run_at(const uint32_t (&v)[4], int ncig, int j) {
    int acc = 0, accb = 0, op = -1, is = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ln = k < ncig ? (int)(v[k] >> 4) : 0;
        const int o = (int)(v[k] & 15u);
        const bool here = op < 0 && j < acc + ln;
        const bool cb = o != 2;
        is = here ? accb + (cb ? j - acc : 0) : is;
        op = here ? o : op;
        acc += ln;
        accb += cb ? ln : 0;
    }
    return RunPos{op, op < 0 ? accb : is};
}

// insertion columns below column s of a record's mask (T <= 256)
__device__ __forceinline__ int ins_below(const uint64_t (&im)[4], int s) {
    int n = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int nb = min(max(s - 64 * w, 0), 64);
        const uint64_t m = nb == 64 ? im[w] : (im[w] & ((1ull << nb) - 1ull));
        n += __popcll(m);
    }
    return n;
}

// --------------------------------------------------------------- phase 2
// Likelihood slots (see header): U = the chain shared by all unseen classes,
// s[j] = chain of the j-th distinct class seen in the column, k[j] its class,
// n[j] its row count.
struct Acc {
    double U;
    double s[6];
    int k[6];
    int n[6];
    int ns;                    // slots used by this lane
    int nbad;                  // rows with an invalid character
};

__device__ __forceinline__ void acc_init(Acc &A) {
    A.U = 1.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        A.s[j] = 1.0;
        A.k[j] = -1;
        A.n[j] = 0;
    }
    A.ns = 0;
    A.nbad = 0;
}

// first sighting of class cls in this lane's column: L_cls == U until now
__device__ __forceinline__ void acc_new_class(Acc &A, bool isnew, uint32_t cls, double Uold, double fmatch) {
    if (!isnew) return;
    if (cls == 7) {
        A.nbad += 1;
        return;
    }
    const double v = Uold * fmatch;
    const int j = A.ns;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        if (i == j) {
            A.s[i] = v;
            A.k[i] = (int)cls;
            A.n[i] = 1;
        }
    }
    A.ns = j + 1;
}

// one read's factors for all six classes (:594-600) with NS live slots;
// returns true when some lane now needs more than NS slots
template <int NS>
__device__ __forceinline__ bool acc_step(Acc &A, uint32_t e, double2 f) {
    const uint32_t cls = e >> 9;
    const double Uold = A.U;
    A.U = Uold * f.y;
    bool match = false;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const bool m = cls == (uint32_t)A.k[j];
        A.s[j] *= m ? f.x : f.y;
        A.n[j] += m;
        match |= m;
    }
    const bool isnew = cls != 6 && !match;
    if (__ballot(isnew)) {
        acc_new_class(A, isnew, cls, Uold, f.x);
        return __ballot(A.ns > NS) != 0;
    }
    return false;
}

// most_likely_nucleotide over reads 0..R-1 in read order.  Two live slots
// cover the usual column (one true base plus one error class); a wave that
// meets a third distinct class switches to six slots for the rest of the tile.
// Element codes and LUT factors are fetched four reads ahead of their use.
template <class Src>
__device__ __forceinline__ void accumulate(Acc &A, int R, const Src &src, const double2 *lut) {
    // a later 64-read chunk of the same columns continues the slots: start wide
    // when some lane already holds more than two (else a third class would be
    // matched against slots 0-1 only and opened a second time)
    bool wide = __ballot(A.ns > 2) != 0;
    int r = 0;
    auto step = [&](uint32_t e, double2 f) {
        if (!wide) wide = acc_step<2>(A, e, f);
        else (void)acc_step<6>(A, e, f);
    };
    for (; r + 4 <= R; r += 4) {
        const uint32_t e0 = src(r), e1 = src(r + 1), e2 = src(r + 2), e3 = src(r + 3);
        const double2 f0 = lut[e0 & 511], f1 = lut[e1 & 511], f2 = lut[e2 & 511], f3 = lut[e3 & 511];
        step(e0, f0);
        step(e1, f1);
        step(e2, f2);
        step(e3, f3);
    }
    for (; r < R; ++r) {
        const uint32_t e = src(r);
        step(e, lut[e & 511]);
    }
}

struct ColOut {
    int ch, q, d, e;
    bool overflow;
};

// consensus quality Q for error x > 0 finite: the exact table boundaries
// (params.py) decide; a float log10 only proposes the candidate.
// Q = lo - 1 with lo = first i with qthr[i] <= x (lo = maxQ + 1 if none).
__device__ __forceinline__ int phred_from_table(double x, int maxq, const double *qthr) {
    const float lf = __builtin_amdgcn_logf((float)x);          // log2
    float qe = rintf(-3.01029995663981198f * lf);               // -10 log10 x
    qe = fminf(fmaxf(qe, -1.0f), (float)maxq);
    int q = (int)qe;
    bool ok_lo = q == maxq || qthr[q + 1] <= x;
    bool ok_hi = q < 0 || qthr[q] > x;
    if (__builtin_expect(!(ok_lo && ok_hi), 0)) {
        int lo = 0, hi = maxq + 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (qthr[mid] <= x) hi = mid; else lo = mid + 1;
        }
        q = lo - 1;
    }
    return q;
}

// posterior, mask and output quality of one column from its six likelihoods
// (:603-621, :699-709): S summed left to right (:608), np.argmax (first max,
// first NaN wins) and np.max, masking below the threshold (NaN never), then
// Q = int(round(-10 log10(e'))) capped at maxQ (ValueError -> maxQ).
struct Posterior {
    int best;        // argmax class index (A T C G + -)
    int ch;          // consensus character
    int q;           // consensus quality
    bool masked;
    bool overflow;   // int(-inf): the reference raises OverflowError
};

__device__ __forceinline__ Posterior posterior(const double (&L)[6], bool has_plus, const dcr_params *P,
                                               const double *qthr, bool simple_q) {
    Posterior o;
    double S = L[0] + L[1];                      // np.sum of 6: left to right (:608)
    S = S + L[2];
    S = S + L[3];
    S = S + L[4];
    S = S + L[5];
    // np.argmax of L[i]/S (first max, first NaN wins) and np.max (:613-614)
    int best = 0;
    double pm;
    const double Lmin = fmin(fmin(fmin(L[0], L[1]), fmin(L[2], L[3])), fmin(L[4], L[5]));
    if (S > 0.0 && S <= 1.79769313486231570815e308 && Lmin >= 0.0) {
        // division by S > 0 is monotone: the first largest L gives the max
        // posterior, unless an earlier class's quotient rounds to the same
        // double (only possible within a few ulps: checked exactly, rarely)
        double Lb = L[0];
#pragma unroll
        for (int i = 1; i < 6; ++i) {
            const bool g = L[i] > Lb;
            best = g ? i : best;
            Lb = g ? L[i] : Lb;
        }
        pm = Lb / S;
        const double near = Lb * 0.99999999999999;
        bool tie = false;
#pragma unroll
        for (int i = 0; i < 5; ++i) tie |= (i < best) && (L[i] >= near);
        if (__builtin_expect(tie, 0)) {
#pragma unroll
            for (int i = 4; i >= 0; --i)
                if (i < best && L[i] >= near && L[i] / S == pm) best = i;
        }
    } else {
        double p[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) p[i] = L[i] / S;
        pm = p[0];
        bool nan = __builtin_isnan(p[0]);
#pragma unroll
        for (int i = 1; i < 6; ++i) {
            if (!nan) {
                if (__builtin_isnan(p[i])) {
                    nan = true;
                    best = i;
                    pm = p[i];
                } else if (p[i] > pm) {
                    best = i;
                    pm = p[i];
                }
            }
        }
    }
    const bool masked = pm < P->post_threshold;  // NaN is never masked (:617)
    const int kc = masked ? 6 : best;
    const bool lower = has_plus && (kc < 4 || kc == 6);
    int ch;
    if (masked) ch = has_plus ? 'n' : 'N';
    else ch = (int)((0x2D2B47435441ull >> (8 * best)) & 0xffu) + (lower ? 32 : 0);   // "ATCG+-"
    // consensus quality (:700-709)
    const double e = 1.0 - pm;
    double x;
    if (simple_q) {
        x = e;                                   // pre = post = 0: the formula reduces to e exactly
    } else {
        const double pre = (double)P->error_rate_pre_labeling;
        const double post = (double)P->error_rate_post_labeling;
        x = pre * (1.0 - e) + (1.0 - post) * e + pre * e * 4.0 / 5.0;
    }
    int q = P->max_base_quality;
    o.overflow = false;
    if (x > 0.0) {                               // else the ValueError branch: max quality
        if (__builtin_isinf(x)) o.overflow = true;
        else q = phred_from_table(x, P->max_base_quality, qthr);
    }
    o.best = best;
    o.ch = ch;
    o.q = q;
    o.masked = masked;
    return o;
}

// posterior, mask, output quality (:603-621, :699-709), depth/errors (:1001-1012)
__device__ __forceinline__ ColOut finalize(const Acc &A, int nsw, int R, bool ins_col, const dcr_params *P,
                                           const double *qthr, bool simple_q) {
    double L[6];
    int c[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        L[i] = A.U;
        c[i] = 0;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        if (j < nsw) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const bool m = A.k[j] == i;
                L[i] = m ? A.s[j] : L[i];
                c[i] = m ? A.n[j] : c[i];
            }
        }
    }
    const int cN = R - c[0] - c[1] - c[2] - c[3] - c[4] - c[5] - A.nbad;
    ColOut o;
    const bool has_plus = c[4] > 0;              // '+' in nucleotides (:613, :618)
    const Posterior po = posterior(L, has_plus, P, qthr, simple_q);
    const int kc = po.masked ? 6 : po.best;
    const bool lower = has_plus && (kc < 4 || kc == 6);
    const int ch = po.ch;
    const int q = po.q;
    o.overflow = po.overflow;
    o.ch = ch;
    o.q = q;
    // depth: rows not in {N, n, +}; errors: rows != consensus char (case-sensitive)
    o.d = R - cN - c[4];
    int cnt = cN;
#pragma unroll
    for (int i = 0; i < 6; ++i) cnt = kc == i ? c[i] : cnt;
    // row characters: insertion columns hold lowercase bases / 'n' / '+',
    // normal columns uppercase bases / 'N' / '-'
    int match;
    if (kc == 4) match = cnt;
    else if (kc == 5) match = ins_col ? 0 : cnt;
    else match = (lower == ins_col) ? cnt : 0;
    o.e = R - match;
    return o;
}

// ------------------------------------------------- decision pass (general)
// The fast kernel's integer decision (see k_consensus_fast below), for the
// general kernel's records without insertion columns: any number of reads,
// reads of one M run or of M D M runs ('-' rows), T <= 256.  Per column:
// 32-bit sums of the rounded-down LLR terms of A T C G '-', row counts and
// Z = the rounded-up sum of -ln(p'/5) over every row.  A column is decided
// when L_b - L_2nd - n_other >= T16 (the call is b with quality maxQ, unmasked)
// and Z - L_b <= 16 * 700: ln L_b = LLR_b - sum(-ln(p'/5)) >= -700, so the
// reference's product L_b stays a normal double (no underflow to a NaN
// posterior, :603-618).
//
// The sums are order-free, so reads are visited in staging order: the bytes of
// the record's reads (contiguous in HBM) go through the wave's LDS stage as
// element codes, 2 KiB per round trip (dword loads, 16 per lane), and every
// read in the stage adds its row to all NT column tiles (lane = column).
// Writes kb | d << 3 | e << 15 per column into `cw` and returns true when every
// column is decided; false (the caller then runs the reference's double
// arithmetic) on any undecided column, an invalid letter, a row quality the
// bound does not cover, or another read layout.
struct DecideAcc {
    uint32_t s[5];          // LLR sums A T C G '-'
    uint32_t n[6];          // rows A T C G '-' N
    uint32_t z;
};

template <int NT>
__device__ __forceinline__ void decide_zero(DecideAcc (&A)[NT]) {
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
#pragma unroll
        for (int k = 0; k < 5; ++k) A[tt].s[k] = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) A[tt].n[k] = 0;
        A[tt].z = 0;
    }
}

// the rows of reads [r0, r1) of the record added into A (lane = column of
// each tile); false on an invalid letter, a row quality the bound does not
// cover, or a read layout other than M / M D M

template <bool DUPLEX, int NT>
__device__ bool decide_accumulate(const Args &a, const int64_t rec, const int r0, const int r1, const int T,
                                  const int minpos, uint16_t *stage, const uint32_t *s_wtab, const int lane,
                                  DecideAcc (&A)[NT]) {
    const int minbq = a.P->min_base_quality;
    const uint8_t *gb = DUPLEX ? a.ss.seq : a.in.bases;
    const uint8_t *gq = DUPLEX ? a.ss.qual : a.in.quals;
    bool bad = false;
    for (int cb = r0; cb < r1; cb += kWave) {
        // lane r: read cb + r -- first column, kept length, first byte, and
        // the runs M a1, D b1 (a1 = len, b1 = 0 for one M run)
        int col = 0, len = 0, a1 = 0, b1 = 0;
        int64_t ss = 0;
        bool other = false;
        const int nr = min(kWave, r1 - cb);
        if (lane < nr) {
            const ReadRef rd = get_read<DUPLEX>(a, rec, cb + lane);
            col = rd.pos - minpos;
            len = rd.len;
            ss = rd.seq_start;
            a1 = len;
            if (rd.ncig == 3) {
                const uint32_t c0 = rd.cig[0], c1 = rd.cig[1], c2 = rd.cig[2];
                other = (c0 & 15u) != 0 || (c1 & 15u) != 2 || (c2 & 15u) != 0;
                a1 = (int)(c0 >> 4);
                b1 = (int)(c1 >> 4);
            } else {
                other = rd.ncig != 1 || (rd.cig[0] & 15u) != 0;
            }
            other |= len > kStageElems - 4;
        }
        if (__ballot(other)) return false;
        int rr = 0;                                   // reads of this chunk done
        while (rr < nr) {
            // stage [base, base + 2 KiB): the reads rr.. that end inside it
            const int64_t base = (int64_t)(((uint64_t)(uint32_t)readlane((int)((uint64_t)ss >> 32), rr) << 32) |
                                           (uint32_t)readlane((int)(uint32_t)ss, rr)) & ~(int64_t)3;
            const bool in = lane >= rr && lane < nr && ss + len - base <= kStageElems;
            const uint64_t fm = ~__ballot(in) >> rr;      // first read past the stage
            const int nfit = fm ? min((int)__builtin_ctzll(fm), nr - rr) : nr - rr;
            const int rlast = rr + nfit - 1;
            const int64_t ssl = (int64_t)(((uint64_t)(uint32_t)readlane((int)((uint64_t)ss >> 32), rlast) << 32) |
                                          (uint32_t)readlane((int)(uint32_t)ss, rlast));
            const int span = (int)(ssl + readlane(len, rlast) - base);
            const int nd = (span + 3) >> 2;
            const uint32_t *b4 = (const uint32_t *)(gb + base);
            const uint32_t *q4 = (const uint32_t *)(gq + base);
            uint32_t vb[kStageElems / 4 / kWave], vq[kStageElems / 4 / kWave];
#pragma unroll
            for (int u = 0; u < kStageElems / 4 / kWave; ++u) {
                const int d = u * kWave + lane;
                vb[u] = d < nd ? b4[d] : 0u;
                vq[u] = d < nd ? q4[d] : 0u;
            }
            wave_fence();                             // the previous stage's readers are done
#pragma unroll
            for (int u = 0; u < kStageElems / 4 / kWave; ++u) {
                const int d = u * kWave + lane;
                if (d < nd) {
                    uint32_t cc[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        cc[k] = make_code<DUPLEX>((vb[u] >> (8 * k)) & 255u, (vq[u] >> (8 * k)) & 255u, minbq);
                    *(uint2 *)&stage[4 * d] = make_uint2(cc[0] | (cc[1] << 16), cc[2] | (cc[3] << 16));
                }
            }
            wave_fence();
            for (int r = rr; r <= rlast; ++r) {
                const int cr = readlane(col, r), lr = readlane(len, r);
                const int ar = readlane(a1, r), br = readlane(b1, r);
                const int so = (int)((int64_t)(((uint64_t)(uint32_t)readlane((int)((uint64_t)ss >> 32), r) << 32) |
                                               (uint32_t)readlane((int)(uint32_t)ss, r)) - base);
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    const int t = 64 * tt + lane;
                    const int j = t - cr;
                    const bool del = j >= ar && j < ar + br;
                    const int is = j < ar ? j : j - br;
                    uint32_t e;
                    if (t >= T || j < 0 || (del ? ar : is) >= lr) e = kPad;   // is >= len: pad (:514, :540)
                    else e = del ? kDel : (uint32_t)stage[so + is];
                    const uint32_t cls = e >> 9;
                    const uint32_t w = s_wtab[e & 511u];
                    bad |= cls == 7 || (cls != 6 && (w >> 31) != 0);
                    const uint32_t l = w & 0xFFFFu;
                    A[tt].s[0] += cls == 0 ? l : 0u;
                    A[tt].s[1] += cls == 1 ? l : 0u;
                    A[tt].s[2] += cls == 2 ? l : 0u;
                    A[tt].s[3] += cls == 3 ? l : 0u;
                    A[tt].s[4] += cls == 5 ? l : 0u;
                    A[tt].z += (w >> 16) & 0x7FFFu;
                    A[tt].n[0] += cls == 0;
                    A[tt].n[1] += cls == 1;
                    A[tt].n[2] += cls == 2;
                    A[tt].n[3] += cls == 3;
                    A[tt].n[4] += cls == 5;
                    A[tt].n[5] += cls == 6;
                }
            }
            if (__ballot(bad)) return false;
            rr += nfit;
        }
    }
    return true;
}

// the decision from the sums of all R rows: column words kb | d << 3 | e << 15
// into cw; true when every column is decided
template <int NT>
__device__ bool decide_columns(const Args &a, const int R, const int T, const DecideAcc (&A)[NT], int32_t *cw,
                               const int lane) {
    bool undecided = false;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        const int t = 64 * tt + lane;
        const uint32_t S[5] = {A[tt].s[0], A[tt].s[1], A[tt].s[2], A[tt].s[3], A[tt].s[4]};
        const uint32_t N[6] = {A[tt].n[0], A[tt].n[1], A[tt].n[2], A[tt].n[3], A[tt].n[4], A[tt].n[5]};
        // the first largest in the reference's order A T C G + - ('+' absent: 0)
        uint32_t Lb = S[0], kb = 0, nb = N[0];
        if (S[1] > Lb) { Lb = S[1]; kb = 1; nb = N[1]; }
        if (S[2] > Lb) { Lb = S[2]; kb = 2; nb = N[2]; }
        if (S[3] > Lb) { Lb = S[3]; kb = 3; nb = N[3]; }
        if (S[4] > Lb) { Lb = S[4]; kb = 5; nb = N[4]; }
        uint32_t L2 = 0;
        L2 = max(L2, kb != 0 ? S[0] : 0u);
        L2 = max(L2, kb != 1 ? S[1] : 0u);
        L2 = max(L2, kb != 2 ? S[2] : 0u);
        L2 = max(L2, kb != 3 ? S[3] : 0u);
        L2 = max(L2, kb != 5 ? S[4] : 0u);
        const int d = R - (int)N[5];                     // rows not 'N' ('-' counts, :1001)
        const int e = R - (int)nb;                       // rows != the call (:1011)
        const bool ok = (int)(Lb - L2) - (d - (int)nb) >= a.t16 && (int)A[tt].z - (int)Lb <= 16 * 700;
        if (t < T) {
            undecided |= !ok;
            cw[t] = (int32_t)(kb | ((uint32_t)d << 3) | ((uint32_t)e << 15));
        }
    }
    return __ballot(undecided) == 0;
}

template <bool DUPLEX, int NT>
__device__ bool decide_tiles(const Args &a, const int64_t rec, const int R, const int T, const int minpos,
                             int32_t *cw, uint16_t *stage, const uint32_t *s_wtab, const int lane) {
    DecideAcc A[NT];
    decide_zero<NT>(A);
    if (!decide_accumulate<DUPLEX, NT>(a, rec, 0, R, T, minpos, stage, s_wtab, lane, A)) return false;
    return decide_columns<NT>(a, R, T, A, cw, lane);
}

template <bool DUPLEX>
__device__ bool decide_record(const Args &a, const int64_t rec, const int R, const int T, const int minpos,
                              int32_t *cw, uint16_t *stage, const uint32_t *s_wtab, const int lane) {
    const uint8_t *gb = DUPLEX ? a.ss.seq : a.in.bases;
    const uint8_t *gq = DUPLEX ? a.ss.qual : a.in.quals;
    if (a.t16 < 0 || R > 4095 || T > 256 || T <= 0 || ((((uintptr_t)gb) | ((uintptr_t)gq)) & 3) != 0) return false;
    if (T <= 64) return decide_tiles<DUPLEX, 1>(a, rec, R, T, minpos, cw, stage, s_wtab, lane);
    if (T <= 128) return decide_tiles<DUPLEX, 2>(a, rec, R, T, minpos, cw, stage, s_wtab, lane);
    if (T <= 192) return decide_tiles<DUPLEX, 3>(a, rec, R, T, minpos, cw, stage, s_wtab, lane);
    return decide_tiles<DUPLEX, 4>(a, rec, R, T, minpos, cw, stage, s_wtab, lane);
}

// ------------------------------------------------ k_decide_deep's row table
// The staged codes are byte offsets of 32-byte rows of `tab` that hold an
// element's increments, packed: the LLR terms of A T C G in 16-bit fields
// (P0); the '-' term (16 bits), the six row counts and a bad-row count (6-bit
// fields) (P1); z.  A row is one ds_read_b128 plus one ds_read_b32 and three
// adds instead of a dozen compares and conditional adds; the packed sums are
// widened every 62 rows (no field overflows: 62 x 1040 < 2^16, 62 < 2^6).
// Rows (class, quality): A T C G N (0..4) x qualities 0..127 at 5 q + class,
// so the five classes of one quality sit in five different LDS bank groups
// (lanes = columns of one read read rows of one quality and mixed letters);
// the single-strand mask (:280) is folded in (rows of a quality below
// min_base_quality are 'N' rows); then '-' and the invalid-input row.
// Qualities >= 128 and invalid letters give up the record (general kernel).
constexpr uint32_t kTabDel = 5u * 128u * 32u;              // '-' (LUT row 257)
constexpr uint32_t kTabBad = kTabDel + 32u;                // unused by the codes; kept for completeness
constexpr uint32_t kTabZero = kTabBad + 32u;               // no row (the missing partner of an odd read)
constexpr uint32_t kTabPad = (5u * 2u + 4u) * 32u;         // 'N', quality 2 (:509-510, :543-544)
constexpr int kTabBytes = (int)kTabZero + 32;

// row i of the table; wtab: the LUT rows of the decision pass (dcr_capi.hip wide_table)
__device__ __forceinline__ void deep_tab_row(uint8_t *tab, int i, const uint32_t *wtab, int minbq) {
    uint32_t cls, row;
    if (i < 5 * 128) {
        cls = (uint32_t)i % 5u;
        row = (uint32_t)i / 5u;
        if (cls == 4 || (int)row < minbq) cls = 6;             // 'N' (sequenced or masked)
    } else if (i == (int)(kTabDel / 32u)) { cls = 5; row = DCR_LUT_DEL; }
    else if (i == (int)(kTabBad / 32u)) { cls = 7; row = 0; }
    else {
        *(uint4 *)(tab + 32 * i) = make_uint4(0u, 0u, 0u, 0u);
        *(uint4 *)(tab + 32 * i + 16) = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    const uint32_t w = wtab[row];
    const uint32_t l = w & 0xFFFFu;
    const uint32_t bad = cls == 7 || (cls != 6 && (w >> 31) != 0);
    const uint64_t p0 = cls < 4 ? (uint64_t)l << (16 * cls) : 0ull;
    const int k = cls < 4 ? (int)cls : (cls == 5 ? 4 : 5);
    const uint64_t p1 = (cls == 5 ? (uint64_t)l : 0ull) | (cls == 7 ? 0ull : 1ull << (16 + 6 * k)) |
                        ((uint64_t)bad << 52);
    *(uint4 *)(tab + 32 * i) = make_uint4((uint32_t)p0, (uint32_t)(p0 >> 32), (uint32_t)p1, (uint32_t)(p1 >> 32));
    *(uint4 *)(tab + 32 * i + 16) = make_uint4((w >> 16) & 0x7FFFu, 0u, 0u, 0u);
}

// four row offsets from four bases and qualities (SWAR): the class from a
// byte permute of (b >> 1) & 7 (A 0, C 2, T 1, G 3, N 4), whose letter a
// second permute checks (:580-585); `bad` collects the bits of an invalid
// letter or a quality >= 128 in the bytes `keep` selects (their codes are
// then don't-care)
__device__ __forceinline__ uint2 tab_codes4(uint32_t B, uint32_t Q, uint32_t keep, uint32_t &bad) {
    const uint32_t h = (B >> 1) & 0x07070707u;
    const uint32_t cls = __builtin_amdgcn_perm(0x04000000u, 0x03010200u, h);
    bad |= ((B ^ __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, h)) | (Q & 0x80808080u)) & keep;
    // per 16-bit field (5 q + class) * 32; no field carries into the next (q < 128)
    const uint32_t qlo = __builtin_amdgcn_perm(0u, Q, 0x04010400u), qhi = __builtin_amdgcn_perm(0u, Q, 0x04030402u);
    const uint32_t clo = __builtin_amdgcn_perm(0u, cls, 0x04010400u), chi = __builtin_amdgcn_perm(0u, cls, 0x04030402u);
    return make_uint2(__umul24(qlo & 0x007F007Fu, 160u) + (clo << 5), __umul24(qhi & 0x007F007Fu, 160u) + (chi << 5));
}

// decide_accumulate for k_decide_deep (single-strand): the rows of reads
// [r0, r1) through the table, widened into the block's LDS sums `acc`
// (12 x 256 words: s[5], n[6], z per column) with ds_add_u32.
// - staging: range-checked buffer loads based at the stage's first byte (no
//   exec-masked loads to zero-fill), the next stage's bytes loaded before the
//   current stage's rows are added;
// - rows two reads at a time: both reads' codes, then their table rows, then
//   the adds (64-bit adds of the packed sums), so LDS latencies overlap;
//   reads without a deletion (the common case) take a short address path.
template <int NT>
__device__ bool decide_accumulate_tab(const Args &a, const int64_t rec, const int r0, const int r1, const int T,
                                      const int minpos, uint16_t *stage, const uint8_t *tab, uint32_t *acc,
                                      const int lane) {
    constexpr int kU = kStageElems / 4 / kWave;
    uint64_t P0[NT], P1[NT];
    uint32_t Z[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        P0[tt] = P1[tt] = 0;
        Z[tt] = 0;
    }
    int prow = 0;
    uint32_t bad = 0;
    auto widen = [&]() {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            uint32_t *c = acc + 64 * tt + lane;
#pragma unroll
            for (int k = 0; k < 4; ++k) atomicAdd(c + 256 * k, (uint32_t)(P0[tt] >> (16 * k)) & 0xFFFFu);
            atomicAdd(c + 256 * 4, (uint32_t)P1[tt] & 0xFFFFu);
#pragma unroll
            for (int k = 0; k < 6; ++k) atomicAdd(c + 256 * (5 + k), (uint32_t)(P1[tt] >> (16 + 6 * k)) & 63u);
            atomicAdd(c + 256 * 11, Z[tt]);
            bad |= (uint32_t)(P1[tt] >> 52);
            P0[tt] = 0;
            P1[tt] = 0;
            Z[tt] = 0;
        }
        prow = 0;
    };
    for (int cb = r0; cb < r1; cb += kWave) {
        // lane r: read cb + r -- first column, kept length, first byte, runs M a1, D b1
        int col = 0, len = 0, a1 = 0, b1 = 0;
        int64_t ss = 0;
        bool other = false;
        const int nr = min(kWave, r1 - cb);
        if (lane < nr) {
            const ReadRef rd = get_read<false>(a, rec, cb + lane);
            col = rd.pos - minpos;
            len = rd.len;
            ss = rd.seq_start;
            a1 = len;
            if (rd.ncig == 3) {
                const uint32_t c0 = rd.cig[0], c1 = rd.cig[1], c2 = rd.cig[2];
                other = (c0 & 15u) != 0 || (c1 & 15u) != 2 || (c2 & 15u) != 0;
                a1 = (int)(c0 >> 4);
                b1 = (int)(c1 >> 4);
            } else {
                other = rd.ncig != 1 || (rd.cig[0] & 15u) != 0;
            }
            other |= len > kStageElems - 4;
        }
        if (__ballot(other)) return false;
        // bytes are addressed from the chunk's first read (a chunk spans < 2^31 bytes)
        const int64_t s0 = (int64_t)(((uint64_t)(uint32_t)readlane((int)((uint64_t)ss >> 32), 0) << 32) |
                                     (uint32_t)readlane((int)(uint32_t)ss, 0)) & ~(int64_t)3;
        const int rel = (int)(ss - s0);              // the lane's read: first byte from s0
        const int u = rel - col;                      // stage offset of its column 0 + the stage's base
        // one stage: the reads rr.. that end inside [base, base + 2 KiB)
        struct Plan { int base, rr, nfit, span; };
        auto plan = [&](int rr) {
            Plan p;
            p.rr = rr;
            p.base = readlane(rel, rr) & ~3;
            const bool in = lane >= rr && lane < nr && rel + len - p.base <= kStageElems;
            const uint64_t fm = ~__ballot(in) >> rr;
            p.nfit = fm ? min((int)__builtin_ctzll(fm), nr - rr) : nr - rr;
            const int rlast = rr + p.nfit - 1;
            p.span = readlane(rel, rlast) + readlane(len, rlast) - p.base;
            return p;
        };
        uint32_t vb[kU], vq[kU];
        auto load = [&](const Plan &p) {
            const int nbytes = (p.span + 3) & ~3;
            const __amdgpu_buffer_rsrc_t rb =
                __builtin_amdgcn_make_buffer_rsrc((void *)(a.in.bases + s0 + p.base), (short)0, nbytes, 0x00020000);
            const __amdgpu_buffer_rsrc_t rq =
                __builtin_amdgcn_make_buffer_rsrc((void *)(a.in.quals + s0 + p.base), (short)0, nbytes, 0x00020000);
#pragma unroll
            for (int k = 0; k < kU; ++k) {
                vb[k] = __builtin_amdgcn_raw_buffer_load_b32(rb, 4 * lane + 256 * k, 0, 0);
                vq[k] = __builtin_amdgcn_raw_buffer_load_b32(rq, 4 * lane + 256 * k, 0, 0);
            }
        };
        Plan cur = plan(0);
        load(cur);
        for (;;) {
            wave_fence();                             // the previous stage's readers are done
            const int nd = (cur.span + 3) >> 2;
#pragma unroll
            for (int k = 0; k < kU; ++k) {
                const int d = k * kWave + lane;
                if (k * kWave < nd) {                 // wave-uniform
                    const int nb = cur.span - 4 * d;  // bytes of the span in this dword
                    const uint32_t keep = nb >= 4 ? 0xFFFFFFFFu : (nb > 0 ? (1u << (8 * nb)) - 1u : 0u);
                    *(uint2 *)&stage[4 * d] = tab_codes4(vb[k], vq[k], keep, bad);
                }
            }
            wave_fence();
            const int rend = cur.rr + cur.nfit;
            Plan nxt = cur;
            if (rend < nr) {                          // the next stage's bytes in flight meanwhile
                nxt = plan(rend);
                load(nxt);
            }
            // stage index of read r's element in column t: su(r) + t
            auto su = [&](int r) { return readlane(u, r) - cur.base; };
            for (int r = cur.rr; r < rend; r += 2) {
                const bool two = r + 1 < rend;
                const int rb = two ? r + 1 : r;
                const int br0 = readlane(b1, r), br1 = two ? readlane(b1, rb) : 0;
                uint32_t e0[NT], e1[NT];
                if ((br0 | br1) == 0) {
                    // one M run each: column t holds element t - col when 0 <= t - col < len
                    const int c0 = readlane(col, r), l0 = readlane(len, r), s0a = su(r);
                    const int c1 = readlane(col, rb), l1 = readlane(len, rb), s1a = su(rb);
#pragma unroll
                    for (int tt = 0; tt < NT; ++tt) {
                        const int t = 64 * tt + lane;
                        e0[tt] = (uint32_t)(t - c0) < (uint32_t)l0 ? (uint32_t)stage[s0a + t] : kTabPad;
                        e1[tt] = !two ? kTabZero : (uint32_t)(t - c1) < (uint32_t)l1 ? (uint32_t)stage[s1a + t] : kTabPad;
                    }
                } else {
                    auto code = [&](int rr2, uint32_t (&e)[NT]) {
                        const int cr = readlane(col, rr2), lr = readlane(len, rr2);
                        const int ar = readlane(a1, rr2), br = readlane(b1, rr2);
                        const int so = readlane(rel, rr2) - cur.base;
#pragma unroll
                        for (int tt = 0; tt < NT; ++tt) {
                            const int t = 64 * tt + lane;
                            const int j = t - cr;
                            const bool del = j >= ar && j < ar + br;
                            const int is = j < ar ? j : j - br;
                            if (t >= T || j < 0 || (del ? ar : is) >= lr) e[tt] = kTabPad;   // pad (:514, :540)
                            else e[tt] = del ? kTabDel : (uint32_t)stage[so + is];
                        }
                    };
                    code(r, e0);
                    if (two) code(rb, e1);
                    else
#pragma unroll
                        for (int tt = 0; tt < NT; ++tt) e1[tt] = kTabZero;
                }
                uint4 f0[NT], f1[NT];
                uint32_t g0[NT], g1[NT];
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    f0[tt] = *(const uint4 *)(tab + e0[tt]);
                    g0[tt] = *(const uint32_t *)(tab + e0[tt] + 16);
                    f1[tt] = *(const uint4 *)(tab + e1[tt]);
                    g1[tt] = *(const uint32_t *)(tab + e1[tt] + 16);
                }
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    P0[tt] += (((uint64_t)f0[tt].y << 32) | f0[tt].x) + (((uint64_t)f1[tt].y << 32) | f1[tt].x);
                    P1[tt] += (((uint64_t)f0[tt].w << 32) | f0[tt].z) + (((uint64_t)f1[tt].w << 32) | f1[tt].z);
                    Z[tt] += g0[tt] + g1[tt];
                }
                prow += 2;
                if (prow >= 62) widen();              // <= 62 rows per packed field
            }
            if (__ballot(bad != 0)) return false;     // an invalid byte staged; bad rows at the next widening
            if (rend >= nr) break;
            cur = nxt;
        }
    }
    widen();
    return __ballot(bad != 0) == 0;
}

// One column tile of the general kernel's layouts decided from integer LLR
// bounds (as k_decide, with '+' rows as a sixth class): `src(r)` gives read r's
// element code in the lane's column.  Returns true when every live column is
// decided (call b, quality maxQ, unmasked) and fills `co` with the reference's
// finalize outputs for it (:603-621, :1001-1012); false leaves the tile to the
// double products.
struct DecideSums {
    uint32_t S[6] = {0, 0, 0, 0, 0, 0}, N[6] = {0, 0, 0, 0, 0, 0};
    uint32_t nN = 0, Z = 0;
    bool bad = false;
    __device__ __forceinline__ void add(uint32_t e, const uint32_t *s_wtab) {
        const uint32_t cls = e >> 9;
        const uint32_t w = s_wtab[e & 511u];
        bad |= cls == 7 || (cls != 6 && (w >> 31) != 0);
        const uint32_t l = w & 0xFFFFu;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            S[k] += cls == (uint32_t)k ? l : 0u;
            N[k] += cls == (uint32_t)k;
        }
        nN += cls == 6;
        Z += (w >> 16) & 0x7FFFu;
    }
};
__device__ __forceinline__ bool decide_usable(const Args &a, int R) { return a.t16 >= 0 && R <= 4095; }
// the decision from the summed rows (see decide_tile)
__device__ __forceinline__ bool decide_end(const Args &a, int R, bool live, bool ins_col, const DecideSums &D,
                                           ColOut &co) {
    // the first largest in the reference's order A T C G + -
    uint32_t Lb = D.S[0], kb = 0;
#pragma unroll
    for (int k = 1; k < 6; ++k) {
        const bool g = D.S[k] > Lb;
        Lb = g ? D.S[k] : Lb;
        kb = g ? (uint32_t)k : kb;
    }
    uint32_t L2 = 0, nb = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        L2 = max(L2, kb != (uint32_t)k ? D.S[k] : 0u);
        nb = kb == (uint32_t)k ? D.N[k] : nb;
    }
    const int nother = R - (int)D.nN - (int)nb;         // rows of the other classes (each adds <= 1/16 nat)
    const bool ok = !D.bad && (int)(Lb - L2) - nother >= a.t16 && (int)D.Z - (int)Lb <= 16 * 700;
    if (__ballot(live && !ok)) return false;
    // finalize (:613-618, :1001-1012) for an unmasked call kb
    const bool has_plus = D.N[4] > 0;
    const bool lower = has_plus && kb < 4;
    co.ch = (int)((0x2D2B47435441ull >> (8 * kb)) & 0xffu) + (lower ? 32 : 0);   // "ATCG+-"
    co.q = a.P->max_base_quality;
    co.d = R - (int)D.nN - (int)D.N[4];
    int match;
    if (kb == 4) match = (int)nb;
    else if (kb == 5) match = ins_col ? 0 : (int)nb;
    else match = (lower == ins_col) ? (int)nb : 0;
    co.e = R - match;
    co.overflow = false;
    return true;
}
template <class Src>
__device__ __forceinline__ bool decide_tile(const Args &a, int R, bool live, bool ins_col, const Src &src,
                                            const uint32_t *s_wtab, ColOut &co) {
    if (!decide_usable(a, R)) return false;
    DecideSums D;
    for (int r = 0; r < R; ++r) D.add(src(r), s_wtab);
    return decide_end(a, R, live, ins_col, D, co);
}

// --------------------------------------------------- per-read register view
// lane r of these registers holds read r (R <= 64); read back with readlane
struct LaneReads {
    int cl;      // first column of the read (pos - min_pos) | kept length << 16
    int sn;      // stage offset of its first kept base | runs << 16
};

// diagnostic phase clock of the general kernel (DCR_GSTAMP builds): cycles per
// phase and per record class, summed per wave, flushed at the kernel's end
struct GStamp {
    uint64_t t = 0, t0 = 0;
    uint64_t acc[20] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void start() {
        if (DCR_GSTAMP) t = t0 = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void mark(int k) {
        if (DCR_GSTAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            acc[k] += now - t;
            t = now;
        }
    }
    __device__ __forceinline__ void record(int cls) {     // record class: total cycles, count
        if (DCR_GSTAMP) {
            acc[8 + cls] += __builtin_amdgcn_s_memtime() - t0;
            acc[12 + cls] += 1;
        }
    }
};

// ------------------------------------------------------------ k_consensus
// One consensus record (single-strand subfamily or duplex pair) on one wave.
// FAST: only the staged layout (no insertion column, <= 64 reads, bytes fit the
// LDS stage, T <= kColsLds); any other record is appended to the overflow list
// and processed by the general kernel.
template <bool DUPLEX, bool FAST>
__device__ __forceinline__ void process_record(const Args &a, const int64_t rec, WaveLds &W, const double2 *s_lut,
                                               const double *s_qthr, const uint32_t *s_wtab, const bool dec,
                                               const int lane, GStamp &gs) {
    const dcr_params *P = a.P;
    gs.start();

    const dcr_out &O = DUPLEX ? a.ds : a.ss;
    const int64_t *col_off = DUPLEX ? a.in.ds_col_off : a.in.ss_col_off;
    const int64_t off = col_off[rec];
    const int64_t cap = col_off[rec + 1] - off;
    const int minbq = P->min_base_quality;
    const bool simple_q = P->error_rate_pre_labeling == 0 && P->error_rate_post_labeling == 0;

    const int R = DUPLEX ? 2 : (a.in.sub_off[rec + 1] - a.in.sub_off[rec]);

    // staging range: every read of a record lies in one contiguous byte range
    // (single-strand: its reads are consecutive in the batch; duplex: the two
    // single-strand regions are adjacent), known one hop before the per-read data
    const uint8_t *gb = DUPLEX ? a.ss.seq : a.in.bases;
    const uint8_t *gq = DUPLEX ? a.ss.qual : a.in.quals;
    int64_t lo_byte, hi_byte;
    if (!DUPLEX) {
        const int g0 = a.in.sub_off[rec];
        lo_byte = R > 0 ? a.in.seq_off[g0] : 0;
        hi_byte = R > 0 ? a.in.seq_off[g0 + R - 1] + a.in.seq_len[g0 + R - 1] : 0;
    } else {
        lo_byte = a.in.ss_col_off[2 * rec];
        hi_byte = a.in.ss_col_off[2 * rec + 1] + a.ss.len[2 * rec + 1];
    }
    const int64_t base_al = lo_byte & ~(int64_t)3;
    const int64_t span = hi_byte - base_al;
    const bool fits = R <= kWave && span <= kStageElems && ((((uintptr_t)gb) | ((uintptr_t)gq)) & 3) == 0;
    // issue the staging loads now (consumed after the setup reductions)
    constexpr int kStageDw = kStageElems / 4 / kWave;       // dwords per lane
    uint32_t vb[kStageDw], vq[kStageDw];
    const int nd = fits ? (int)((span + 3) >> 2) : 0;
    {
        const uint32_t *b4 = (const uint32_t *)(gb + base_al);
        const uint32_t *q4 = (const uint32_t *)(gq + base_al);
#pragma unroll
        for (int u = 0; u < kStageDw; ++u) {
            const int d = u * kWave + lane;
            vb[u] = d < nd ? b4[d] : 0u;
            vq[u] = d < nd ? q4[d] : 0u;
        }
    }

    // ---- setup: lane = read
    int minpos = 0x7fffffff, maxend = -0x7fffffff, up = 0, empty = 0, ins = 0, msum = 0, fst = 0;
    ReadRef myrd{};
    for (int c = 0; c < R; c += kWave) {
        const int r = c + lane;
        const int rst = r < R ? get_read<DUPLEX>(a, rec, r).status : 0;
        const unsigned long long fm = __ballot(rst != 0);
        if (!fst && fm) fst = __shfl(rst, __ffsll((long long)fm) - 1);   // the first failing read (:1272-1283)
        if (r < R) {
            const ReadRef rd = get_read<DUPLEX>(a, rec, r);
            if (r < kWave) myrd = rd;
            up |= rd.status != 0;
            empty |= rd.len <= 0;
            minpos = min(minpos, rd.pos);
            maxend = max(maxend, rd.pos + rd.len);
            msum += rd.mapq;
            if (!DUPLEX) {
                ins |= a.ws.info[a.in.sub_off[rec] + r].has_ins;
            } else {
                for (int k = 0; k < rd.ncig; ++k) ins |= (rd.cig[k] & 15) == 1;
            }
        }
    }
    minpos = wave_min(minpos);
    maxend = wave_max(maxend);
    up = __ballot(up) != 0;
    empty = __ballot(empty) != 0;
    ins = __ballot(ins) != 0;
    msum = wave_sum(msum);

    auto write_status = [&](int st) {
        if (lane == 0) {
            O.status[rec] = (uint8_t)st;
            O.pos[rec] = 0;
            O.mapq[rec] = 0;
            O.len[rec] = 0;
            O.n_cig[rec] = 0;
            O.n_de[rec] = 0;
            O.D[rec] = 0;
            O.M[rec] = 0;
            O.E[rec] = 0.0;
        }
    };
    if (R == 0) { write_status(DCR_ST_VALUE_ERROR); return; }      // min([]) (:458)
    if (up) { write_status(DUPLEX ? DCR_ST_UPSTREAM : (DCR_ST_PREP | (fst & 15))); return; }
    if (empty) { write_status(DCR_ST_TYPE_ERROR); return; }     // list(None) at :402
    const int T = maxend - minpos;                                  // :458-459
    if (T > cap) {
        if (lane == 0) atomicOr(a.ws.err, 1);
        write_status(255);
        return;
    }
    gs.mark(0);

    const bool cols_lds = T <= kColsLds;
    // ordering of the record's scratch between lanes: LDS only (wave-local DS
    // order) when the columns live in LDS, else also the global scratch (a
    // vmcnt drain, which also waits for every output store in flight)
    auto sfence = [&]() {
        if (cols_lds) lds_fence();
        else wave_fence();
    };
    int32_t *cons = cols_lds ? W.cons : a.ws.cons + off;
    double *et = cols_lds ? W.et : a.ws.et + off;
    uint16_t *od = O.d + off;
    uint16_t *oe = O.e + off;

    bool idx_err = false;      // IndexError inside reconstruct_alignment
    int nbad = 0;              // invalid nucleotide somewhere (:582)
    int n_de = 0, dmax = -1, dmin = 0x7fffffff;
    int first = -1, last = -1;
    bool qoverflow = false;    // int(-inf) consensus quality

    const bool big = R > kWave;
    const bool staged = fits && !ins;
    if (DCR_ABL == 9 && ins && big) return;       // diagnostic: general kernel without the > 64-read insertion layout
    if (DCR_ABL == 10 && ins && !big) return;     // diagnostic: ... without the <= 64-read insertion layout
    if (DCR_ABL == 11 && !ins) return;            // diagnostic: ... without the records free of insertions
    if (DCR_ABL == 12 && ins) return;             // diagnostic: ... without any insertion layout
    if constexpr (FAST) {
        if (!staged || !cols_lds) {          // general kernel takes it
            if (lane == 0) {
                const int idx = atomicAdd(&a.ws.ovf_count[DUPLEX ? 1 : 0], 1);
                a.ws.ovf[idx] = (int)rec;
            }
            return;
        }
    }

    // ---- k_decide proved every column's call from integer LLR bounds: the
    // tiles below take call / d / e from its column words instead of forming
    // the products
    const bool decided = !FAST && dec;

    // ---- phase 0: element codes into LDS (every record whose bytes fit: the
    // fast layout reads them by column, the insertion layout by read)
    if (fits && !decided) {
#pragma unroll
        for (int u = 0; u < kStageDw; ++u) {
            const int d = u * kWave + lane;
            if (d < nd) {
                uint32_t cc[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    cc[k] = make_code<DUPLEX>((vb[u] >> (8 * k)) & 255u, (vq[u] >> (8 * k)) & 255u, minbq);
                uint2 w;
                w.x = cc[0] | (cc[1] << 16);
                w.y = cc[2] | (cc[3] << 16);
                *(uint2 *)&W.stage[4 * d] = w;
            }
        }
        sfence();
    }
    if (DCR_ABL == 1) {
        if (lane == 0) O.pos[rec] = minpos + nd + (int)W.stage[lane];
        return;
    }
    LaneReads lr;
    lr.cl = (myrd.pos - minpos) | (myrd.len << 16);
    lr.sn = (int)(myrd.seq_start - base_al) | (myrd.ncig << 16);

    // R > 64 with insertion columns: precompute the insertion-column flags
    // (all reads must be consulted per column, :476-478) and keep per-read
    // layout state in global scratch between column tiles.
    uint8_t *insflag = a.ws.insflag + off;
    int4 *gstate = DUPLEX ? nullptr : a.ws.state + a.in.sub_off[rec];
    // up to kBigCh * 64 reads the layout state stays in registers (lane = read
    // within 64-read chunk c): the flags pass walks the runs without touching
    // HBM, and the tiles stage each chunk's next 32 bytes per read
    constexpr int kBigCh = 4;
    // insertion records that k_ins_layout laid out: the tiles load their rows
    // (no column steps, flag pass or windows here)
    const int64_t lrec = (DUPLEX ? 4 * (int64_t)a.in.n_fam : 0) + rec;
    const bool laid = DCR_LAYOUT_KERNEL && !FAST && ins && cols_lds && R <= kBigCh * kWave && a.ws.lay_base[lrec] > 0;
    uint64_t imask[4] = {0ull, 0ull, 0ull, 0ull};
    const uint16_t *lrows = nullptr;
    if (laid) {
        const uint64_t *mk = a.ws.lay_mask + 4 * lrec;
#pragma unroll
        for (int w = 0; w < 4; ++w) imask[w] = mk[w];
        lrows = a.ws.lay + (DUPLEX ? (int64_t)a.in.n_reads + 2 * rec : (int64_t)a.in.sub_off[rec]) * kLayRow;
    }
    const bool regbig = !FAST && ins && big && !DUPLEX && R <= kBigCh * kWave && !laid;
    struct SlimRead {
        int pos, len, ncig;
        const uint32_t *cig;
        int64_t seq_start;
    };
    SlimRead brd[kBigCh];
    Sim bs[kBigCh];
    auto slim_ref = [&](const SlimRead &b) {
        ReadRef rd{};
        rd.pos = b.pos;
        rd.len = b.len;
        rd.ncig = b.ncig;
        rd.cig = b.cig;
        rd.seq_start = b.seq_start;
        return rd;
    };
    if (regbig) {
#pragma unroll
        for (int c = 0; c < kBigCh; ++c) {
            brd[c] = SlimRead{0x7fffffff, 0, 0, nullptr, 0};
            bs[c] = Sim{0, 0, 0, -1, 0, 0u};
            const int r = c * kWave + lane;
            if (c * kWave < R && r < R) {
                const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                brd[c] = SlimRead{rd.pos, rd.len, rd.ncig, rd.cig, rd.seq_start};
                sim_load_run(bs[c], rd);
            }
        }
        for (int t = 0; t < T; ++t) {
            bool any = false;
#pragma unroll
            for (int c = 0; c < kBigCh; ++c)
                if (c * kWave < R) any |= __ballot(c * kWave + lane < R && bs[c].curop == 1) != 0;
#pragma unroll
            for (int c = 0; c < kBigCh; ++c)
                if (c * kWave < R && c * kWave + lane < R)
                    (void)sim_step_e<DUPLEX>(bs[c], slim_ref(brd[c]), minpos + t, any, idx_err,
                                             [](int) { return 0u; });
            if (lane == 0) insflag[t] = any;
        }
#pragma unroll
        for (int c = 0; c < kBigCh; ++c) {
            bs[c] = Sim{0, 0, 0, -1, 0, 0u};
            if (c * kWave < R && c * kWave + lane < R) sim_load_run(bs[c], slim_ref(brd[c]));
        }
        wave_fence();
    }
    if (!FAST && ins && big && !DUPLEX && !regbig && !laid) {
        for (int c = 0; c < R; c += kWave) {
            const int r = c + lane;
            if (r < R) {
                const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                Sim s{0, 0, 0, 0, 0};
                sim_load_run(s, rd);
                gstate[r] = make_int4(s.k, s.o, s.is, 0);
            }
        }
        wave_fence();
        for (int t = 0; t < T; ++t) {
            bool any = false;
            for (int c = 0; c < R; c += kWave) {
                const int r = c + lane;
                bool isI = false;
                if (r < R) {
                    const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                    const int4 st = gstate[r];
                    isI = st.x < rd.ncig && (rd.cig[st.x] & 15) == 1;
                }
                any |= __ballot(isI) != 0;
            }
            for (int c = 0; c < R; c += kWave) {
                const int r = c + lane;
                if (r < R) {
                    const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                    const int4 st = gstate[r];
                    Sim s{st.x, st.y, st.z, 0, 0};
                    sim_load_run(s, rd);
                    (void)sim_step<DUPLEX>(s, rd, minpos + t, any, minbq, idx_err);
                    gstate[r] = make_int4(s.k, s.o, s.is, 0);
                }
            }
            if (lane == 0) insflag[t] = any;
            wave_fence();
        }
        for (int c = 0; c < R; c += kWave) {
            const int r = c + lane;
            if (r < R) {
                const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                Sim s{0, 0, 0, 0, 0};
                sim_load_run(s, rd);
                gstate[r] = make_int4(s.k, s.o, s.is, 0);
            }
        }
        wave_fence();
    }

    // small-R insertion layout keeps its state in registers (lane = read)
    Sim sim{0, 0, 0, 0, 0};
    if (ins && !big && !laid && lane < R) sim_load_run(sim, myrd);

    // the next 32 bytes of a read from seq index is0 (the most a 32-column tile
    // consumes) as codes in the stage, [k][lane], from 9 range-checked dword
    // loads per lane issued together (records whose bytes do not fit the stage)
    auto stage_window = [&](bool on, int64_t seq_start, int is0) {
        if (!on) return;
        const int64_t o = seq_start + is0 - base_al;      // >= 0: base_al is the first read's byte
        // the range in whole dwords: a buffer load returns 0 for a dword that
        // reaches past it, which would zero the last bases of the batch's last
        // read (the arrays are padded to 256 bytes, so the rounded-up dword is
        // ours to read)
        const int64_t total = DUPLEX ? a.in.ss_cols : a.in.n_bases;
        const int64_t left = ((total + 3) & ~(int64_t)3) - base_al;
        const int nrec = (int)min(left, (int64_t)0x7FFFFFF0);
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)(gb + base_al), (short)0, nrec,
                                                                            0x00020000);
        const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void *)(gq + base_al), (short)0, nrec,
                                                                            0x00020000);
        const int oa = (int)(o & ~(int64_t)3);
        const uint32_t sh = (uint32_t)(o & 3);
        uint32_t db[9], dq[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            db[i] = __builtin_amdgcn_raw_buffer_load_b32(rb, oa + 4 * i, 0, 0);
            dq[i] = __builtin_amdgcn_raw_buffer_load_b32(rq, oa + 4 * i, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t wb = __builtin_amdgcn_alignbyte(db[i + 1], db[i], sh);
            const uint32_t wq = __builtin_amdgcn_alignbyte(dq[i + 1], dq[i], sh);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                W.stage[((4 * i + j) << 6) + lane] =
                    (uint16_t)make_code<DUPLEX>((wb >> (8 * j)) & 255u, (wq >> (8 * j)) & 255u, minbq);
        }
    };

    gs.mark(1);
    // ---- phases 1+2: column tiles (lane = column)
    const int tw = ins ? kTileIns : kWave;       // insertion layout: 32-column tiles
    for (int c0 = 0; c0 < T; c0 += tw) {
        const int t = c0 + lane;
        const bool live = lane < tw && t < T;
        const int ncol = min(tw, T - c0);
        Acc A;
        acc_init(A);
        bool ins_col = false;
        bool tdec = false;                           // this tile decided by decide_tile
        ColOut tco{};
        if (decided) {
            // the call, d and e of a decided column; quality maxQ (kb: A T C G + -)
        } else if (staged) {
            // fast layout from LDS: op index j = t - col of read r (:473-545 without I)
            auto src = [&](int r) -> uint32_t {
                const int cl = readlane(lr.cl, r);
                const int sn = readlane(lr.sn, r);
                const int col = cl & 0xffff, ln = (unsigned)cl >> 16;
                const int so = sn & 0xffff, nc = (unsigned)sn >> 16;
                const int j = t - col;
                uint32_t e = kPad;
                if (nc == 1) {
                    if (live && (unsigned)j < (unsigned)ln) e = W.stage[so + j];
                } else if (live && j >= 0) {
                    const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                    int is;
                    bool del;
                    if (walk_runs(rd.cig, rd.ncig, j, ln, is, del)) e = del ? kDel : W.stage[so + is];
                }
                return e;
            };
            accumulate(A, R, src, s_lut);
            gs.mark(4);
        } else if (FAST) {
            // unreachable: the fast kernel only keeps staged records
        } else if (!ins) {
            auto src = [&](int r) -> uint32_t {
                const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                const int j = t - (rd.pos - minpos);
                uint32_t e = kPad;
                int is;
                bool del;
                if (live && j >= 0 && walk_runs(rd.cig, rd.ncig, j, rd.len, is, del))
                    e = del ? kDel : base_elem<DUPLEX>(rd, is, minbq);
                return e;
            };
            accumulate(A, R, src, s_lut);
            gs.mark(4);
        } else if (laid) {
            // the rows k_ins_layout wrote: two reads per load (lanes 32-63 the
            // second), every load of a chunk issued before its tile is used
            const uint64_t mw = c0 < 64 ? imask[0] : c0 < 128 ? imask[1] : c0 < 192 ? imask[2] : imask[3];
            ins_col = live && ((mw >> (t & 63)) & 1ull) != 0;
            const int tt = lane & (kTileIns - 1);
            const int hcol = c0 + tt, hi = lane >> 5;
            for (int cb = 0; cb < R; cb += kWave) {
                const int nr = min(kWave, R - cb);
                // this tile of the chunk's reads: nr rows of 64 bytes, one block
                const uint4 *src4 = (const uint4 *)(lrows + ((int64_t)(c0 >> 5) * R + cb) * kTileIns);
                uint4 *dst4 = (uint4 *)&W.tile[0][0];
                uint4 q[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (u * kWave + lane < 4 * nr) q[u] = src4[u * kWave + lane];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (u * kWave + lane < 4 * nr) dst4[u * kWave + lane] = q[u];
                (void)hi;
                (void)hcol;
                sfence();
                gs.mark(3);
                auto src = [&](int rr) -> uint32_t { return live ? (uint32_t)W.tile[rr][lane & (kTileIns - 1)] : kPad; };
                if (R <= kWave) {
                    tdec = decide_tile(a, R, live, ins_col, src, s_wtab, tco);
                    if (!tdec) accumulate(A, R, src, s_lut);
                } else {
                    accumulate(A, nr, src, s_lut);
                }
                sfence();
                gs.mark(4);
            }
        } else if (!big) {
            uint64_t insmask = 0;
            // bytes that do not fit the stage: each read's next 32 bytes (the
            // most a 32-column tile consumes) as codes in the stage, [k][lane],
            // from 9 range-checked dword loads per lane issued together
            const int is0 = sim.is;
            if (!fits) {
                sfence();
                stage_window(lane < R, myrd.seq_start, is0);
                sfence();
            }
            gs.mark(2);
            if (DCR_GSTAMP) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                gs.mark(17);          // [17] memory operations drained before the steps (diagnostic)
                gs.acc[16] += ncol;   // [16] column steps
            }
            for (int tt = 0; tt < ncol; ++tt) {
                const bool isI = lane < R && sim.curop == 1;
                const bool any = __ballot(isI) != 0;
                insmask |= (uint64_t)any << tt;
                if (lane < R) {
                    uint32_t e;
                    if (fits) {
                        const int so = (int)(myrd.seq_start - base_al);
                        e = sim_step_e<DUPLEX>(sim, myrd, minpos + c0 + tt, any, idx_err,
                                               [&](int is) { return (uint32_t)W.stage[so + is]; });
                    } else {
                        e = sim_step_e<DUPLEX>(sim, myrd, minpos + c0 + tt, any, idx_err,
                                               [&](int is) { return (uint32_t)W.stage[((is - is0) << 6) + lane]; });
                    }
                    W.tile[lane][tt] = (uint16_t)e;
                }
            }
            sfence();
            gs.mark(3);
            ins_col = live && ((insmask >> lane) & 1);
            auto src = [&](int r) -> uint32_t { return live ? (uint32_t)W.tile[r][lane & (kTileIns - 1)] : kPad; };
            tdec = decide_tile(a, R, live, ins_col, src, s_wtab, tco);
            if (!tdec) accumulate(A, R, src, s_lut);
            sfence();
            gs.mark(4);
        } else if (regbig) {
            // this tile's insertion-column flags, one load per lane
            const uint64_t fm = __ballot(lane < ncol && insflag[c0 + lane] != 0);
            ins_col = live && ((fm >> lane) & 1);
#pragma unroll
            for (int c = 0; c < kBigCh; ++c) {
                if (c * kWave >= R) continue;
                const int nr = min(kWave, R - c * kWave);
                const bool mine = lane < nr;
                const int is0 = bs[c].is;
                sfence();
                stage_window(mine, brd[c].seq_start, is0);
                sfence();
                gs.mark(2);
                if (mine) {
                    const ReadRef rd = slim_ref(brd[c]);
                    for (int tt = 0; tt < ncol; ++tt)
                        W.tile[lane][tt] = (uint16_t)sim_step_e<DUPLEX>(
                            bs[c], rd, minpos + c0 + tt, ((fm >> tt) & 1) != 0, idx_err,
                            [&](int is) { return (uint32_t)W.stage[((is - is0) << 6) + lane]; });
                }
                sfence();
                gs.mark(3);
                auto src = [&](int rr) -> uint32_t { return live ? (uint32_t)W.tile[rr][lane & (kTileIns - 1)] : kPad; };
                accumulate(A, nr, src, s_lut);
                gs.mark(4);
            }
            sfence();
        } else {
            ins_col = live && insflag[t];
            for (int c = 0; c < R; c += kWave) {
                const int r = c + lane;
                const int nr = min(kWave, R - c);
                if (r < R) {
                    const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                    const int4 st = gstate[r];
                    Sim s{st.x, st.y, st.z, 0, 0};
                    sim_load_run(s, rd);
                    for (int tt = 0; tt < ncol; ++tt)
                        W.tile[lane][tt] = (uint16_t)sim_step<DUPLEX>(s, rd, minpos + c0 + tt, insflag[c0 + tt] != 0,
                                                                      minbq, idx_err);
                    gstate[r] = make_int4(s.k, s.o, s.is, 0);
                }
                wave_fence();
                auto src = [&](int rr) -> uint32_t { return live ? (uint32_t)W.tile[rr][lane & (kTileIns - 1)] : kPad; };
                accumulate(A, nr, src, s_lut);
                wave_fence();
            }
        }
        ColOut co;
        if (tdec) {
            co = tco;
        } else if (decided) {
            const uint32_t w = live ? (uint32_t)a.ws.cons[off + t] : 0u;
            co.ch = (int)((0x2D2B47435441ull >> (8 * (w & 7u))) & 0xffu) + (((w >> 27) & 1u) ? 32 : 0);   // "ATCG+-"
            co.q = P->max_base_quality;
            co.d = (int)((w >> 3) & 4095u);
            co.e = (int)((w >> 15) & 4095u);
            co.overflow = false;
        } else {
            nbad += live ? A.nbad : 0;
            const int nsw = wave_max(A.ns);
            if (DCR_ABL == 2) {
                if (live) cons[t] = (int)(A.U * 1e9) + nsw + A.n[0];
                continue;
            }
            co = finalize(A, nsw, R, ins_col, P, s_qthr, simple_q);
        }
        if (live) {
            cons[t] = co.ch | (co.q << 8);
            qoverflow |= co.overflow;
        }
        // d / e over columns whose consensus is not '+' (:1003, :1013)
        const bool keep = live && co.ch != '+';
        const uint64_t km = __ballot(keep);
        const int idx = n_de + __popcll(km & lanemask_lt(lane));
        if (keep) {
            od[idx] = (uint16_t)co.d;
            oe[idx] = (uint16_t)co.e;
            et[idx] = co.d == 0 ? 1.0 : (double)co.e / (double)co.d;
            dmax = max(dmax, co.d);
            dmin = min(dmin, co.d);
        }
        n_de += __popcll(km);
        // 5'/3' trims count uppercase 'N' only (:770-784)
        const uint64_t nn = __ballot(live && co.ch != 'N');
        if (nn) {
            if (first < 0) first = c0 + __builtin_ctzll(nn);
            last = c0 + 63 - __builtin_clzll(nn);
        }
        gs.mark(5);
    }
    if (DCR_ABL == 2 || DCR_ABL == 3) {
        if (lane == 0) O.pos[rec] = cons[0] + n_de + first + last;
        return;
    }
    const int Dmax = wave_max(dmax);
    const int Dmin = wave_min(dmin);
    idx_err = __ballot(idx_err) != 0;
    const bool bad = __ballot(nbad != 0) != 0;
    qoverflow = __ballot(qoverflow) != 0;
    if (idx_err) { write_status(DCR_ST_INDEX_ERROR); return; }
    if (bad) { write_status(DCR_ST_EXIT_BADCHAR); return; }
    if (qoverflow) { write_status(DCR_ST_OVERFLOW_ERROR); return; }
    sfence();

    // ---- phase 3: adjust_consensus_fields (:745-871) over [first, last]
    const int lo = first < 0 ? T : first;
    const int hi = first < 0 ? T : last + 1;
    uint8_t *oseq = O.seq + off;
    uint8_t *oqual = O.qual + off;
    uint32_t *ocig = O.cigar + off;
    // run starts: LDS (the staging region is dead now) when they fit
    uint32_t *rstart_buf = cols_lds ? (uint32_t *)W.stage : ocig;
    int nruns = 0, nops = 0, nlen = 0, last_op = -1, chain_start = lo;
    bool kept_overflow = false;
    for (int c0 = lo; c0 < hi; c0 += kWave) {
        const int t = c0 + lane;
        const bool live = t < hi;
        int ch = 0, q = 0, chn = 0, chp = 0;
        if (live) {
            const int v = cons[t];
            ch = v & 255;
            q = v >> 8;
            chn = t + 1 < hi ? (cons[t + 1] & 255) : 0;
            chp = t > lo ? (cons[t - 1] & 255) : 0;
        }
        const bool isL = ch >= 'a' && ch <= 'z';
        const bool isD = ch == '-';
        const bool isP = ch == '+';
        const bool nL = chn >= 'a' && chn <= 'z';
        const bool pL = chp >= 'a' && chp <= 'z';
        // a lowercase/'-' pair (either order) collapses into one M (:805-840)
        const bool alt = live && ((isL && chn == '-') || (isD && nL));
        const bool alt_prev = live && t > lo && ((pL && isD) || (chp == '-' && isL));
        const uint64_t bm = __ballot(live && !alt_prev);           // chain starts
        const uint64_t below = bm & ((lane == 63) ? ~0ull : ((2ull << lane) - 1ull));
        const int cs = below ? c0 + 63 - __builtin_clzll(below) : chain_start;
        const bool skipped = ((t - cs) & 1) != 0;
        int op = -1;
        if (live && !skipped) {
            if (alt) op = 0;
            else if (isP) op = -1;
            else if (isL) op = 1;
            else if (isD) op = 2;
            else op = 0;
        }
        if (bm) chain_start = c0 + 63 - __builtin_clzll(bm);
        // run-length compression of the op list (:716-742)
        const bool valid = op >= 0;
        const uint64_t vm = __ballot(valid);
        const uint64_t vbelow = vm & lanemask_lt(lane);
        int prev_op = last_op;
        {
            const int src = vbelow ? 63 - __builtin_clzll(vbelow) : lane;
            const int sop = __shfl(op, src);
            if (vbelow) prev_op = sop;
        }
        const bool rstart = valid && op != prev_op;
        const uint64_t rm = __ballot(rstart);
        if (rstart) {
            const int ri = nruns + __popcll(rm & lanemask_lt(lane));
            const int oi = nops + __popcll(vbelow);
            rstart_buf[ri] = ((uint32_t)oi << 4) | (uint32_t)op;  // run start, converted below
        }
        if (vm) last_op = __shfl(op, 63 - __builtin_clzll(vm));
        nruns += __popcll(rm);
        nops += __popcll(vm);
        // sequence / qualities: drop '+' and '-', uppercase (:857-865)
        const bool ks = live && !isP && !isD;
        const uint64_t sm = __ballot(ks);
        if (ks) {
            const int si = nlen + __popcll(sm & lanemask_lt(lane));
            oseq[si] = (uint8_t)(isL ? ch - 32 : ch);
            oqual[si] = (uint8_t)q;
            kept_overflow |= (q < 0 || q > 255);
        }
        nlen += __popcll(sm);
    }
    kept_overflow = __ballot(kept_overflow) != 0;
    if (nruns == 0) { write_status(DCR_ST_INDEX_ERROR); return; }   // compress_cigarlist([])
    if (n_de == 0) { write_status(DCR_ST_VALUE_ERROR); return; }     // max([]) at :1005
    if (kept_overflow) { write_status(DCR_ST_OVERFLOW_ERROR); return; }
    // single-strand: the rest of the region reads 'N' / quality 0, so the duplex
    // pass, which stages this region whole, never sees a byte that is not a
    // valid letter (the fast kernel pads its records the same way)
    if (!DUPLEX)
        for (int64_t i = nlen + lane; i < cap; i += kWave) {
            oseq[i] = 'N';
            oqual[i] = 0;
        }
    sfence();
    for (int i0 = 0; i0 < nruns; i0 += kWave) {
        const int i = i0 + lane;
        uint32_t v = 0, nx = 0;
        if (i < nruns) {
            v = rstart_buf[i];
            nx = i + 1 < nruns ? (rstart_buf[i + 1] >> 4) : (uint32_t)nops;
        }
        sfence();
        if (i < nruns) ocig[i] = ((nx - (v >> 4)) << 4) | (v & 15);
    }

    gs.mark(6);
    // ---- E = round(mean(e/d), 3) with numpy's pairwise summation (:1015-1018)
    // pairwise_sum(a, n): n < 8 sequential; n <= 128 eight accumulators; else
    // split at n2 = n/2 rounded down to a multiple of 8 and add the halves.
    sfence();
    auto leaf = [&](int fo, int fn) -> double {
        double res;
        if (fn < 8) {
            res = -0.0;
            for (int i = 0; i < fn; ++i) res += et[fo + i];
        } else {
            const int body = fn - (fn % 8);
            double r = 0.0;
            if (lane < 8) {
                r = et[fo + lane];
#pragma unroll 4
                for (int i = 8; i < body; i += 8) r += et[fo + i + lane];
            }
            const double r0 = __shfl(r, 0), r1 = __shfl(r, 1), r2 = __shfl(r, 2), r3 = __shfl(r, 3);
            const double r4 = __shfl(r, 4), r5 = __shfl(r, 5), r6 = __shfl(r, 6), r7 = __shfl(r, 7);
            res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
            for (int i = body; i < fn; ++i) res += et[fo + i];
        }
        return res;
    };
    double total;
    if (n_de <= 128) {
        total = leaf(0, n_de);
    } else if (n_de <= 240) {           // both halves <= 128 (ceil(n/2) + 7 <= 128)
        int n2 = n_de / 2;
        n2 -= n2 % 8;
        const double left = leaf(0, n2);
        total = left + leaf(n2, n_de - n2);
    } else if (!FAST) {
        // general depth: explicit uniform stack in LDS
        int *stk_off = W.stk_off, *stk_n = W.stk_n, *stk_stage = W.stk_stage;
        double *stk_left = W.stk_left;
        int sp = 0;
        stk_off[0] = 0;
        stk_n[0] = n_de;
        stk_stage[0] = 0;
        double ret = 0.0;
        while (sp >= 0) {
            const int fo = stk_off[sp], fn = stk_n[sp];
            if (fn <= 128) {
                ret = leaf(fo, fn);
                --sp;
                continue;
            }
            int n2 = fn / 2;
            n2 -= n2 % 8;
            if (stk_stage[sp] == 0) {
                stk_stage[sp] = 1;
                ++sp;
                stk_off[sp] = fo;
                stk_n[sp] = n2;
                stk_stage[sp] = 0;
            } else if (stk_stage[sp] == 1) {
                stk_left[sp] = ret;
                stk_stage[sp] = 2;
                ++sp;
                stk_off[sp] = fo + n2;
                stk_n[sp] = fn - n2;
                stk_stage[sp] = 0;
            } else {
                ret = stk_left[sp] + ret;
                --sp;
            }
        }
        total = ret;
    } else {
        total = 0.0;   // unreachable in the fast kernel (T <= kColsLds)
    }
    total = 0.0 + total;
    const double mean = total / (double)n_de;
    const double E = __builtin_rint(mean * 1000.0) / 1000.0;

    if (lane == 0) {
        O.status[rec] = DCR_ST_OK;
        O.pos[rec] = minpos + lo;                   // :790
        O.mapq[rec] = msum / R;                     // trunc(np.mean) (:887, :1377)
        O.len[rec] = nlen;
        O.n_cig[rec] = nruns;
        O.n_de[rec] = n_de;
        O.D[rec] = Dmax;
        O.M[rec] = Dmin;
        O.E[rec] = E;
    }
    gs.mark(7);
    gs.record(!ins ? 0 : laid ? (big ? 2 : 1) : !big ? 1 : regbig ? 2 : 3);
}


// numpy pairwise_sum over a[0..n), n <= 240 (at most two blocks of <= 128, 8 accumulators):
// accumulator j of block b lives on lane 8b + j and loads its <= 16 elements
// up front; the fixed association order of numpy is kept exactly.
__device__ __forceinline__ double pairwise_small(const double *a, int n, int lane) {
    if (n < 8) {
        double res = -0.0;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    int n2 = n, nb = 1;
    if (n > 128) {
        n2 = n / 2;
        n2 -= n2 % 8;
        nb = 2;
    }
    const int blk = (lane >> 3) & 1;
    const int bo = blk ? n2 : 0;                 // block offset
    const int bn = blk ? n - n2 : n2;            // block length (>= 8 when it is a block)
    const int body = bn - (bn % 8);
    const int j = lane & 7;
    // accumulator j: a[j], a[j + 8], ... in order; loaded four at a time
    double r = 0.0;
#pragma unroll 1
    for (int i0 = 0; i0 < 16; i0 += 4) {
        double v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = j + 8 * (i0 + k);
            v[k] = (lane < 8 * nb && idx < body) ? a[bo + idx] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (8 * (i0 + k) < body) r = i0 + k == 0 ? v[k] : r + v[k];
    }
    // per block: ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)), then the tail in order
    const double p01 = r + __shfl_xor(r, 1);
    const double p0123 = p01 + __shfl_xor(p01, 2);
    const double s8 = p0123 + __shfl_xor(p0123, 4);
    double res[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        double x = __shfl(s8, 8 * b);
        const int o = b ? n2 : 0, m = b ? n - n2 : n2;
        const int bd = m - (m % 8);
        if (b < nb)
            for (int i = bd; i < m; ++i) x += a[o + i];
        res[b] = x;
    }
    return nb == 1 ? res[0] : res[0] + res[1];
}

// 64-bit DPP move (two 32-bit halves)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    // full-row permutations: every lane reads a valid source, so no "old" value
    const int2 h = __builtin_bit_cast(int2, v);
    int2 r;
    r.x = __builtin_amdgcn_mov_dpp(h.x, CTRL, 0xF, 0xF, true);
    r.y = __builtin_amdgcn_mov_dpp(h.y, CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, r);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const int2 h = __builtin_bit_cast(int2, v);
    return __builtin_bit_cast(double, make_int2(readlane(h.x, l), readlane(h.y, l)));
}

// numpy pairwise_sum over a[0..n) in LDS, n <= 240, for the fast kernel: as
// pairwise_small, with every load issued up front (two batches of eight per
// accumulator lane and the tails of both blocks) and the eight-accumulator
// combine ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) done with DPP instead of LDS
// permutes.  Same association order, bit for bit.
__device__ __forceinline__ double pairwise_et(const double *a, int n, int lane) {
    if (n < 8) {
        double res = -0.0;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    int n2 = n, nb = 1;
    if (n > 128) {
        n2 = n / 2;
        n2 -= n2 % 8;
        nb = 2;
    }
    const int blk = (lane >> 3) & 1;
    const int bo = blk ? n2 : 0;                 // block offset
    const int bn = blk ? n - n2 : n2;            // block length (>= 8 when it is a block)
    const int body = bn - (bn % 8);
    const int j = lane & 7;
    const bool acc = lane < 8 * nb;
    // tails (< 8 elements after the body of each block), loaded by lanes 0 and 8
    const int tail = bn % 8;
    double tv[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) tv[i] = (acc && j == 0 && i < tail) ? a[bo + body + i] : 0.0;
    double r = 0.0;
#pragma unroll
    for (int i0 = 0; i0 < 16; i0 += 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int idx = j + 8 * (i0 + k);
            v[k] = (acc && idx < body) ? a[bo + idx] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (8 * (i0 + k) < body) r = i0 + k == 0 ? v[k] : r + v[k];
    }
    const double p01 = r + dpp_f64<0xB1>(r);            // quad_perm [1,0,3,2]
    const double p0123 = p01 + dpp_f64<0x4E>(p01);      // quad_perm [2,3,0,1]
    const double s8 = p0123 + dpp_f64<0x141>(p0123);    // row_half_mirror: quad 0 <-> quad 1
    double res[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        double x = readlane_f64(s8, 8 * b);
        const int m = b ? n - n2 : n2;
        const int tc = b < nb ? m % 8 : 0;
#pragma unroll
        for (int i = 0; i < 7; ++i)
            if (i < tc) x += readlane_f64(tv[i], 8 * b);
        res[b] = x;
    }
    return nb == 1 ? res[0] : res[0] + res[1];
}

// ------------------------------------------------------------ k_recmeta
// Classifies every record before any consensus work: the status the reference
// reaches first (a read that failed preprocessing, or an empty read — :1291-1300
// via the read statuses of prep_read), a fast record, or a general one.  For fast
// records it writes the launch metadata the fast kernel fetches with one scalar
// load per record plus one 8-byte load per read.
//
// One wave per a.rpw records (64, or fewer when records are deep, so that the
// read pass of a C4-shape batch still spreads over thousands of waves).  Reads are visited lane = read (coalesced loads) and
// folded into their record's LDS slot with LDS atomics; the record of a read
// comes from a marker per record start and a DPP prefix-max scan.  List appends
// are wave-aggregated (one global atomic per wave per list).
struct RdLite {
    int pos, len, ncig, status, mapq;
    int64_t seq_start;
    uint32_t cig0;
};

template <bool DUPLEX, bool CIG>
__device__ __forceinline__ RdLite rd_lite(const Args &a, int64_t k) {
    RdLite r;
    r.cig0 = 0;
    if (!DUPLEX) {                              // k: read index; clips only (the 3' trim is the fast kernel's)
        const ClipView cv = clip_view(a.in, k);
        r.pos = a.in.read_pos[k];
        r.len = cv.len;
        r.ncig = cv.single_m ? 1 : 2;
        r.status = cv.len <= 0 ? DCR_ST_TYPE_ERROR : 0;   // empty sequence: enumerate(None) at :279
        r.mapq = a.in.read_mapq[k];
        r.seq_start = cv.seq_start;
    } else {                                    // k: single-strand record index
        r.pos = a.ss.pos[k];
        r.len = a.ss.len[k];
        r.ncig = a.ss.n_cig[k];
        r.status = a.ss.status[k];
        r.mapq = a.ss.mapq[k];
        r.seq_start = a.in.ss_col_off[k];
        if (CIG && r.status == 0 && r.ncig == 1 && r.len > 0) r.cig0 = a.ss.cigar[r.seq_start];
    }
    return r;
}

// rd_lite in two halves so that a wave keeps several 64-read chunks' loads in
// flight: the independent per-read fields first, then the one dependent load
// (the first CIGAR word); reads whose CIGAR is not one M/=/X run take the full
// clip_view (rare)
struct RdRaw {
    int64_t seq_off;
    int seq_len, pos, mapq, n, status;
    int32_t cig_off;
    uint32_t cig0;
};

template <bool DUPLEX>
__device__ __forceinline__ void rd_raw_load(const Args &a, int64_t k, RdRaw &w) {
    if (!DUPLEX) {
        w.cig_off = a.in.cig_off[k];
        w.n = a.in.cig_n[k];
        w.seq_off = a.in.seq_off[k];
        w.seq_len = a.in.seq_len[k];
        w.pos = a.in.read_pos[k];
        w.mapq = a.in.read_mapq[k];
    } else {
        w.pos = a.ss.pos[k];
        w.seq_len = a.ss.len[k];
        w.n = a.ss.n_cig[k];
        w.status = a.ss.status[k];
        w.mapq = a.ss.mapq[k];
        w.seq_off = a.in.ss_col_off[k];
    }
}

template <bool DUPLEX>
__device__ __forceinline__ void rd_raw_cig(const Args &a, RdRaw &w) {
    if (!DUPLEX) w.cig0 = w.n >= 1 ? a.in.cigar[w.cig_off] : 0u;
    else w.cig0 = (w.status == 0 && w.n == 1 && w.seq_len > 0) ? a.ss.cigar[w.seq_off] : 0u;
}

template <bool DUPLEX>
__device__ __forceinline__ RdLite rd_raw_finish(const Args &a, int64_t k, const RdRaw &w) {
    RdLite r;
    if (!DUPLEX) {
        const uint32_t op = w.cig0 & 15u;
        if (w.n == 1 && (op == 0 || op == 7 || op == 8)) {   // one M/=/X run: no clip (clip_view's fast case)
            r.pos = w.pos;
            r.len = w.seq_len;
            r.ncig = (int)(w.cig0 >> 4) == w.seq_len ? 1 : 2;
            r.status = w.seq_len <= 0 ? DCR_ST_TYPE_ERROR : 0;
            r.mapq = w.mapq;
            r.seq_start = w.seq_off;
            r.cig0 = 0;
        } else {
            r = rd_lite<false, true>(a, k);
        }
    } else {
        r.pos = w.pos;
        r.len = w.seq_len;
        r.ncig = w.n;
        r.status = w.status;
        r.mapq = w.mapq;
        r.seq_start = w.seq_off;
        r.cig0 = w.cig0;
    }
    return r;
}

__device__ __forceinline__ void write_status_at(const dcr_out &O, int64_t rec, int st) {
    O.status[rec] = (uint8_t)st;
    O.pos[rec] = 0;
    O.mapq[rec] = 0;
    O.len[rec] = 0;
    O.n_cig[rec] = 0;
    O.n_de[rec] = 0;
    O.D[rec] = 0;
    O.M[rec] = 0;
    O.E[rec] = 0.0;
}

// wave-local LDS ordering: a wave's DS instructions execute in order, so only
// the compiler must be kept from reordering (no vmcnt drain of prefetches)
// A value the compiler cannot see through: per-lane addresses built from it
// are formed where used instead of being hoisted out of the record loop (and
// held in registers across it).
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));


// IEEE max / min of two doubles known not to be NaN (no canonicalising moves)
__device__ __forceinline__ double vmax_f64(double x, double y) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ double vmin_f64(double x, double y) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}


// inclusive prefix max over the wave (DPP row shifts, then row broadcasts)
__device__ __forceinline__ int wave_scan_max(int v) {
    constexpr int I = -0x7fffffff - 1;
    v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x142, 0xA, 0xF, false));   // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return v;
}

// record (wave lane) owning read c + lane; records are contiguous runs of reads
__device__ __forceinline__ int read_record(int64_t c, int g0, int R, int *mark, int lane, int &carry,
                                           bool *starts = nullptr) {
    mark[lane] = -1;
    lds_fence();
    if (R > 0 && g0 >= c && g0 < c + kWave) atomicMax(&mark[g0 - c], lane);
    lds_fence();
    const int mk = mark[lane];
    if (starts) *starts = mk >= 0;
    const int k = max(wave_scan_max(mk), carry);
    carry = readlane(k, 63);
    return k;
}

struct RecAgg {
    int minpos, maxend, flags, kind;
    unsigned long long lo, hi;     // kept byte window; lo becomes base_al for fast records
    unsigned long long fst;        // first failing read: global index << 4 | its status
    int pos0, msum;                // pos of the record's first read, sum of the reads' MAPQs
};
static_assert(sizeof(RecAgg) == 48, "recmeta_lds_bytes assumes a 48-byte RecAgg");

// The list appends take one device-scope atomic per list per BLOCK of
// kRecmetaWaves waves (a prefix over the block's waves in LDS): appends to one
// counter serialise at about 30 ns each on this part (one extra atomic per
// wave cost +0.62 ms per 1.25 M records, tools/ablate.py), so a per-wave
// atomic alone had made this pass 0.26 ms.  A wave past the last record still
// reaches the block's barriers (no reads, no records).  Blocks of records with
// many reads (rpw < 64) are 4 waves: a block's barrier waits for its slowest
// wave, and their lists are short.  LDS is sized by the launch
// (recmeta_lds_bytes).
template <bool DUPLEX>
__global__ __launch_bounds__(kRecmetaWaves * kWave) void k_recmeta(Args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t rm_lds[];
    const int nwb = (int)(blockDim.x >> 6);                      // waves in this block
    RecAgg (*s_agg)[kWave] = (RecAgg (*)[kWave])rm_lds;
    int (*s_mark)[kWave] = (int (*)[kWave])(rm_lds + sizeof(RecAgg) * kWave * nwb);
    int *s_cnt = (int *)(rm_lds + (sizeof(RecAgg) + sizeof(int)) * kWave * nwb);   // [3][nwb]
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    RecAgg *agg = s_agg[wave];
    int *mark = s_mark[wave];
    const int64_t rb = min(((int64_t)blockIdx.x * nwb + wave) * a.rpw, a.n_rec);
    const int64_t rk = rb + lane;
    const bool vk = lane < a.rpw && rk < a.n_rec;
    const int64_t rend = min(rb + a.rpw, a.n_rec);
    int g0 = 0, R = 0;
    int64_t gbeg, gend;
    if (!DUPLEX) {
        if (vk) {
            g0 = a.in.sub_off[rk];
            R = a.in.sub_off[rk + 1] - g0;
        }
        gbeg = a.in.sub_off[rb];
        gend = a.in.sub_off[rend];
    } else {
        g0 = (int)(2 * rk);                     // pair p uses single-strand records 2p, 2p+1 (:1575-1576)
        R = vk ? 2 : 0;
        gbeg = 2 * rb;
        gend = 2 * rend;
    }
    agg[lane] = RecAgg{0x7fffffff, -0x7fffffff, 0, -1, ~0ull, 0ull, ~0ull, 0, 0};
    lds_fence();
    // one pass: fold every read into its record, and write the read's word for
    // the fast kernel (relative to the record's first read, so it needs no
    // record-level result); a read whose offset from the first read does not fit
    // 16 bits sends its record to the general kernel (flag 4)
    int carry = -1;
    constexpr int kBatch = 6;                     // 64-read chunks with their loads in flight together
    for (int64_t cb = gbeg; cb < gend; cb += kBatch * kWave) {
    RdRaw raw[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
        const int64_t gr = cb + j * kWave + lane;
        if (gr < gend) rd_raw_load<DUPLEX>(a, gr, raw[j]);
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
        const int64_t gr = cb + j * kWave + lane;
        if (gr < gend) rd_raw_cig<DUPLEX>(a, raw[j]);
    }
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
        const int64_t c = cb + j * kWave;
        if (c >= gend) break;
        bool starts;
        const int k = read_record(c, g0, R, mark, lane, carry, &starts);
        const int64_t gr = c + lane;
        RdLite rd{};
        if (gr < gend) {
            rd = rd_raw_finish<DUPLEX>(a, gr, raw[j]);
            if (starts) agg[k].pos0 = rd.pos;
        }
        lds_fence();
        if (gr < gend) {
            const int dpos = rd.pos - agg[k].pos0;
            const int fl = (rd.status != 0) | ((rd.len <= 0) << 1) |
                           ((rd.ncig != 1 || (DUPLEX && rd.len > 0 && (rd.cig0 & 15u) != 0) || dpos < -32768 ||
                             dpos > 32767) << 2);   // single M run only
            atomicMin(&agg[k].minpos, rd.pos);
            atomicMax(&agg[k].maxend, rd.pos + rd.len);
            atomicAdd(&agg[k].msum, rd.mapq & 255);
            if (fl) atomicOr(&agg[k].flags, fl);
            if (rd.status) atomicMin(&agg[k].fst, ((unsigned long long)gr << 4) | (unsigned)(rd.status & 15));
            atomicMin(&agg[k].lo, (unsigned long long)rd.seq_start);
            atomicMax(&agg[k].hi, (unsigned long long)(rd.seq_start + rd.len));
            a.ws.rmeta[gr] = make_uint2(((uint32_t)rd.len & 255u) | (((uint32_t)rd.mapq & 255u) << 8) |
                                            ((uint32_t)dpos << 16),
                                        (uint32_t)rd.seq_start);
        }
    }
    }
    lds_fence();
    // per record: lane = record
    int kind = -1;                               // 0 fast, 1 general, -1 finished here
    RecMeta m{};
    if (vk) {
        const dcr_out &O = DUPLEX ? a.ds : a.ss;
        const int64_t *col_off = DUPLEX ? a.in.ds_col_off : a.in.ss_col_off;
        const uint8_t *gb = DUPLEX ? a.ss.seq : a.in.bases;
        const uint8_t *gq = DUPLEX ? a.ss.qual : a.in.quals;
        const RecAgg g = agg[lane];
        int st = -1;
        if (R == 0) st = DCR_ST_VALUE_ERROR;         // min([]) in reconstruct_alignment (:458)
        else if (R > kWave) kind = 1;
        else if (g.flags & 1) st = DUPLEX ? DCR_ST_UPSTREAM : (DCR_ST_PREP | (int)(g.fst & 15));
        else if (g.flags & 2) st = DCR_ST_TYPE_ERROR;
        else {
            const int T = g.maxend - g.minpos;
            const int64_t off = col_off[rk];
            const int64_t cap = col_off[rk + 1] - off;
            const int64_t base_al = (int64_t)g.lo & ~(int64_t)15;     // 16-byte staging loads
            const int64_t span = (int64_t)g.hi - base_al;
            const bool aligned = ((((uintptr_t)gb) | ((uintptr_t)gq)) & 15) == 0;
            // single-strand: the fast kernel pads its region to T rounded to 16
            // columns, which must be the whole region (the duplex pass stages it)
            const bool region_ok = DUPLEX ? T <= cap : cap == (((int64_t)T + 15) & ~(int64_t)15);
            if ((g.flags & 4) || !aligned || R > kFastMaxR || span > kStageElems || T > kFastMaxT || !region_ok ||
                !a.fast_ok || base_al + span >= 0xFFFFF000ll) {
                kind = 1;
            } else {
                kind = 0;
                m.base_al = (uint32_t)base_al;
                // MAPQ = trunc(mean) of the reads' MAPQs (:874-889, :1377), here
                // rather than a wave reduction per record in the fast kernel
                m.d0 = (g.pos0 - g.minpos) | ((g.msum / R) << 16);
                m.off = off;
                m.rec = (int32_t)rk;
                m.g0 = g0;
                m.minpos = g.minpos;
                m.w = (uint32_t)R | ((uint32_t)T << 7) | ((uint32_t)((span + 3) >> 2) << 15);
                agg[lane].lo = (unsigned long long)base_al;
            }
        }
        agg[lane].kind = kind;
        if (st >= 0) write_status_at(O, rk, st);
    }
    const uint64_t bf = __ballot(kind == 0);
    const uint64_t bg = __ballot(kind == 1);
    if (lane < 2) s_cnt[lane * nwb + wave] = __popcll(lane == 0 ? bf : bg);
    __syncthreads();
    if (threadIdx.x < 2) {                       // list t: the waves' exclusive prefix, one atomic
        const int t = threadIdx.x;
        int tot = 0;
        for (int w = 0; w < nwb; ++w) {
            const int c = s_cnt[t * nwb + w];
            s_cnt[t * nwb + w] = tot;
            tot += c;
        }
        int *ctr = t == 0 ? &a.ws.fast_count[DUPLEX ? 1 : 0] : &a.ws.ovf_count[DUPLEX ? 1 : 0];
        const int base = tot ? atomicAdd(ctr, tot) : 0;
        for (int w = 0; w < nwb; ++w) s_cnt[t * nwb + w] += base;
    }
    __syncthreads();
    const int basef = s_cnt[wave], baseg = s_cnt[nwb + wave];
    const uint64_t lt = lanemask_lt(lane);
    if (kind == 0) a.ws.meta[basef + __popcll(bf & lt)] = m;
    if (kind == 1) a.ws.ovf[baseg + __popcll(bg & lt)] = (int)rk;
    // single-strand reads of records the fast kernel does not take need the full
    // preprocessing (3' trim included) for the general kernel and the host;
    // records of more than 64 reads are left to k_prep_big (a block per record,
    // not one wave walking every read of 64 records)
    if (!DUPLEX) agg[lane].kind = (vk && R > kWave) ? 2 : kind;
    if (DUPLEX || __ballot(vk && kind != 0 && R <= kWave) == 0) return;
    lds_fence();
    carry = -1;
    for (int64_t c = gbeg; c < gend; c += kWave) {
        const int k = read_record(c, g0, R, mark, lane, carry);
        const int64_t gr = c + lane;
        if (gr < gend && agg[k].kind != 0 && agg[k].kind != 2) prep_read(a.in, a.P, a.ws, gr);
    }
}

// per-read preprocessing of the general list's records of more than 64 reads
// (k_recmeta leaves them out): one block per record, 256 reads at a time
__global__ __launch_bounds__(256) void k_prep_big(Args a) {
    const int n = a.ws.ovf_count[0];
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t rec = a.ws.ovf[i];
        const int g0 = a.in.sub_off[rec];
        const int R = a.in.sub_off[rec + 1] - g0;
        if (R <= kWave) continue;
        for (int r = threadIdx.x; r < R; r += blockDim.x) prep_read(a.in, a.P, a.ws, g0 + r);
    }
}

// ------------------------------------------------------- fast kernel (v6)
// Records of the dominant shape: every read a single M run (no insertion
// column, no '-' row), <= 63 reads, bytes fit one LDS stage, T <= 240, every
// staged quality <= 122, every staged base a valid letter and every kept base's
// quality >= fast_qlo (else the record is handed to the general kernel).  Then
// every aligned row is a base, a masked 'N' or a pad 'N', and the consensus
// CIGAR is one M run over the trimmed span (:797-848 yields M for every such
// column).
//
// The decision, not the products.  The reference keeps six likelihood products
// per column (:594-600, order A T C G + -; without '+'/'-' rows the last two are
// the chain U of p'/5 factors).  What the fast path writes depends only on the
// call b and on whether the reference's finalize gives quality maxQ without
// masking (:617, :699-709): then the record's fields are b, maxQ, d, e.  So the
// fast kernel proves that decision instead of forming the products:
//   L_k / L_b = exp(LLR_k - LLR_b),  U / L_b = exp(-LLR_b),
//   LLR_k = sum over class-k rows of ln((1-p')/(p'/5))      ('N' rows add 0),
// and S - L_b <= 5 exp(-gap) L_b with gap = LLR_b - max(LLR_k (k != b), 0).
// The per-row terms are host-rounded DOWN to 1/16 nat (16-bit fields, exact
// integer sums), so LLR_b >= L_b / 16 and LLR_k <= (L_k + n_k) / 16; the column
// is decided when L_b - L_2nd - n_other >= T16 = ceil(16 ln(5 / cc)) + 1 with
// cc = min(qthresh[maxQ], 1 - threshold, 1/4) -- a margin of 1/16 nat, far
// beyond every rounding of the reference's double arithmetic.  Any column
// outside sends its record to the general kernel (the reference's finalize).
//
// Element codes ARE LDS byte addresses of 16-byte table rows: code = (k << 11)
// | 16 (q + k) for class k (N 0, A 1, T 2, C 3, G 4; the 16 k shift spreads the
// classes over LDS banks).  Row: u64 LLR increments (16-bit fields A T C G),
// u32 count increment 1 << 6k (6-bit counters N A T C G, R <= 63).
//
// LDS of one 16-wave block (one per CU): table (10 KiB), per-wave stages,
// e/d table [d][e], pad sentinel, pointer cache, per-wave read words, later
// descriptor and column words.
namespace fk {
constexpr int kWaves = kFastWaves;                         // waves per block
constexpr int kBlockThreads = kFastBlock;
constexpr int kRowMax = 122;                               // quality rows 0..122
constexpr uint32_t kPadCode = 16u * 2u;                    // class N, quality 2 (:509-510, :543-544)
constexpr uint32_t kPadCode8 = 8u * 2u;                    // the same in the narrow table (common instantiation)
constexpr int kTable = 5 * 0x800;                          // 5 class banks of 2 KiB (narrow: of 1 KiB)
constexpr int kTable8 = 5 * 0x400;
constexpr int kPtrs = kTable;                              // u64 [32] pointers (kP* below)
constexpr int kSent = kPtrs + 32 * 8;                      // u16 pad code (out-of-read sentinel)
constexpr int kM720 = kSent + 16;                          // u32 [64] 720720 / d for depths d <= 16, else 0
constexpr int kInvD = kM720 + 64 * 4;                      // f64 [64] 1 / d
constexpr int kSofs = kInvD + 64 * 8;                      // u32 [10][2]: record-scalar array offsets from sbase, shifts
constexpr int kMv = kSofs + 10 * 8;                        // per wave: u32 [8] a later record's descriptor
constexpr int kWave0 = kMv + kWaves * 32;                  // the waves' regions
static_assert(16 * (kRowMax + 5) <= 0x800, "a class bank fits 2 KiB");
static_assert(kWave0 % 16 == 0, "16-byte aligned stages");
// a wave's region: the staged element codes (2 B per byte of the record),
// the current record's read words (u64 [64]) and, EXACT, the column words
// (u16 [256], d | e << 6 | call << 12).  The EXACT instantiation stages up to
// 2,048 bytes against the wide table (16-byte rows): 31,968 B per 4-wave
// block, four blocks per CU at its 128 VGPRs.  The common instantiation stages
// records of at most 1,536 bytes (larger ones go to the EXACT queue unstaged)
// against the narrow table (8-byte rows, 5 KiB, so wave 0's region lies in the
// table's unused half) and keeps its column words in the codes' space, dead
// once the evidence is summed: 22,240 B per block, seven blocks (28 waves)
// per CU.
#ifndef DCR_LDS_PAD
#define DCR_LDS_PAD 0
#endif
template <bool EXACT>
struct Region {
    static constexpr int kCodes = EXACT ? 0x1000 : 0xC00;
    static constexpr int kRm = kCodes;                     // offset of the read words
    static constexpr int kOv = EXACT ? kCodes + 512 : 0;   // offset of the column words
    static constexpr int kList = kCodes + 1024;            // EXACT: u8 [256] the undecided columns, compacted
    static constexpr int kBytes = kCodes + 512 + (EXACT ? 512 + 256 : 0);
    static constexpr int kDw = kCodes / 2 / 4 / kWave;     // staged dwords per lane: 8 / 6
    static constexpr int kLds = kWave0 + (EXACT ? kWaves : kWaves - 1) * kBytes + DCR_LDS_PAD;   // PAD: diagnostic builds
    __device__ static constexpr int base(int wave) {       // wave's region
        return EXACT ? kWave0 + wave * kBytes : (wave == 0 ? kTable8 : kWave0 + (wave - 1) * kBytes);
    }
    __device__ static constexpr int ov(int wave) { return base(wave) + kOv; }   // column words
};
static_assert(kTable8 + Region<false>::kBytes <= kTable, "wave 0's region in the narrow table's unused half");
// the LDS cliffs (measured, DESIGN §3: 32,016 B ran four 4-wave blocks per CU
// where 31,968 B ran five, 26 % slower): 1,280-byte units, 128 per CU
constexpr int kLdsUnit = 1280;
constexpr int lds_units(int b) { return (b + kLdsUnit - 1) / kLdsUnit; }
static_assert(4 * lds_units(Region<true>::kLds) <= 128, "EXACT: four blocks per CU");
static_assert(7 * lds_units(Region<false>::kLds) <= 128 && 7 * Region<false>::kLds <= 160000,
              "common: seven blocks (28 waves) per CU");
// pointer-cache slots: every pointer the record loop stores through is read
// from LDS where it is used, so none is held in scalar registers across the
// loop (the kernel's arguments no longer spill into VGPR lanes, whose
// restores are VALU instructions)
constexpr int kPNormCig = 10, kPCigOff = 11, kPOvf = 12, kPOvfCount = 13, kPXlist = 14, kPXcount = 15;
constexpr int kPD = 16, kPE = 17, kPSeq = 18, kPQual = 19, kPStatus = 20, kPInfo = 21, kPParams = 22, kPSbase = 23;
constexpr int kPE1000 = 24, kPRows = 25, kNPtrs = 26;
}  // namespace fk

template <int NDW>
struct FastStage {
    uint32_t vb[NDW], vq[NDW];             // raw base / quality bytes, dword u * 64 + lane of the record
    uint2 rm;                              // this lane's read meta (lane < R)
    uint32_t mv;                           // dword `lane` of a later record's descriptor (lanes < 8)
};

// issue a record's loads (consumed by the next record's stage_codes).  Buffer
// loads on a resource based at the record's first byte: dword u * 64 + lane at
// voffset 4 lane + immediate 256 u, no per-lane address arithmetic, and bytes
// past the end of the array read as 0 (range-checked) instead of faulting.
template <bool DUPLEX, int NDW>
__device__ __forceinline__ void fast_load(const FastArgs &a, RecMeta m, const RecMeta *mlater, int lane,
                                          FastStage<NDW> &st) {
    const int ndw = (int)(m.w >> 15);
    if (DCR_ABL == 6 && !DUPLEX) m.base_al = a.meta[0].base_al;   // diagnostic: cache-resident bytes
    // range: the array's last dword read whole (device allocations are padded
    // to at least 16 bytes, as the 16-byte-aligned staging already assumes)
    const int64_t left = ((a.nbytes + 3) & ~(int64_t)3) - m.base_al;
    const int nrec = (int)min(left, (int64_t)0x7FFFFFF0);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)(a.gb + m.base_al), (short)0, nrec,
                                                                        0x00020000);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void *)(a.gq + m.base_al), (short)0, nrec,
                                                                        0x00020000);
#pragma unroll
    for (int u = 0; u < NDW; ++u) {
        if (u * kWave < ndw) {
            st.vb[u] = __builtin_amdgcn_raw_buffer_load_b32(rb, 4 * lane + 256 * u, 0, DCR_LCPOL);
            st.vq[u] = __builtin_amdgcn_raw_buffer_load_b32(rq, 4 * lane + 256 * u, 0, DCR_LCPOL);
        }
    }
    const int R = (int)(m.w & 127u);
    if (DCR_ABL == 6 && !DUPLEX) m.g0 = a.meta[0].g0;
    st.rm = a.rmeta[m.g0 + min(lane, R - 1)];
    st.mv = ((const uint32_t *)mlater)[lane & 7];
}

// Four element codes from four bases and qualities (SWAR).  The class comes
// from a byte permute indexed by (b >> 1) & 7, distinct for A C T G N; a second
// permute gives the letter of that index, and a byte that differs from it is
// not a valid nucleotide (:580-585): flagged in `bad` (the record then goes to
// the general kernel, which reproduces the exit), as are a quality > 122 and a
// kept base below fast_qlo.  Single-strand inputs mask qual < min_base_quality
// to class N keeping the quality (:280): v_lerp_u8 computes (q + 256 - m) >> 1,
// whose bit 7 is q >= m.  code = (k << 11) | 16 (q + k) per byte.
// The single-strand mask (qual < min_base_quality -> 'N' keeping the quality,
// :280) is folded into the table: the rows of (base class, quality below the
// mask) ARE 'N' rows.  An invalid letter is flagged even when its quality is
// masked (the reference would read it as 'N'): its record takes the general
// kernel, which reproduces that exactly.  LO: some unmasked quality lies below
// fast_qlo, so the bytes are checked for it (not with the default flags).
// NARROW (the common instantiation's table of 8-byte rows): code = (k << 10) | 8 (q + k).
template <bool DUPLEX, bool LO, bool NARROW>
__device__ __forceinline__ uint2 make_codes4(uint32_t B, uint32_t Q, uint32_t kq, uint32_t kqlo, uint32_t &bad) {
    const uint32_t h = (B >> 1) & 0x07070707u;
    const uint32_t k = __builtin_amdgcn_perm(0u, 0x04020301u, h);                 // A1 C3 T2 G4 . . . N0
    const uint32_t x = B ^ __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, h);   // 0 for a valid letter
    uint32_t lo = 0;
    if (LO) {
        lo = ~(Q + kqlo) & __builtin_amdgcn_perm(0u, 0xFFFFFFFFu, h);            // bit 7: a base with q < fast_qlo
        if (!DUPLEX) {
            const uint32_t L = __builtin_amdgcn_lerp(Q, kq, 0x01010101u);
            lo &= __builtin_amdgcn_perm(L << 8, L, 0x090B080Au);                  // masked bytes are 'N' rows
        }
    }
    bad |= x | ((((Q + 0x05050505u) | Q) | lo) & 0x80808080u);
    const uint32_t w = k + Q;                                                     // per byte, <= 126
    const uint32_t hi = NARROW ? ((w >> 5) & 0x03030303u) | (k << 2) : ((w >> 4) & 0x07070707u) | (k << 3);
    const uint32_t lw = NARROW ? (w << 3) & 0xF8F8F8F8u : (w << 4) & 0xF0F0F0F0u;
    return make_uint2(__builtin_amdgcn_perm(hi, lw, 0x05010400u), __builtin_amdgcn_perm(hi, lw, 0x07030602u));
}

template <int NT>
struct Evidence {
    uint64_t llr[NT];      // 16-bit fields A T C G: sums of the class rows' rounded-down LLR terms
    uint32_t cnt[NT];      // 6-bit counters: N A T C G
};

// The narrow evidence (common instantiation, records of at most 15 reads):
// one 8-byte table row per (class, quality), the class's 16-bit field holding
// llr8 << 4 | 1 (llr8 = the row's LLR term in 1/u nat, rounded down, <= 273,
// u = 16 with the default parameters, 8 or 4 for extreme qualities;
// the low 4 bits count the class's rows), 'N' and masked rows 0.  A column's
// sum is then one u64: field k = L_k << 4 | n_k, with no carry between fields
// (15 rows: 15 * 273 < 2^12, n_k <= 15), and comparing fields compares L_k.
template <int NT>
struct Evidence8 {
    uint32_t lo[NT], hi[NT];   // fields A T | C G (two 32-bit halves: no 64-bit adds)
};

template <int NT, bool FULL>
__device__ __forceinline__ void run_evidence8(Evidence8<NT> &ev, const uint8_t *lds, int R, uint32_t rmx, int crv,
                                              int lane) {
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) ev.lo[tt] = ev.hi[tt] = 0u;
    if (FULL && DCR_STRIDE) {
        // the reads' stage addresses evenly spaced (reads of one length packed
        // back to back: the C2 shape): a lane's code address is one VGPR
        // stepped by the stride, with no per-read readlane or scalar clamp.
        // The last step's codes of reads R, R + 1 are loaded from past the
        // record and never used (LDS reads past the allocation return 0).
        const int cr0 = readlane(crv, 0);
        const int step = R > 1 ? readlane(crv, 1) - cr0 : 0;
        if (__ballot(lane < R && crv != cr0 + lane * step) == 0) {
            const uint8_t *p = lds + cr0 + 2 * lane;
            auto codes_at = [&](const uint8_t *q, uint32_t (&cd)[NT]) {
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) cd[tt] = *(const uint16_t *)(q + 128 * tt);
            };
            uint32_t c0[NT], c1[NT];
            codes_at(p, c0);
            codes_at(p + step, c1);
            p += 2 * step;
            int r = 0;
            for (; r + 2 <= R; r += 2) {
                uint2 f0[NT], f1[NT];
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    f0[tt] = *(const uint2 *)(lds + c0[tt]);
                    f1[tt] = *(const uint2 *)(lds + c1[tt]);
                }
                codes_at(p, c0);
                codes_at(p + step, c1);
                p += 2 * step;
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    ev.lo[tt] += f0[tt].x + f1[tt].x;
                    ev.hi[tt] += f0[tt].y + f1[tt].y;
                }
            }
            if (r < R) {
#pragma unroll
                for (int tt = 0; tt < NT; ++tt) {
                    const uint2 f0 = *(const uint2 *)(lds + c0[tt]);
                    ev.lo[tt] += f0.x;
                    ev.hi[tt] += f0.y;
                }
            }
            return;
        }
    }
    auto codes = [&](int r, uint32_t (&cd)[NT]) {
        const int rr = min(r, R - 1);
        const int cr = readlane(crv, rr);          // stage address of the read's column 0
        if (FULL) {
            const uint8_t *p = lds + cr + 2 * lane;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) cd[tt] = *(const uint16_t *)(p + 128 * tt);
        } else {
            const int x = readlane((int)rmx, rr);
            const int col = x & 255, len = (x >> 8) & 255;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                const int t = 64 * tt + lane;
                const uint32_t a = (uint32_t)(t - col) < (uint32_t)len ? (uint32_t)(cr + 2 * t) : (uint32_t)fk::kSent;
                cd[tt] = *(const uint16_t *)(lds + a);
            }
        }
    };
    auto rows = [&](const uint32_t (&cd)[NT], uint2 (&f)[NT]) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) f[tt] = *(const uint2 *)(lds + cd[tt]);
    };
    // two reads per step: no field carries (above), so each 32-bit half is a
    // three-input add (v_add3_u32)
    auto add2 = [&](const uint2 (&f)[NT], const uint2 (&g)[NT]) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            ev.lo[tt] += f[tt].x + g[tt].x;
            ev.hi[tt] += f[tt].y + g[tt].y;
        }
    };
    uint32_t c0[NT], c1[NT];
    codes(0, c0);
    codes(1, c1);
    int r = 0;
    for (; r + 2 <= R; r += 2) {
        uint2 f0[NT], f1[NT];
        rows(c0, f0);
        rows(c1, f1);
        uint32_t n0[NT], n1[NT];
        codes(r + 2, n0);
        codes(r + 3, n1);
        add2(f0, f1);
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            c0[tt] = n0[tt];
            c1[tt] = n1[tt];
        }
    }
    if (r < R) {
        uint2 f0[NT];
        rows(c0, f0);
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            ev.lo[tt] += f0[tt].x;
            ev.hi[tt] += f0[tt].y;
        }
    }
}

// Evidence sums in read order (integer, so the order is free).  FULL: every
// read covers every column (the C2 shape), so a read's codes are one base
// address plus immediate offsets; otherwise a column outside the read loads
// the pad sentinel.  Two reads per step: the table rows of reads r and r + 1
// are in flight together while the codes of r + 2 and r + 3 are read.
template <int NT, bool FULL>
__device__ __forceinline__ void run_evidence(Evidence<NT> &ev, const uint8_t *lds, int R, uint32_t rmx, int crv,
                                             int lane) {
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        ev.llr[tt] = 0;
        ev.cnt[tt] = 0;
    }
    auto codes = [&](int r, uint32_t (&cd)[NT]) {
        const int rr = min(r, R - 1);
        const int cr = readlane(crv, rr);          // stage address of the read's column 0
        if (FULL) {
            const uint8_t *p = lds + cr + 2 * lane;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) cd[tt] = *(const uint16_t *)(p + 128 * tt);
        } else {
            const int x = readlane((int)rmx, rr);
            const int col = x & 255, len = (x >> 8) & 255;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                const int t = 64 * tt + lane;
                const uint32_t a = (uint32_t)(t - col) < (uint32_t)len ? (uint32_t)(cr + 2 * t) : (uint32_t)fk::kSent;
                cd[tt] = *(const uint16_t *)(lds + a);
            }
        }
    };
    auto rows = [&](const uint32_t (&cd)[NT], uint4 (&f)[NT]) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) f[tt] = *(const uint4 *)(lds + cd[tt]);
    };
    auto add = [&](const uint4 (&f)[NT]) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            ev.llr[tt] += ((uint64_t)f[tt].y << 32) | f[tt].x;
            ev.cnt[tt] += f[tt].z;
        }
    };
    // two reads' rows at once: no 16-bit field ever reaches 2^16 (at most 63
    // rows of at most 16 ln(5 10^12.2) < 476 each), so no carry crosses the
    // two 32-bit halves and each half is a three-input add (v_add3_u32)
    auto add2 = [&](const uint4 (&f)[NT], const uint4 (&g)[NT]) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            const uint32_t lo = (uint32_t)ev.llr[tt] + f[tt].x + g[tt].x;
            const uint32_t hi = (uint32_t)(ev.llr[tt] >> 32) + f[tt].y + g[tt].y;
            ev.llr[tt] = ((uint64_t)hi << 32) | lo;
            ev.cnt[tt] += f[tt].z + g[tt].z;
        }
    };
    uint32_t c0[NT], c1[NT];
    codes(0, c0);
    int r = 0;
    if constexpr (NT <= 3) {
    codes(1, c1);
    for (; r + 2 <= R; r += 2) {
        uint4 f0[NT], f1[NT];
        rows(c0, f0);
        rows(c1, f1);
        uint32_t n0[NT], n1[NT];
        codes(r + 2, n0);
        codes(r + 3, n1);
        add2(f0, f1);
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            c0[tt] = n0[tt];
            c1[tt] = n1[tt];
        }
    }
    }
    // one read per step (NT = 4 keeps fewer rows in flight)
    for (; r < R; ++r) {
        uint4 f0[NT];
        rows(c0, f0);
        uint32_t n0[NT];
        if (r + 1 < R) codes(r + 1, n0);
        add(f0);
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) c0[tt] = n0[tt];
    }
}

// destination of record scalar k (lane k: field k of dcr_out) as one word:
// pointer | shift << 56, address = pointer + (index << shift), index = the
// record (the output column offset for k = 9, the CIGAR).  Kept in LDS (read
// once per record) rather than in registers for the whole kernel.
__device__ __forceinline__ uint64_t scalar_dest(const dcr_out &O, int k) {
    const uint64_t shift = (k == 7 || k == 8) ? 3u : 2u;
    const uint8_t *p;
    switch (k) {
    case 0: p = (const uint8_t *)O.pos; break;
    case 1: p = (const uint8_t *)O.mapq; break;
    case 2: p = (const uint8_t *)O.len; break;
    case 3: p = (const uint8_t *)O.n_cig; break;
    case 4: p = (const uint8_t *)O.n_de; break;
    case 5: p = (const uint8_t *)O.D; break;
    case 6: p = (const uint8_t *)O.M; break;
    case 7: p = (const uint8_t *)O.E; break;
    case 8: p = (const uint8_t *)O.E + 4; break;
    default: p = (const uint8_t *)O.cigar; break;
    }
    return (uint64_t)(uintptr_t)p | (shift << 56);
}

// a pointer cached in LDS at kernel start, as a per-lane value (one
// broadcast LDS read; stores through it take a 64-bit VGPR address)
// (global address space: stores through a pointer read back from LDS would
// otherwise be flat stores, which count in lgkmcnt too, so every later LDS
// wait of the record loop also waited for them)
#if defined(__HIP_DEVICE_COMPILE__)
#define DCR_G __attribute__((address_space(1)))
#define DCR_C __attribute__((address_space(4)))   // constant: uniform loads become scalar loads
#else
#define DCR_G                  // the host pass only parses device functions
#define DCR_C
#endif
template <class Tp>
__device__ __forceinline__ DCR_G Tp *lds_vptr(const uint8_t *lds, int slot) {
    return (DCR_G Tp *)(uintptr_t)(*(const uint64_t *)(lds + fk::kPtrs + 8 * slot));
}

// a record's failure status from the fast kernel: status byte and zeroed
// scalars as write_status_at writes them, lane k storing field k
__device__ __forceinline__ void fast_status(const uint8_t *lds, int64_t rec, int st, int lane) {
    if (lane < 9) {
        const uint64_t pw = *(const uint64_t *)(lds + fk::kPtrs + 8 * lane);
        *(DCR_G uint32_t *)((pw & 0x00FFFFFFFFFFFFFFull) + ((uint64_t)rec << (pw >> 56))) = 0u;
    } else if (lane == 10) {
        lds_vptr<uint8_t>(lds, fk::kPStatus)[rec] = (uint8_t)st;
    }
}

// a pointer cached in LDS, as a wave-uniform global pointer (stores through
// it take an SGPR base and a per-lane 32-bit offset: no 64-bit address VALU)
template <class Tp>
__device__ __forceinline__ DCR_G Tp *lds_sgptr(const uint8_t *lds, int slot) {
    const uint64_t v = *(const uint64_t *)(lds + fk::kPtrs + 8 * slot);
    const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (DCR_G Tp *)(uintptr_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// v_writelane: an SGPR value into one lane of a VGPR (one VALU, no compare)
template <int L>
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t x) {
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(L));
    return v;
}

// a pointer cached in LDS at kernel start (rare paths), as a scalar
template <class Tp>
__device__ __forceinline__ Tp *lds_ptr(const uint8_t *lds, int slot) {
    const uint64_t v = *(const uint64_t *)(lds + fk::kPtrs + 8 * slot);
    const int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (Tp *)(uintptr_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// diagnostic phase clock (DCR_STAMP builds): cycles per phase, summed per wave
struct Stamps {
    uint64_t t_prev = 0;
    uint64_t acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void mark(int k) {
        if (DCR_STAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (k > 0) acc[k - 1] += now - t_prev;
            t_prev = now;
        }
    }
};

// phase 0: element codes of the prefetched bytes into the stage (dword d of
// the record's bytes -> four codes at stage + 8 d); returns the lanes'
// invalid-input flags
template <bool DUPLEX, bool LO, bool NARROW, int NDW>
__device__ __forceinline__ uint32_t stage_codes(const FastArgs &a, const RecMeta &m, const FastStage<NDW> &st,
                                                uint8_t *lds, int stage_addr, int lane) {
    const int ndw = (int)(m.w >> 15);
    uint32_t bad = 0;
    uint8_t *sp = lds + stage_addr + 8 * lane;       // group u at the immediate offset 512 u
#pragma unroll
    for (int u = 0; u < NDW; ++u) {
        if (u * kWave < ndw) {
            // every lane of the group converts and stores (the stage holds
            // NDW * 64 dwords' codes); a dword past the record's is not
            // checked: only the group holding the record's last dword
            // compares lanes (a uniform branch, no per-lane one)
            uint32_t b = 0;
            const uint2 c = LO ? make_codes4<DUPLEX, true, NARROW>(st.vb[u], st.vq[u], a.kq, a.kqlo, b)
                               : make_codes4<DUPLEX, false, NARROW>(st.vb[u], st.vq[u], a.kq, a.kqlo, b);
            const int lim = (u + 1) * kWave <= ndw ? kWave : ndw - u * kWave;   // uniform
            bad |= lane < lim ? b : 0u;
            *(uint2 *)(sp + 512 * u) = c;
        }
    }
    return bad;
}

// the general kernel takes the record: it reads the preprocessed reads (info,
// normalised runs); pointers from the LDS cache
template <bool DUPLEX>
__device__ __forceinline__ void send_to_general_(int rec, int g0, int R, uint32_t rmx, const uint8_t *lds, int lane) {
    if (!DUPLEX && lane < R) {
        const int tl = ((int)rmx >> 8) & 255;
        DCR_G uint32_t *norm_cig = lds_sgptr<uint32_t>(lds, fk::kPNormCig);
        const DCR_G int32_t *cig_off = lds_sgptr<const int32_t>(lds, fk::kPCigOff);
        if (tl > 0) norm_cig[cig_off[g0 + lane]] = (uint32_t)tl << 4;   // one M run
    }
    // global (not generic) pointers: a flat store or atomic left pending on
    // this rare path made the record loop's waitcnt model assume FLAT events
    // at its header, so the staging's wait for the prefetch was a vmcnt(0)
    // that also waited for the previous record's stores
    DCR_G int *ovf = lds_sgptr<int>(lds, fk::kPOvf);
    DCR_G int *ovf_count = lds_sgptr<int>(lds, fk::kPOvfCount);
    if (lane == 0) {
        const int idx = __hip_atomic_fetch_add(ovf_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ovf[idx] = rec;
    }
}
template <bool DUPLEX>
__device__ __forceinline__ void send_to_general(const FastArgs &a, const RecMeta &m, uint2 rm, const uint8_t *lds,
                                                int lane) {
    const int R = (int)(m.w & 127u);
    if (!DUPLEX && !a.want_info && lane < R) {
        // trim_record left the read info out (nobody asked for it), but the
        // general kernel reads it: the same values trim_record writes
        const int tl = ((int)rm.x >> 8) & 255;
        dcr_read_info inf;
        inf.seq_start = m.base_al + (int64_t)rm.y;
        inf.len = tl;
        inf.n_cig = tl > 0 ? 1 : 0;
        inf.status = tl > 0 ? DCR_ST_OK : DCR_ST_INDEX_ERROR;
        inf.has_ins = 0;
        lds_vptr<dcr_read_info>(lds, fk::kPInfo)[m.g0 + lane] = inf;
    }
    send_to_general_<DUPLEX>(m.rec, m.g0, R, rm.x, lds, lane);
}

struct Staged {
    uint2 rm;      // the lane's read meta (single-strand: length after the 3' trim)
    int T;         // columns (:458-459, on the trimmed reads)
    int state;     // 0 consensus here, 1 general kernel, 2 finished (status written),
                   // 3 consensus here, 3' trim checked after the evidence (finish_record)
    uint32_t fl;   // state 3: the lane's read's first | last element code << 16 (loads in flight)
};

// trim_3prime_N (:292-325) on the staged codes: drop each read's trailing 'N'
// (sequenced, or masked below min_base_quality, :280): codes of class N, from
// the end.  T shrinks only when every read reaching it lost its tail; a read
// left empty ends the record with the status compress_cigarlist([]) raises
// (:740 via :322).  Returns 2 when that status was written, else 0.
// an element's table row is an 'N' row (class N, or a quality masked below
// min_base_quality, :280): wide rows count it in the N counter, narrow rows
// are all zero
template <bool NARROW>
__device__ __forceinline__ bool row_is_n(const uint8_t *lds, uint32_t code) {
    if (NARROW) {
        const uint2 r = *(const uint2 *)(lds + code);
        return (r.x | r.y) == 0u;
    }
    return (*(const uint32_t *)(lds + code + 8) & 63u) != 0u;
}

template <bool DUPLEX, bool NARROW>
__device__ __forceinline__ int trim_walk(const FastArgs &a, const RecMeta &m, uint2 &rm, int &T, const uint8_t *lds,
                                         int stage_addr, int lane) {
    const int R = (int)(m.w & 127u);
    const int x = (int)rm.x, y = (int)rm.y;
    const int col = x & 255;
    int tl = lane < R ? (x >> 8) & 255 : 0;
    bool go = tl > 0;
    while (__ballot(go)) {
        if (go) {
            const uint32_t code = *(const uint16_t *)(lds + stage_addr + 2 * (y + tl - 1));
            // an 'N' row: sequenced 'N' or a masked quality (:280, folded into the table)
            if (row_is_n<NARROW>(lds, code)) --tl; else go = false;
            go = go && tl > 0;
        }
    }
    if (lane < R && (a.want_info || tl == 0)) {
        dcr_read_info inf;
        inf.seq_start = m.base_al + y;
        inf.len = tl;
        inf.n_cig = tl > 0 ? 1 : 0;
        inf.status = tl > 0 ? DCR_ST_OK : DCR_ST_INDEX_ERROR;   // compress_cigarlist([]) :740 via :322
        inf.has_ins = 0;
        lds_vptr<dcr_read_info>(lds, fk::kPInfo)[m.g0 + lane] = inf;
    }
    rm.x = (rm.x & ~0xFF00u) | ((uint32_t)tl << 8);
    if (__ballot(lane < R && col + tl == T) == 0) T = wave_max(lane < R ? col + tl : 0);
    if (__ballot(lane < R && tl == 0)) {
        fast_status(lds, m.rec, DCR_ST_PREP | DCR_ST_INDEX_ERROR, lane);
        return 2;
    }
    return 0;
}

// after the codes: 3' trim (single-strand), read info, T; invalid input -> general
//
// QUICK (the common instantiation, read info not requested): the trim cannot
// change a DECIDED column.  A trimmed base is an 'N' row either way (class N,
// or a base masked below min_base_quality): its LLR term is 0 and it counts
// as 'N' in d and e (:1001, :1011), exactly as the padding 'N' that replaces
// it.  So the trim matters only when it empties a read (compress_cigarlist([])
// :740 via :322), when it shrinks T (every read reaching the last column ends
// in 'N'), or for the products of undecided columns (the pad quality is 2),
// which the EXACT instantiation recomputes from scratch with the full trim.
// A record whose reads all span its T columns (the C2 shape) is left to
// finish_record (state 3): both conditions show in the evidence counts it
// builds anyway (every read ends at column T - 1 and starts at column 0), so
// no code is read back here.  Otherwise QUICK reads each read's first and
// last element only: a read whose last element is a base keeps its length,
// one whose first element is a base keeps at least one; when some read
// ending at T ends in a base, T stays.  Anything else (and invalid input,
// whose record the general kernel takes with the trimmed lengths) runs the
// full trim.
template <bool DUPLEX, bool QUICK>
__device__ __forceinline__ Staged trim_record(const FastArgs &a, const RecMeta &m, uint2 rm, uint32_t bad,
                                              const uint8_t *lds, int stage_addr, int lane) {
    Staged s;
    const int R = (int)(m.w & 127u);
    s.T = (int)((m.w >> 7) & 255u);
    s.state = 0;
    const bool any_bad = __ballot(bad != 0) != 0;
    if (!DUPLEX) {
        const int x = (int)rm.x, y = (int)rm.y;
        const int col = x & 255;
        const int tl = lane < R ? (x >> 8) & 255 : 0;
        bool full = true;
        if (QUICK && !a.want_info && !any_bad) {
            if (DCR_TRIM2 && __ballot(lane < R && (col != 0 || tl != s.T)) == 0) {
                // the first / last codes are only loaded here; finish_record
                // reads them after the evidence, so no round trip is waited on
                lds_fence();
                const int yy = lane < R ? y : 0;
                const uint32_t cf = *(const uint16_t *)(lds + stage_addr + 2 * yy);
                const uint32_t cl = *(const uint16_t *)(lds + stage_addr + 2 * (yy + s.T - 1));
                s.fl = cf | cl << 16;
                s.rm = rm;
                s.state = 3;
                return s;
            }
            lds_fence();
            bool lastN = true, firstN = true;
            if (tl > 0) {
                const uint32_t cl = *(const uint16_t *)(lds + stage_addr + 2 * (y + tl - 1));
                const uint32_t cf = *(const uint16_t *)(lds + stage_addr + 2 * y);
                lastN = row_is_n<QUICK>(lds, cl);
                firstN = row_is_n<QUICK>(lds, cf);
            }
            full = __ballot(lane < R && lastN && firstN) != 0 || __ballot(lane < R && col + tl == s.T && !lastN) == 0;
        }
        if (full) {
            lds_fence();
            s.state = trim_walk<DUPLEX, QUICK>(a, m, rm, s.T, lds, stage_addr, lane);
        }
    }
    s.rm = rm;
    if (s.state == 0 && any_bad) s.state = 1;
    return s;
}

// k / 1000 correctly rounded for 0 <= k <= 1000 (numpy's round(x, 3) divides
// rint(1000 x) by 1000): the product with 0.001 and one fma correction,
// checked exhaustively over that range (tests/test_fast_math.py)
__device__ __forceinline__ double div1000(int k) {
    const double kd = (double)k;
    const double q = kd * 0.001;
    return __builtin_fma(__builtin_fma(-q, 1000.0, kd), 0.001, q);
}

// products, finalize, outputs of a staged record of T <= 64 NT columns.
// Returns false (nothing written) when the record has a column the bound does
// not decide and this is not the EXACT instantiation: the caller queues it for
// the EXACT kernel, which computes those columns in the reference's arithmetic.
// finish_record's outcomes: the caller queues the record for the EXACT
// instantiation / the record's row was written (or, EXACT, its outputs) /
// a status was written (nothing else to do)
constexpr int kFinQueue = 0, kFinDone = 1, kFinStatus = 2;

// a decided record's row (lanes 0-3), held until the next record is staged (DCR_DEFER)
struct Pend {
    uint32_t v;
};

template <bool DUPLEX, int NT, bool EXACT>
__device__ __forceinline__ int finish_record(const FastArgs &a, const RecMeta &m, const Staged &sg, uint8_t *lds,
                                             const int stage_addr, const int ov_addr, const int rm_addr, const int list_addr,
                                             const int lane,
                                             Stamps &sp, const double2 *xt, const uint32_t *r1, const double *qt,
                                             const int fi, Pend &pd) {
    const int64_t rec = m.rec;
    const int64_t off = m.off;
    const int R = (int)(m.w & 127u);
    int T = sg.T;
    const int minpos = m.minpos;
    uint2 rm = sg.rm;
    lds_fence();
    if (DCR_ABL == 1) {                 // diagnostic: staging only
        if (lane == 0) a.O.pos[rec] = *(const uint16_t *)(lds + stage_addr + 2 * (int)(rm.y & 7)) + m.d0;
        return kFinDone;
    }
    const int colr = (int)(rm.x & 255u), lenr = (int)((rm.x >> 8) & 255u);
    const int crv = stage_addr + 2 * ((int)rm.y - colr);
    Evidence<NT> ev;                     // EXACT: wide rows
    Evidence8<NT> ev8;                   // common: narrow rows (R <= 15)
    const bool full_cols = __ballot(lane < R && (colr != 0 || lenr < T)) == 0;
    if constexpr (EXACT) {
        if (full_cols) run_evidence<NT, true>(ev, lds, R, rm.x, crv, lane);
        else run_evidence<NT, false>(ev, lds, R, rm.x, crv, lane);
    } else {
        if (full_cols) run_evidence8<NT, true>(ev8, lds, R, rm.x, crv, lane);
        else run_evidence8<NT, false>(ev8, lds, R, rm.x, crv, lane);
    }
    sp.mark(5);                          // [4] products
    if (DCR_ABL == 2) {                 // diagnostic: staging + products
        uint32_t x = 0;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt)
            x += EXACT ? (uint32_t)ev.llr[tt] ^ (uint32_t)(ev.llr[tt] >> 32) ^ ev.cnt[tt]
                       : ev8.lo[tt] ^ ev8.hi[tt];
        if (lane == 0) a.O.pos[rec] = (int)x;
        return kFinDone;
    }
    if (!EXACT && !DUPLEX && sg.state == 3) {
        // the 3' trim of a record whose reads all span [0, T) (trim_record,
        // QUICK): a read whose last element is a base keeps its length, one
        // whose first element is a base keeps at least one, and T stays when
        // some read ends in a base; otherwise the caller trims and comes back.
        // An element is an 'N' row when its class is N or its quality is
        // masked (:280): narrow code bank 0, or (code >> 3 & 127) - bank < min_bq.
        auto is_n = [&](uint32_t c) {
            const uint32_t k = c >> 10;
            return k == 0u || (int)(((c >> 3) & 127u) - k) < a.minbq;
        };
        const bool lastN = is_n(sg.fl >> 16), firstN = is_n(sg.fl & 0xFFFFu);
        if (__ballot(lane < R && lastN && firstN) != 0 || __ballot(lane < R && !lastN) == 0) {
            // rare: the full trim (the evidence is unchanged, T may shrink)
            if (trim_walk<DUPLEX, true>(a, m, rm, T, lds, stage_addr, lane) == 2) return kFinStatus;
        }
    }
    // decide every tile in registers (integer, straight-line): call, depth d
    // and errors e (:970-1021) as the column word d | e << 6 | call << 12
    const double *invd = (const double *)(lds + fk::kInvD);
    uint8_t *ov = lds + ov_addr;
    uint32_t und = 0;                  // bit tt: the lane's live column is not decided
    // the common instantiation stores every column as it is decided (lane =
    // column, uniform bases + 32-bit lane offsets, no LDS round trip): 'N' /
    // quality 0 past T up to the region's end (the untrimmed T rounded to 16
    // columns; d / e there are don't-care).  A record that turns out to have
    // an undecided column is queued and the EXACT kernel rewrites all of it.
    // The column words go to ov only where they are read again: EXACT, and
    // the double mean of records of more than 16 reads.
    const int T16 = ((int)((m.w >> 7) & 255u) + 15) & ~15;
    // the common instantiation's column stores: buffer stores on resources
    // based at the record's region and sized to it (T16 columns), so the last
    // tile's lanes past the region are dropped by the range check instead of
    // branching around them (no exec-mask branch in the loop over tiles)
    // (made where they are used, so their 16 scalar registers are not held
    // across the tile loop; unused in the EXACT instantiation)
// (DCR_ABL 7, diagnostic: every record's columns stored over the first 4,096
// columns of the arrays, cache-resident: the stores without their HBM traffic)
#define DCR_OFF_ (DCR_ABL == 7 ? (off & 4095) : DCR_ABL == 8 ? (off & ~(int64_t)63) : off)
#define DCR_RSRC_D __builtin_amdgcn_make_buffer_rsrc((void *)(a.O.d + DCR_OFF_), (short)0, 2 * T16, 0x00020000)
#define DCR_RSRC_E __builtin_amdgcn_make_buffer_rsrc((void *)(a.O.e + DCR_OFF_), (short)0, 2 * T16, 0x00020000)
#define DCR_RSRC_S __builtin_amdgcn_make_buffer_rsrc((void *)(a.O.seq + DCR_OFF_), (short)0, T16, 0x00020000)
#define DCR_RSRC_Q __builtin_amdgcn_make_buffer_rsrc((void *)(a.O.qual + DCR_OFF_), (short)0, T16, 0x00020000)
    // more reads than r_safe: L_b may underflow (fast_constants), no column is decided here
    const bool force = R > a.r_safe;
    int dmax = -1, dmin = 0x7fffffff;
    // sum over the lane's live columns of e * 720720 / d: the mean's numerator
    // in fixed point, exact for depths <= 16 (720720 = lcm(1..16); < 2^32 over
    // 240 columns)
    uint32_t fx = 0;
    int fxd = 0;                       // EXACT: the exact columns' change to fx (their e, d == 0 -> e/d = 1)
    const uint32_t *m720 = (const uint32_t *)(lds + fk::kM720);
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        const int t = 64 * tt + lane;
        const bool live = tt < NT - 1 || t < T;                      // only the last tile is partial
        const uint32_t lo = EXACT ? (uint32_t)ev.llr[tt] : ev8.lo[tt];
        const uint32_t hi = EXACT ? (uint32_t)(ev.llr[tt] >> 32) : ev8.hi[tt];
        // (A, C) and (T, G) fields as 16-bit pairs: one packed max / min gives both halves
        const u16x2 P1 = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi, lo, 0x05040100u));
        const u16x2 P2 = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi, lo, 0x07060302u));
        const u16x2 M = __builtin_elementwise_max(P1, P2), N = __builtin_elementwise_min(P1, P2);
        const uint32_t top = max((uint32_t)M.x, (uint32_t)M.y);
        const uint32_t sec = max(min((uint32_t)M.x, (uint32_t)M.y), max((uint32_t)N.x, (uint32_t)N.y));   // second largest
        uint32_t kb = (uint32_t)P1.y == top ? 2u : 3u;               // the first largest ("ATCG")
        kb = (uint32_t)P2.x == top ? 1u : kb;
        kb = (uint32_t)P1.x == top ? 0u : kb;
        uint32_t Lb, L2;
        int d, nb;
        if constexpr (EXACT) {
            const uint32_t cnt = ev.cnt[tt];
            Lb = top;
            L2 = sec;
            d = R - (int)(cnt & 63u);                                             // rows that are not 'N'
            nb = (int)__builtin_amdgcn_ubfe(cnt, 6u * kb + 6u, 6u);
        } else {
            // fields L << 4 | n: a decided column's call has the unique largest
            // L, so its field is the largest and carries its row count; the
            // rows that are not 'N' are the four counts (one byte permute, the
            // low nibbles, a byte sum)
            Lb = top >> 4;
            L2 = sec >> 4;
            nb = (int)(top & 15u);
            d = (int)__builtin_amdgcn_sad_u8(__builtin_amdgcn_perm(hi, lo, 0x06040200u) & 0x0F0F0F0Fu, 0u, 0u);
        }
        const int e = R - nb;                                                     // rows that differ from the call
        // decided: LLR_b - max(LLR_k, 0) >= (Lb - L2 - (d - nb)) / u >= margin / u
        // (u = 16 wide; narrow: fast_constants' unit)
        const bool undecided = (int)(Lb - L2) - (d - nb) < (EXACT ? a.t16 : a.t8) || force;
        und |= (uint32_t)(live && undecided) << tt;
        if (EXACT) *(uint16_t *)(ov + 2 * t) = (uint16_t)((uint32_t)d | ((uint32_t)e << 6) | (kb << 12));
        if (!EXACT && DCR_ABL != 5) {
            // "ATCG"[call] and maxQ; past T (last tile only) 'N' / 0
            // maxQ made where it is stored (opaque): a VGPR copy hoisted out of
            // the record loop was spilled to scratch, and its reload's
            // vmcnt(0) waited for the next record's prefetch mid-decision
            uint32_t letter = __builtin_amdgcn_perm(0u, 0x47435441u, kb), qv = (uint32_t)opaque(a.maxq);
            if (tt == NT - 1) {
                letter = t < T ? letter : 0x4Eu;
                qv = t < T ? qv : 0u;
            }
            if (DCR_ST4) {
                // the column word (d | e << 6 | sel << 12, sel = the call or
                // 4: 'N' / quality 0 past T) into the free stage; the stores
                // go four columns per lane once the record is known decided
                const uint32_t sel = tt == NT - 1 && t >= T ? 4u : kb;
                *(uint16_t *)(ov + 2 * t) = (uint16_t)((uint32_t)d | ((uint32_t)e << 6) | (sel << 12));
            } else {
            // the tile's offset as the scalar offset (no per-tile vector add)
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)d, DCR_RSRC_D, 2 * lane, 128 * tt, DCR_SCPOL);
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)e, DCR_RSRC_E, 2 * lane, 128 * tt, DCR_SCPOL);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)letter, DCR_RSRC_S, lane, 64 * tt, DCR_SCPOL);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)qv, DCR_RSRC_Q, lane, 64 * tt, DCR_SCPOL);
            }
        }
        fx += live ? __umul24((uint32_t)e, m720[d]) : 0u;
        dmax = max(dmax, live ? d : -1);
        dmin = min(dmin, live ? d : 0x7fffffff);
    }
    // Columns the bound does not decide get the reference's own arithmetic
    // here (most_likely_nucleotide :594-621 in read order, IEEE binary64, then
    // the quality of :699-709): their call may be masked 'N' and their quality
    // below maxQ.  The kept span then runs from the first to the last column
    // that is not 'N' (:770-790), still one M run (no '+' / '-' rows here).
    int first = 0, last = T - 1;
    sp.mark(12);                         // [11] decision (of [5] finalize)
    const bool exact = __ballot(und) != 0;
    if (!EXACT && exact) return kFinQueue;
    if (!EXACT && DCR_ST4 && DCR_ABL != 5) {
        // d / e / seq / qual four columns per lane (8-, 8-, 4- and 4-byte
        // stores): 4 store instructions per record instead of 4 per tile.
        // The vector memory path pays per instruction (and per lane), not per
        // byte: a C2 record's twelve 1- and 2-byte stores cost the kernel
        // ~20 % (profiles/r06g), range-checked-out ones nothing.
        lds_fence();
        // lanes past the region (4 lane >= T16) are dropped by the resources' range checks
        const uint2 w = *(const uint2 *)(ov + 8 * lane);
        const uint32_t sel = ((w.x >> 12) & 7u) | ((w.x >> 20) & 0x700u) | ((w.y << 4) & 0x70000u) |
                             ((w.y >> 4) & 0x7000000u);
        const uint32_t letters = __builtin_amdgcn_perm(0x4Eu, 0x47435441u, sel);            // "ATCG"[call] or 'N'
        const uint32_t quals = __builtin_amdgcn_perm(0u, (uint32_t)a.maxq * 0x01010101u, sel); // maxQ or 0
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i dv = {(int)(w.x & 0x003F003Fu), (int)(w.y & 0x003F003Fu)};
        const v2i evv = {(int)((w.x >> 6) & 0x003F003Fu), (int)((w.y >> 6) & 0x003F003Fu)};
        __builtin_amdgcn_raw_buffer_store_b64(dv, DCR_RSRC_D, 8 * lane, 0, DCR_SCPOL);
        __builtin_amdgcn_raw_buffer_store_b64(evv, DCR_RSRC_E, 8 * lane, 0, DCR_SCPOL);
        __builtin_amdgcn_raw_buffer_store_b32(letters, DCR_RSRC_S, 4 * lane, 0, DCR_SCPOL);
        __builtin_amdgcn_raw_buffer_store_b32(quals, DCR_RSRC_Q, 4 * lane, 0, DCR_SCPOL);
    }
    // exact columns' character | quality << 8, as u16 per column in the wave's
    // read-word LDS (free once the read words are in registers)
    uint16_t *chq = (uint16_t *)(lds + rm_addr);
    if (exact) {
        const dcr_params *P = lds_ptr<const dcr_params>(lds, fk::kPParams);
        const double *qthr = EXACT ? qt : P->qthresh;     // EXACT: LDS copy of the quality table
        bool fail = false;             // '+' / '-' call or int(-inf) quality: general kernel
        if (!DUPLEX && R == 1) {
            // the lane's column results: posterior and 8-bit row counts of A T C G
            Posterior po[NT];
            uint32_t cnt[NT];
            uint32_t tiles = 0;                           // tiles holding an undecided column (uniform)
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) tiles |= (uint32_t)(__ballot((und >> tt) & 1u) != 0) << tt;
            // one read: the column's posterior is a function of its row
            // (class after the mask, raw quality), tabulated per block in
            // the kernel's prologue by the products below and posterior()
            const int cr = readlane(crv, 0);
            const int x = readlane((int)rm.x, 0);
            const int col = x & 255, len = (x >> 8) & 255;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                if (!((tiles >> tt) & 1u)) continue;
                const int t = 64 * tt + lane;
                const uint32_t ad = (uint32_t)(t - col) < (uint32_t)len ? (uint32_t)(cr + 2 * t) : (uint32_t)fk::kSent;
                const uint32_t code = *(const uint16_t *)(lds + ad);
                const uint32_t kc = code >> 11;
                const uint32_t q = ((code >> 4) & 127u) - kc;
                const uint32_t k = (kc == 0 || (int)q < a.minbq) ? 0u : kc;   // as the table's rows
                const uint32_t te = r1[k * 128u + q];
                po[tt].ch = (int)(te & 255u);
                po[tt].q = (int)((te >> 8) & 1023u) - 1;
                po[tt].best = (int)((te >> 18) & 7u);
                po[tt].masked = (te >> 21) & 1u;
                po[tt].overflow = (te >> 22) & 1u;
                cnt[tt] = k ? 1u << (8 * (k - 1)) : 0u;
            }
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                const int t = 64 * tt + lane;
                if ((und >> tt) & 1u) {
                    fail |= po[tt].overflow || (!po[tt].masked && po[tt].best > 3);
                    const uint32_t w = *(const uint16_t *)(ov + 2 * t);
                    const int d = (int)(w & 63u);
                    const int nb = po[tt].best <= 3 ? (int)((cnt[tt] >> (8 * po[tt].best)) & 255u) : 0;
                    const int e = po[tt].masked ? d : R - nb;           // rows != the consensus character
                    fxd += (d == 0 ? 720720 : e * (int)m720[d]) - (int)((w >> 6) & 63u) * (int)m720[d];
                    *(uint16_t *)(ov + 2 * t) = (uint16_t)((uint32_t)d | ((uint32_t)e << 6));
                    chq[t] = (uint16_t)((uint32_t)po[tt].ch | ((uint32_t)po[tt].q << 8));
                }
            }
        } else {
            // the undecided columns compacted (u8 list in LDS, lane order):
            // only ceil(n / 64) tiles of products and posteriors instead of
            // every tile holding one such column (a record with a few
            // undecided columns spread over three tiles ran all three)
            uint8_t *ul = lds + list_addr;
            int nund = 0;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
                const bool u = (und >> tt) & 1u;
                const uint64_t bm = __ballot(u);
                const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                if (u) ul[nund + pre] = (uint8_t)(64 * tt + lane);
                nund += __popcll(bm);
            }
            lds_fence();
            // one compacted tile at a time (a record rarely has more than 64
            // undecided columns): the products in read order (:594-600), two
            // reads per step so their row loads overlap, then the posterior
            for (int ct = 0; 64 * ct < nund; ++ct) {
                const int t = 64 * ct + lane < nund ? (int)ul[64 * ct + lane] : -1;
                double L4[4] = {1.0, 1.0, 1.0, 1.0}, U = 1.0;
                uint32_t cn = 0;
                auto row = [&](int r, uint32_t &k, double2 &f) {
                    const int cr = readlane(crv, r);
                    const int x = readlane((int)rm.x, r);
                    const int col = x & 255, len = (x >> 8) & 255;
                    const uint32_t ad = (uint32_t)(t - col) < (uint32_t)len ? (uint32_t)(cr + 2 * t) : (uint32_t)fk::kSent;
                    const uint32_t code = *(const uint16_t *)(lds + ad);
                    const uint32_t kc = code >> 11;                  // code bank: N 0, A 1, T 2, C 3, G 4
                    const uint32_t q = ((code >> 4) & 127u) - kc;    // raw quality (pad 'N': 2)
                    // class after the mask: the table's 'N' rows are class N
                    // or a quality below min_base_quality (:280)
                    k = (kc == 0 || (int)q < a.minbq) ? 0u : kc;
                    f = xt[q];                                       // (1 - p', p'/5), LDS copy of P's rows
                };
                auto mul = [&](uint32_t k, double2 f) {
                    U = U * f.y;
#pragma unroll
                    for (int i = 0; i < 4; ++i) L4[i] = L4[i] * (k == (uint32_t)(i + 1) ? f.x : f.y);
                    cn += k ? 1u << (8 * (k - 1)) : 0u;
                };
                if (R == 2) {
                    // two reads: the column's outcome from the table (k_r2_table)
                    auto kq = [&](int rr, uint32_t &k, uint32_t &q) {
                        const int cr = readlane(crv, rr);
                        const int x = readlane((int)rm.x, rr);
                        const int col = x & 255, len = (x >> 8) & 255;
                        const uint32_t ad = (uint32_t)(t - col) < (uint32_t)len ? (uint32_t)(cr + 2 * t) : (uint32_t)fk::kSent;
                        const uint32_t code = *(const uint16_t *)(lds + ad);
                        const uint32_t kc = code >> 11;
                        q = (((code >> 4) & 127u) - kc) & 127u;
                        k = (kc == 0 || (int)q < a.minbq) ? 0u : min(kc, 4u);
                    };
                    uint32_t k0, q0, k1, q1;
                    kq(0, k0, q0);
                    kq(1, k1, q1);
                    const uint32_t te = a.r2tab[((k0 * 128u + q0) * 5u + k1) * 128u + q1];
                    cn = (k0 ? 1u << (8 * (k0 - 1)) : 0u) + (k1 ? 1u << (8 * (k1 - 1)) : 0u);
                    Posterior po;
                    po.ch = (int)(te & 255u);
                    po.q = (int)((te >> 8) & 1023u) - 1;
                    po.best = (int)((te >> 18) & 7u);
                    po.masked = (te >> 21) & 1u;
                    po.overflow = (te >> 22) & 1u;
                    if (t >= 0) {
                        fail |= po.overflow || (!po.masked && po.best > 3);
                        const uint32_t w = *(const uint16_t *)(ov + 2 * t);
                        const int d = (int)(w & 63u);
                        const int nb = po.best <= 3 ? (int)((cn >> (8 * po.best)) & 255u) : 0;
                        const int e = po.masked ? d : R - nb;
                        fxd += (d == 0 ? 720720 : e * (int)m720[d]) - (int)((w >> 6) & 63u) * (int)m720[d];
                        *(uint16_t *)(ov + 2 * t) = (uint16_t)((uint32_t)d | ((uint32_t)e << 6));
                        chq[t] = (uint16_t)((uint32_t)po.ch | ((uint32_t)po.q << 8));
                    }
                    continue;
                }
                int r = 0;
                for (; r + 1 < R; r += 2) {
                    uint32_t k0, k1;
                    double2 f0, f1;
                    row(r, k0, f0);
                    row(r + 1, k1, f1);
                    mul(k0, f0);
                    mul(k1, f1);
                }
                if (r < R) {
                    uint32_t k0;
                    double2 f0;
                    row(r, k0, f0);
                    mul(k0, f0);
                }
                const double L[6] = {L4[0], L4[1], L4[2], L4[3], U, U};
                const Posterior po = posterior(L, false, P, qthr, true);
                if (t >= 0) {
                    fail |= po.overflow || (!po.masked && po.best > 3);
                    const uint32_t w = *(const uint16_t *)(ov + 2 * t);
                    const int d = (int)(w & 63u);
                    const int nb = po.best <= 3 ? (int)((cn >> (8 * po.best)) & 255u) : 0;
                    const int e = po.masked ? d : R - nb;               // rows != the consensus character
                    fxd += (d == 0 ? 720720 : e * (int)m720[d]) - (int)((w >> 6) & 63u) * (int)m720[d];
                    *(uint16_t *)(ov + 2 * t) = (uint16_t)((uint32_t)d | ((uint32_t)e << 6));
                    chq[t] = (uint16_t)((uint32_t)po.ch | ((uint32_t)po.q << 8));
                }
            }
        }
        sp.mark(11);                     // [10] products and posteriors (of [5] finalize)
        lds_fence();
        // kept span: first / last column whose character is not 'N'
        int fst = 0x7fffffff, lst = -1;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            const int t = 64 * tt + lane;
            const bool live = tt < NT - 1 || t < T;
            const bool isn = (und >> tt) & 1u ? (chq[t] & 255u) == 'N' : false;
            if (live && !isn) {
                fst = min(fst, t);
                lst = max(lst, t);
            }
        }
        first = wave_min(fst);
        last = wave_max(lst);
        // all 'N' (compress_cigarlist([]) :740 raises) or an unrepresentable column
        if (__ballot(fail) || last < 0) { send_to_general<DUPLEX>(a, m, rm, lds, lane); return kFinStatus; }
        // characters / qualities of the kept span into the (now free) stage, shifted to its start
        lds_fence();
        uint8_t *sb = lds + stage_addr + 0x800;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            const int t = 64 * tt + lane;
            if (t >= first && t <= last) {
                const uint32_t wv = *(const uint16_t *)(ov + 2 * t);
                const uint32_t v = (und >> tt) & 1u ? (uint32_t)chq[t]
                                                   : (uint32_t)((0x47435441u >> (8 * (wv >> 12))) & 255u) |
                                                         ((uint32_t)a.maxq << 8);
                sb[t - first] = (uint8_t)v;
                sb[0x100 + t - first] = (uint8_t)(v >> 8);
            }
        }
    }
    sp.mark(6);                          // [5] finalize
    const int Dmax = wave_max(dmax);
    const int Dmin = wave_min(dmin);
    const int klen = last - first + 1;   // kept columns
    sp.mark(7);                          // [6] depth reductions
    // d / e / seq / qual from the column words, four columns per lane (one
    // 8-, 8-, 4- and 4-byte store each); the region tail up to the next 16
    // columns gets 'N' / quality 0 so a duplex record staging this region never
    // reads a byte that is not a valid letter (d / e there are don't-care)
    lds_fence();
    if (EXACT && DCR_ABL != 5) {        // diagnostic 5: no per-column stores
        const int c0 = 4 * lane;
        if (c0 < T16) {
            const uint2 w = *(const uint2 *)(ov + 8 * lane);
            *(DCR_G uint2 *)(lds_vptr<uint16_t>(lds, fk::kPD) + off + c0) = make_uint2(w.x & 0x003F003Fu, w.y & 0x003F003Fu);
            *(DCR_G uint2 *)(lds_vptr<uint16_t>(lds, fk::kPE) + off + c0) =
                make_uint2((w.x >> 6) & 0x003F003Fu, (w.y >> 6) & 0x003F003Fu);
            const int nl = min(max(klen - c0, 0), 4);                    // kept columns of the four
            const uint32_t keep = nl == 4 ? 0xFFFFFFFFu : (1u << (8 * nl)) - 1u;
            uint32_t letters, quals;
            if (!exact) {
                const uint32_t sel = ((w.x >> 12) & 3u) | ((w.x >> 20) & 0x300u) | ((w.y << 4) & 0x30000u) |
                                     ((w.y >> 4) & 0x3000000u);
                letters = __builtin_amdgcn_perm(0u, 0x47435441u, sel);  // "ATCG"[call]
                quals = (uint32_t)a.maxq * 0x01010101u;
            } else {
                const uint8_t *sb = lds + stage_addr + 0x800;
                letters = *(const uint32_t *)(sb + c0);
                quals = *(const uint32_t *)(sb + 0x100 + c0);
            }
            *(DCR_G uint32_t *)(lds_vptr<uint8_t>(lds, fk::kPSeq) + off + c0) = (letters & keep) | (0x4E4E4E4Eu & ~keep);
            *(DCR_G uint32_t *)(lds_vptr<uint8_t>(lds, fk::kPQual) + off + c0) = quals & keep;
        }
    }
    sp.mark(8);                          // [7] per-column stores
    // E = round(mean(e/d), 3) (:1015-1018).  numpy's mean is a pairwise sum
    // divided by T, then rounded at 3 decimals.  Any summation order lands
    // within 1e-12 (relative) of it, so the rounding agrees unless mean x 1000
    // sits that close to a half-integer; a DPP tree sum decides, and the exact
    // pairwise walk (over the e/d columns written into the now free stage) runs
    // only near such a boundary.
    // R <= 16 (every column decided, or the exact columns' e folded into fx by
    // fxd above): the mean is the rational
    // 1000 sum(e/d) / T = 25 fx / (18018 T) exactly (fx = 720720 sum(e/d)), and
    // its rounding is read off the integer remainder.  A value that is not a
    // tie lies >= 1 / (2 * 18018 T) > 1e-7 from a half-integer, far beyond the
    // reference's own double rounding (< 1e-9 here), so rint agrees with
    // numpy's; a tie, or any other record, takes the double sum below.
    double E = 0.0;
    uint32_t E_lo = 0, E_hi = 0;         // E's words, scalar registers
    uint32_t S = 0;                      // the rational mean's numerator (rows: k_fast_rows rounds it)
    // (the common instantiation holds records of at most 15 reads)
    bool slow = EXACT ? (R > 16 || DCR_ABL == 4) : false;
    if (!slow) {
        S = (uint32_t)wave_sum((int)(fx + (uint32_t)fxd));
        if (EXACT || !DCR_ROWS) {
            // the rational 25 S / (18018 T) in doubles: k = rint, remainder exact
            const int64_t num = 25 * (int64_t)S;
            const int den = 18018 * T;
            const double dn = (double)den;
            double rc = __builtin_amdgcn_rcp(dn);
            rc = __builtin_fma(__builtin_fma(-dn, rc, 1.0), rc, rc);
            const int k = __builtin_amdgcn_readfirstlane((int)__builtin_rint((double)num * rc));
            const int64_t r = num - (int64_t)k * den;
            slow = 2 * (r < 0 ? -r : r) >= den || k > 1000;                   // a tie (or a bad estimate)
            const double Ed = div1000(k);
            E_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__double_as_longlong(Ed));
            E_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)__double_as_longlong(Ed) >> 32));
            // the common kernel kept no column words for the double walk: the
            // EXACT kernel takes the record (a tie is rare)
            if (!EXACT && slow) return kFinQueue;
        }
    }
    if (slow) {
    double sum = 0.0;
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
        const int t = 64 * tt + lane;
        const uint32_t w = *(const uint16_t *)(ov + 2 * t);
        const uint32_t d = w & 63u;
        // e/d to 1 ulp (the decision below tolerates 1e-9; the exact walk divides), d == 0 -> 1 (:1010-1012)
        const double etv = d == 0 ? 1.0 : (double)((w >> 6) & 63u) * invd[d];
        sum += (tt < NT - 1 || t < T) ? etv : 0.0;
    }
    sum += dpp_f64<0xB1>(sum);                   // quad_perm [1,0,3,2]
    sum += dpp_f64<0x4E>(sum);                   // quad_perm [2,3,0,1]
    sum += dpp_f64<0x141>(sum);                  // row_half_mirror
    sum += dpp_f64<0x140>(sum);                  // row_mirror
    sum = (readlane_f64(sum, 0) + readlane_f64(sum, 16)) + (readlane_f64(sum, 32) + readlane_f64(sum, 48));
    double rt = __builtin_amdgcn_rcp((double)T);                             // 1 / T, then one Newton step
    rt = __builtin_fma(__builtin_fma(-(double)T, rt, 1.0), rt, rt);
    const double y = (sum * rt) * 1000.0;                                    // mean x 1000, to ~1e-15
    const double fr = y - __builtin_floor(y);
    if (__builtin_expect(__builtin_fabs(fr - 0.5) > 1e-9 * (1.0 + y), 1) && DCR_ABL != 4) {
        const double ky = __builtin_rint(y);
        E = ky >= 0.0 && ky <= 1000.0 ? div1000((int)ky) : ky / 1000.0;
    } else if (!EXACT) {
        return kFinQueue;                // near a half-integer: the EXACT pass walks numpy's pairwise sum
    } else {
        lds_fence();
        double *et = (double *)(lds + stage_addr);
        const int ln = lane;
        const uint8_t *ovr = lds + ov_addr;
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            const int t = 64 * tt + ln;
            if (t < T) {
                const uint32_t w = *(const uint16_t *)(ovr + 2 * t);
                const uint32_t dd = w & 63u;
                et[t] = dd == 0 ? 1.0 : (double)((w >> 6) & 63u) / (double)dd;   // e / d exactly (:1010-1012)
            }
        }
        lds_fence();
        const double total = 0.0 + pairwise_et(et, T, ln);
        E = __builtin_rint((total / (double)T) * 1000.0) / 1000.0;
    }
    E_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__double_as_longlong(E));
    E_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)__double_as_longlong(E) >> 32));
    }
    sp.mark(9);                          // [8] mean
    if (!EXACT && DCR_ROWS) {
        // the record's scalars as one 16-byte row at its fast-list index
        // (k_fast_rows expands it into the ten dcr_out arrays and rounds the
        // mean): pos (:790, first = 0 here), T | D << 8 | M << 16 | MAPQ << 24
        // (len = n_de = T, one M run), S, kind 1.
        const int mapq = (int)((uint32_t)m.d0 >> 16);
        uint32_t v = 0;
        v = write_lane<0>(v, __builtin_amdgcn_readfirstlane((uint32_t)minpos));
        v = write_lane<1>(v, __builtin_amdgcn_readfirstlane((uint32_t)T | (uint32_t)Dmax << 8 | (uint32_t)Dmin << 16 |
                                                            (uint32_t)mapq << 24));
        v = write_lane<2>(v, __builtin_amdgcn_readfirstlane(S));
        v = write_lane<3>(v, 1u);
        // lanes 0-3 (a buffer store on the row's 16 bytes: the other lanes'
        // words fall outside it, no branch)
        if (DCR_DEFER) pd.v = v;         // the caller stores it after the next record's staging
        else
            __builtin_amdgcn_raw_buffer_store_b32(v, __builtin_amdgcn_make_buffer_rsrc((void *)(a.rows + fi), (short)0, 16,
                                                                                           0x00020000), 4 * lane, 0, 0);
        sp.mark(10);                     // [9] record scalars
        return kFinDone;
    }
    // the record's scalar fields straight into the dcr_out arrays: lane k
    // stores field k (pos :790, MAPQ, len, n_cig, n_de, D, M, E as two words,
    // the single M run of the kept columns), lane 10 the status byte.  The
    // waves of one XCD take consecutive records (k_consensus_fast), so the
    // lines these 4-byte stores share fill up in one L2
    {
        const int mapq = (int)((uint32_t)m.d0 >> 16);                        // k_recmeta
        uint32_t v = 0;
        v = write_lane<0>(v, __builtin_amdgcn_readfirstlane((uint32_t)(minpos + first)));
        v = write_lane<1>(v, __builtin_amdgcn_readfirstlane((uint32_t)mapq));
        v = write_lane<2>(v, __builtin_amdgcn_readfirstlane((uint32_t)klen));
        v = write_lane<3>(v, 1u);
        v = write_lane<4>(v, __builtin_amdgcn_readfirstlane((uint32_t)T));
        v = write_lane<5>(v, __builtin_amdgcn_readfirstlane((uint32_t)Dmax));
        v = write_lane<6>(v, __builtin_amdgcn_readfirstlane((uint32_t)Dmin));
        v = write_lane<7>(v, E_lo);
        v = write_lane<8>(v, E_hi);
        v = write_lane<9>(v, __builtin_amdgcn_readfirstlane((uint32_t)klen << 4));
        DCR_G uint8_t *sb = lds_sgptr<uint8_t>(lds, fk::kPSbase);
        if (sb && lane < 10) {
            // the ten arrays lie within 4 GiB above sbase (checked by the
            // host): lane k stores at a 32-bit offset from that one base
            const uint2 w = *(const uint2 *)(lds + fk::kSofs + 8 * lane);   // offset of array k, its shift
            const uint32_t idx = lane == 9 ? (uint32_t)off : (uint32_t)rec;
            *(DCR_G uint32_t *)(sb + (w.x + (idx << w.y))) = v;
        } else if (lane < 10) {
            // destination word of field k (scalar_dest), from the LDS cache
            const uint64_t pw = *(const uint64_t *)(lds + fk::kPtrs + 8 * lane);
            const uint64_t idx = lane == 9 ? (uint64_t)off : (uint64_t)rec;
            *(DCR_G uint32_t *)((pw & 0x00FFFFFFFFFFFFFFull) + (idx << (pw >> 56))) = v;
        } else if (lane == 10) {
            lds_vptr<uint8_t>(lds, fk::kPStatus)[rec] = DCR_ST_OK;
        }
    }
    sp.mark(10);                         // [9] record scalars
    return kFinDone;
}

__device__ __forceinline__ RecMeta meta_from_lanes(uint32_t v) {
    RecMeta m;
    m.base_al = (uint32_t)readlane((int)v, 0);
    m.d0 = readlane((int)v, 1);
    m.off = (int64_t)(((uint64_t)(uint32_t)readlane((int)v, 3) << 32) | (uint32_t)readlane((int)v, 2));
    m.rec = readlane((int)v, 4);
    m.g0 = readlane((int)v, 5);
    m.minpos = readlane((int)v, 6);
    m.w = (uint32_t)readlane((int)v, 7);
    return m;
}

// Persistent, one 16-wave block per CU sharing the likelihood and e/d tables:
// wave w of NW takes the contiguous fast-list range [n w / NW, n (w+1) / NW);
// record i + 1's loads are issued (at ONE site, so the prefetch registers are
// never copied while in flight) as soon as record i's codes are in LDS, and the
// descriptor of record i + 2 is fetched by a vector load (vmcnt, not lgkmcnt,
// so LDS waits never drain it).
//
// EXACT = false drains the fast list; a record with a column the integer bound
// does not decide is queued (its fast-list index, 64 at a time per wave) for
// the EXACT = true instantiation, which drains that queue and computes such
// columns in the reference's double arithmetic.  The common kernel thus keeps
// none of the exact path's code or registers.
template <bool DUPLEX, bool EXACT>
__global__ __launch_bounds__(fk::kBlockThreads, EXACT ? DCR_EXACT_OCC : DCR_FAST_OCC) void k_consensus_fast(FastArgs a) {
    using RG = fk::Region<EXACT>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[RG::kLds];
    // Record assignment, XCD-aware: the blocks of one group (blockIdx % 8,
    // the blocks that share an XCD and its L2) take one contiguous range of
    // the list, interleaved over the group's waves, so the records in flight
    // on an XCD at any time are neighbours and the output lines they share
    // (4-byte record scalars, 160-column regions) fill up in that XCD's L2.
    // A block none of whose waves has a record leaves before its tables are
    // built (the EXACT grid is the resident one, its queue mostly short).
    const int n = EXACT ? *a.xcount : *a.fast_count;
    int lo, hi, step, first_i;
    {
        const int nb = (int)gridDim.x, g = (int)(blockIdx.x & 7u);
        int before = 0;                                      // blocks of the groups before g
        for (int y = 0; y < g; ++y) before += (nb - y + 7) >> 3;
        const int mine = (nb - g + 7) >> 3;                  // blocks of group g
        const int64_t nw = (int64_t)nb * fk::kWaves;
        lo = (int)((int64_t)n * (before * fk::kWaves) / nw);
        hi = (int)((int64_t)n * ((before + mine) * fk::kWaves) / nw);
        step = mine * fk::kWaves;
        first_i = lo + (int)(blockIdx.x >> 3) * fk::kWaves;  // the block's wave 0
        if (first_i >= hi) return;
    }
    // EXACT: the likelihood factors of quality rows 0..127 (the exact columns'
    // per-read products read them once per row; the common kernel keeps none)
    // EXACT: the quality table's boundaries (phred_from_table reads two per column)
    __shared__ double s_qt[EXACT ? DCR_MAX_QTHRESH : 1];
    if (EXACT)
        for (int i = threadIdx.x; i < DCR_MAX_QTHRESH; i += fk::kBlockThreads) s_qt[i] = a.P->qthresh[i];
    __shared__ double2 s_xt[EXACT ? 128 : 1];
    if (EXACT)
        for (int i = threadIdx.x; i < 128; i += fk::kBlockThreads) s_xt[i] = make_double2(a.P->match[i], a.P->mismatch[i]);
    // EXACT single-strand: the posterior of a one-read column per (class after
    // the mask, quality), as finish_record's per-read loop and posterior()
    // compute it for R = 1 (the same products: 1.0 * factor)
    __shared__ uint32_t s_r1[EXACT && !DUPLEX ? 5 * 128 : 1];
    if (EXACT && !DUPLEX)
        for (int i = threadIdx.x; i < 5 * 128; i += fk::kBlockThreads) {
            const uint32_t k = (uint32_t)i >> 7, q = (uint32_t)i & 127u;
            const double fm = a.P->match[q], fx = a.P->mismatch[q];
            double L4[4] = {1.0, 1.0, 1.0, 1.0};
            double U = 1.0;
            U = U * fx;
#pragma unroll
            for (int j = 0; j < 4; ++j) L4[j] = L4[j] * (k == (uint32_t)(j + 1) ? fm : fx);
            const double L[6] = {L4[0], L4[1], L4[2], L4[3], U, U};
            const Posterior po = posterior(L, false, a.P, a.P->qthresh, true);
            s_r1[i] = ((uint32_t)po.ch & 255u) | ((uint32_t)(po.q + 1) & 1023u) << 8 | ((uint32_t)po.best & 7u) << 18 |
                      (uint32_t)po.masked << 21 | (uint32_t)po.overflow << 22;
        }
    for (int i = threadIdx.x; i < 5 * (fk::kRowMax + 1); i += fk::kBlockThreads) {
        const int k = i / (fk::kRowMax + 1), q = i % (fk::kRowMax + 1);
        const bool nrow = k == 0 || q < a.minbq;          // 'N', or masked below min_base_quality (:280)
        if (EXACT) {
            const uint64_t inc = nrow ? 0ull : (uint64_t)a.llr16[q] << (16 * (k - 1));
            *(uint4 *)(lds + 0x800 * k + 16 * (q + k)) =
                make_uint4((uint32_t)inc, (uint32_t)(inc >> 32), nrow ? 1u : 1u << (6 * k), 0u);
        } else {
            // narrow row (Evidence8): field k - 1 = llr8 << 4 | 1, 'N' rows 0
            const uint64_t inc = nrow ? 0ull : (uint64_t)(((uint32_t)a.llr8[q] << 4) | 1u) << (16 * (k - 1));
            *(uint2 *)(lds + 0x400 * k + 8 * (q + k)) = make_uint2((uint32_t)inc, (uint32_t)(inc >> 32));
        }
    }
    if (EXACT && threadIdx.x < 64) ((double *)(lds + fk::kInvD))[threadIdx.x] = threadIdx.x == 0 ? 0.0 : 1.0 / (double)threadIdx.x;
    if (threadIdx.x == 0) *(uint16_t *)(lds + fk::kSent) = (uint16_t)(EXACT ? fk::kPadCode : fk::kPadCode8);
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        ((uint32_t *)(lds + fk::kM720))[t] = t == 0 || t > 16 ? 0u : 720720u / (uint32_t)t;
    }
    if (threadIdx.x < 10) {
        const int k = threadIdx.x;
        *(uint2 *)(lds + fk::kSofs + 8 * k) = make_uint2(a.sofs[k], (k == 7 || k == 8) ? 3u : 2u);
    }
    if (threadIdx.x < fk::kNPtrs) {
        const int k = threadIdx.x;
        uint64_t v;
        switch (k) {
        case fk::kPNormCig: v = (uint64_t)(uintptr_t)a.norm_cig; break;
        case fk::kPCigOff: v = (uint64_t)(uintptr_t)a.cig_off; break;
        case fk::kPOvf: v = (uint64_t)(uintptr_t)a.ovf; break;
        case fk::kPOvfCount: v = (uint64_t)(uintptr_t)a.ovf_count; break;
        case fk::kPXlist: v = (uint64_t)(uintptr_t)a.xlist; break;
        case fk::kPXcount: v = (uint64_t)(uintptr_t)a.xcount; break;
        case fk::kPD: v = (uint64_t)(uintptr_t)a.O.d; break;
        case fk::kPE: v = (uint64_t)(uintptr_t)a.O.e; break;
        case fk::kPSeq: v = (uint64_t)(uintptr_t)a.O.seq; break;
        case fk::kPQual: v = (uint64_t)(uintptr_t)a.O.qual; break;
        case fk::kPStatus: v = (uint64_t)(uintptr_t)a.O.status; break;
        case fk::kPInfo: v = (uint64_t)(uintptr_t)a.info; break;
        case fk::kPParams: v = (uint64_t)(uintptr_t)a.P; break;
        case fk::kPSbase: v = (uint64_t)(uintptr_t)a.sbase; break;
        case fk::kPE1000: v = (uint64_t)(uintptr_t)a.e1000; break;
        case fk::kPRows: v = (uint64_t)(uintptr_t)a.rows; break;
        default: v = scalar_dest(a.O, k); break;
        }
        *(uint64_t *)(lds + fk::kPtrs + 8 * k) = v;
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane0 = threadIdx.x & 63;
    const int stage_addr = RG::base(wave);
    const int rm_addr = stage_addr + RG::kRm;
    const int ov_addr = RG::ov(wave);
    const int list_addr = stage_addr + RG::kList;      // EXACT only
    __syncthreads();
    int i = first_i + wave;
    if (i >= hi) return;
    const RecMeta *ML = a.meta;
    auto nxt = [&](int j) { return j + step < hi ? j + step : j; };   // the wave's next record (the last repeats)
    auto midx = [&](int j) { return EXACT ? a.xlist[j] : j; };   // EXACT: the queue holds fast-list indices
    int i1 = nxt(i), i2 = nxt(i1);
    RecMeta m0 = ML[midx(i)];
    RecMeta m1 = ML[midx(i1)];
    FastStage<RG::kDw> st;
    fast_load<DUPLEX>(a, m0, ML + midx(i2), lane0, st);
    // EXACT: the queue index of the record after i2, loaded one record ahead
    // as a vector load (the descriptor load of the prefetch depends on it; a
    // scalar load issued there stalled the issue for its whole latency)
    int xv = EXACT ? a.xlist[opaque(nxt(i2))] : 0;
    if (!EXACT && DCR_VMPAD > 0) {      // the same padding as after every later prefetch (the loop's entry path too)
        const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)a.rows, (short)0, 0, 0x00020000);
#pragma unroll
        for (int k = 0; k < DCR_VMPAD; ++k) __builtin_amdgcn_raw_buffer_store_b32(0u, rz, 4 * lane0, 256 * k, 0);
    }
    Stamps sp;
    int pend = 0, npend = 0;           // !EXACT: queued fast-list indices (lane p holds the p-th)
    // DCR_DEFER: the last decided record's row, stored once the next record's
    // bytes are staged: every VMEM store still in flight at a staging is
    // waited for there (loads and stores share vmcnt on gfx950, so the wait
    // for the prefetch is a vmcnt(0)), and the row was the record's last store
    Pend pd;
    pd.v = 0;
    int row_i = -1;                    // the pending record's fast-list index (-1: none)
    auto store_row = [&](int ln) {
        if (!EXACT && DCR_ROWS && DCR_DEFER && row_i >= 0) {
            __builtin_amdgcn_raw_buffer_store_b32(pd.v, __builtin_amdgcn_make_buffer_rsrc((void *)(a.rows + row_i), (short)0,
                                                                                          16, 0x00020000), 4 * ln, 0, 0);
            row_i = -1;
            pd.v = 0;
        }
    };
    auto flush = [&](int ln) {         // queue pointers from the LDS cache (no scalar registers held)
        int base = 0;
        if (ln == 0) base = __hip_atomic_fetch_add(lds_sgptr<int>(lds, fk::kPXcount), npend, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        base = __builtin_amdgcn_readfirstlane(base);
        if (ln < npend) lds_sgptr<int>(lds, fk::kPXlist)[base + ln] = pend;
        npend = 0;
    };
    for (;;) {
        // lane-derived addresses are formed per record, not hoisted out of the
        // record loop into registers held across it
        const int lane = opaque(lane0);
#if defined(DCR_PADV) && !defined(DCR_NO_PAD)
        if (!EXACT && !DUPLEX) {        // diagnostic builds only: extra VALU issue per record
            int dv;
            asm volatile(".rept " DCR_STR(DCR_PADV) "\n v_mov_b32 %0, 0\n .endr" : "=v"(dv));
        }
#endif
#if defined(DCR_PADM) && !defined(DCR_NO_PAD)
        if (!EXACT && !DUPLEX) {        // diagnostic builds only: extra VMEM stores per record (range-checked out)
            const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)a.rows, (short)0, 0, 0x00020000);
#pragma unroll
            for (int k = 0; k < DCR_PADM; ++k) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)lane, rz, lane, 64 * k, 0);
        }
#endif
#if defined(DCR_PADL) && !defined(DCR_NO_PAD)
        if (!EXACT && !DUPLEX) {        // diagnostic builds only: extra VMEM loads per record (range-checked out)
            const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)a.rows, (short)0, 0, 0x00020000);
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < DCR_PADL; ++k) acc += __builtin_amdgcn_raw_buffer_load_b32(rz, 4 * lane, 256 * k, 0);
            asm volatile("" :: "v"(acc));
        }
#endif
#if defined(DCR_PADS) && !defined(DCR_NO_PAD)
        if (!EXACT && !DUPLEX) {        // diagnostic builds only: extra SALU issue per record
            int ds;
            asm volatile(".rept " DCR_STR(DCR_PADS) "\n s_mov_b32 %0, 0\n .endr" : "=s"(ds));
        }
#endif
        sp.mark(0);
        if (DCR_STAMP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sp.mark(1);                    // [0] wait for this record's prefetched bytes
        // single-strand records of at most direct_r reads almost never have
        // every column decided by the bound (one to three reads stay below
        // maxQ wherever a read is masked or disagrees): they go to the exact
        // queue untouched instead of being staged here and again there
        // so do records larger than this instantiation's stage (common: more
        // than 1,536 bytes; the EXACT instantiation stages up to 2,048)
        // and so do records of more than 15 reads (the narrow rows' counts)
        const bool direct = !EXACT && ((!DUPLEX && (int)(m0.w & 127u) <= a.direct_r) ||
                                       (int)(m0.w >> 15) > RG::kDw * kWave || (int)(m0.w & 127u) > 15 || !a.narrow);
        uint32_t bad = 0;
        if (!direct) {
            bad = a.lo_check ? stage_codes<DUPLEX, true, !EXACT>(a, m0, st, lds, stage_addr, lane)
                             : stage_codes<DUPLEX, false, !EXACT>(a, m0, st, lds, stage_addr, lane);
            // the read words go through LDS: a register copy of them would live
            // across the prefetch's refill of st and force a wait for it at the
            // loop's back edge
            *(uint2 *)(lds + rm_addr + 8 * lane) = st.rm;
        }
        if (lane < 8) *(uint32_t *)(lds + fk::kMv + 32 * wave + 4 * lane) = st.mv;
        sp.mark(2);                    // [1] element codes into LDS
        __builtin_amdgcn_sched_barrier(0);
        // the next record's bytes and the descriptor of the one after the
        // next but one; unconditional (the last record re-loads itself) so the
        // registers have one definition
        const int i3 = nxt(i2);
        fast_load<DUPLEX>(a, m1, ML + (EXACT ? __builtin_amdgcn_readfirstlane(xv) : i3), lane, st);
        if (EXACT) xv = a.xlist[opaque(nxt(i3))];
        store_row(lane);
        if (!EXACT && DCR_VMPAD > 0) {
            // DCR_VMPAD stores that the range check drops (no memory access)
            // right after the prefetch: every path through the record now
            // issues at least that many VMEM ops after the prefetch's loads,
            // so the next staging's wait for them (s_waitcnt vmcnt counts
            // loads and stores in issue order) is vmcnt(DCR_VMPAD) or more,
            // not a drain of this record's column stores
            const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)a.rows, (short)0, 0, 0x00020000);
#pragma unroll
            for (int k = 0; k < DCR_VMPAD; ++k) __builtin_amdgcn_raw_buffer_store_b32(0u, rz, 4 * lane, 256 * k, 0);
        }
        sp.mark(3);                    // [2] prefetch issue
        lds_fence();
        const uint2 rw = *(const uint2 *)(lds + rm_addr + 8 * lane);
        // the read's word relative to this record: col | len << 8 | mapq << 16, stage offset
        const uint2 rm = make_uint2((uint32_t)(((int)rw.x >> 16) + ((DCR_ABL == 6 && !DUPLEX ? a.meta[0].d0 : m0.d0) & 0xFFFF)) |
                                        (rw.x & 0xFFFFu) << 8,
                                    rw.y - (DCR_ABL == 6 && !DUPLEX ? a.meta[0].base_al : m0.base_al));
        const RecMeta m2 = meta_from_lanes(*(const uint32_t *)(lds + fk::kMv + 32 * wave + 4 * (lane & 7)));   // record i2
        // a record this kernel does not decide gets an empty row (kind 0:
        // k_fast_rows leaves its scalars to the kernel that finishes it)
        auto no_row = [&]() {
            if (!EXACT && DCR_ROWS)     // the row's four words zeroed (kind 0), no lane branch
                __builtin_amdgcn_raw_buffer_store_b32(0u, __builtin_amdgcn_make_buffer_rsrc((void *)(a.rows + i), (short)0, 16,
                                                                                            0x00020000), 4 * lane, 0, 0);
        };
        if (direct) {
            no_row();
            if (lane == npend) pend = i;
            if (++npend == kWave) flush(lane);
            i += step;
            if (i >= hi) break;
            m0 = m1;
            m1 = m2;
            i2 = i3;
            continue;
        }
        const Staged sg = trim_record<DUPLEX, !EXACT>(a, m0, rm, bad, lds, stage_addr, lane);
        sp.mark(4);                    // [3] trim, fence
        if (sg.state == 1) {
            send_to_general<DUPLEX>(a, m0, sg.rm, lds, lane);
            no_row();
        } else if (sg.state == 0 || sg.state == 3) {
            // NT comes from T before a state-3 record's 3' trim (finish_record
            // runs it): a trim that shrinks T by a whole tile leaves all-'N'
            // live columns in the earlier tiles, undecided, so such a (rare)
            // record takes the EXACT queue instead of being decided here
            int fin;
            if (sg.T <= 64) fin = finish_record<DUPLEX, 1, EXACT>(a, m0, sg, lds, stage_addr, ov_addr, rm_addr, list_addr, lane, sp, s_xt, s_r1, s_qt, i, pd);
            else if (sg.T <= 128) fin = finish_record<DUPLEX, 2, EXACT>(a, m0, sg, lds, stage_addr, ov_addr, rm_addr, list_addr, lane, sp, s_xt, s_r1, s_qt, i, pd);
            else if (sg.T <= 192) fin = finish_record<DUPLEX, 3, EXACT>(a, m0, sg, lds, stage_addr, ov_addr, rm_addr, list_addr, lane, sp, s_xt, s_r1, s_qt, i, pd);
            else fin = finish_record<DUPLEX, 4, EXACT>(a, m0, sg, lds, stage_addr, ov_addr, rm_addr, list_addr, lane, sp, s_xt, s_r1, s_qt, i, pd);
            if (!EXACT && fin != kFinDone) no_row();
            if (!EXACT && DCR_DEFER && fin == kFinDone) row_i = i;
            if (!EXACT && fin == kFinQueue) {
                if (lane == npend) pend = i;
                if (++npend == kWave) flush(lane);
            }
        } else {
            no_row();
        }
        i += step;
        if (i >= hi) break;
        m0 = m1;
        m1 = m2;
        i2 = i3;
    }
    store_row(lane0);
    if (!EXACT && npend) flush(lane0);
    if (DCR_STAMP && lane0 == 0)
        for (int k = 0; k < 12; ++k)   // fast ss 0-11, ds 16-27; exact ss 32-43, ds 48-59
            atomicAdd(&a.stamps[k + (DUPLEX ? 16 : 0) + (EXACT ? 32 : 0)], (unsigned long long)sp.acc[k]);
}

// The outcome of a two-read column per (class after the mask, quality) of
// each read, index ((k1 * 128 + q1) * 5 + k2) * 128 + q2, packed as the
// one-read table (character, quality + 1, argmax, masked, overflow): the
// EXACT pass's products in read order (1.0 * factor of read 1, then * factor
// of read 2) and posterior(), so a table entry is bit-identical to computing
// the column.  Two-read columns are the exact pass's most common kind (every
// duplex record, single-strand records of two reads).
__global__ __launch_bounds__(256) void k_r2_table(const dcr_params *P, uint32_t *tab) {
    const int i = (int)(blockIdx.x * 256u + threadIdx.x);
    if (i >= kR2Entries) return;
    const uint32_t q2 = (uint32_t)i & 127u, k2 = ((uint32_t)i >> 7) % 5u;
    const uint32_t q1 = ((uint32_t)i / 640u) & 127u, k1 = (uint32_t)i / (640u * 128u);
    const double x1 = P->match[q1], y1 = P->mismatch[q1], x2 = P->match[q2], y2 = P->mismatch[q2];
    double L4[4] = {1.0, 1.0, 1.0, 1.0};
    double U = 1.0;
    U = U * y1;
#pragma unroll
    for (int j = 0; j < 4; ++j) L4[j] = L4[j] * (k1 == (uint32_t)(j + 1) ? x1 : y1);
    U = U * y2;
#pragma unroll
    for (int j = 0; j < 4; ++j) L4[j] = L4[j] * (k2 == (uint32_t)(j + 1) ? x2 : y2);
    const double L[6] = {L4[0], L4[1], L4[2], L4[3], U, U};
    const Posterior po = posterior(L, false, P, P->qthresh, true);
    tab[i] = ((uint32_t)po.ch & 255u) | ((uint32_t)(po.q + 1) & 1023u) << 8 | ((uint32_t)po.best & 7u) << 18 |
             (uint32_t)po.masked << 21 | (uint32_t)po.overflow << 22;
}

// Expands the rows k_consensus_fast wrote for the records it decided (one
// lane per fast-list entry; entries are in record order within a wave's
// range, so the ten stores per lane coalesce across the wave) and rounds the
// mean: E = round(mean(e/d), 3) (:1015-1018) is the rational
// 1000 sum(e/d) / T = 25 S / (18018 T) (S = 720720 sum(e/d), exact for depths
// <= 16) rounded half-even; away from a tie it lies >= 1 / (2 * 18018 T)
// > 1e-7 from a half-integer, beyond the reference's own double rounding
// (< 1e-9), so numpy's rint agrees.  A tie is left to the EXACT pass (the
// double pairwise walk): the record goes on its queue.  Kind 2 rows carry an
// E the fast kernel stored itself.
__global__ __launch_bounds__(256) void k_fast_rows(FastArgs a) {
    if (!DCR_ROWS) return;                       // rows are written (and zeroed) only by DCR_ROWS builds
    const int i = (int)(blockIdx.x * 256u + threadIdx.x);
    if (i >= *a.fast_count) return;
    const uint4 row = a.rows[i];
    if (row.w == 0u) return;
    const RecMeta m = a.meta[i];
    const int64_t rec = m.rec;
    const uint32_t T = row.y & 255u;
    if (row.w == 1u) {
        // 25 S / (18018 T): num < 2^37, den < 2^23.  The quotient from a
        // double estimate (within 1 of the truth) fixed up by the integer
        // remainder: a 64-bit integer division is a ~150-instruction
        // software loop, the slot's largest cost in this kernel
        const int64_t num = 25ll * row.z, den = 18018ll * T;
        int64_t q = (int64_t)((double)num * (1.0 / (double)den));
        int64_t r = num - q * den;
        if (r < 0) { --q; r += den; }
        if (r >= den) { ++q; r -= den; }
        if (2 * r == den) {
            a.xlist[atomicAdd(a.xcount, 1)] = i;
            return;
        }
        a.O.E[rec] = div1000((int)(q + (2 * r > den ? 1 : 0)));
    }
    a.O.pos[rec] = (int32_t)row.x;
    a.O.mapq[rec] = (int32_t)(row.y >> 24);
    a.O.len[rec] = (int32_t)T;
    a.O.n_cig[rec] = 1;
    a.O.n_de[rec] = (int32_t)T;
    a.O.D[rec] = (int32_t)((row.y >> 8) & 255u);
    a.O.M[rec] = (int32_t)((row.y >> 16) & 255u);
    a.O.cigar[m.off] = T << 4;                   // one M run of the kept columns
    a.O.status[rec] = DCR_ST_OK;
}

// persistent: drains the general list written by k_recmeta.  A wave takes
// the record at its grid position, then claims the next ones from a counter
// (reset with the batch's other counters), so a wave that drew deep records
// does not hold the kernel's tail while others idle.  The claim is made by
// the wave's first active lane, not by a fixed lane: with a claim gated on
// lane 0 the compiler lowered this loop as a divergent loop (a per-lane exit
// mask at the latch); once lane 0 dropped out of exec no claim was made
// again and the wave re-read its last index forever (the
// round-1 hang).
template <bool DUPLEX>
#ifndef DCR_GEN_OCC
#define DCR_GEN_OCC 2
#endif
__global__ __launch_bounds__(kBlock, DCR_GEN_OCC) void k_consensus_general(Args a) {
    __shared__ double2 s_lut[DCR_LUT_N];
    __shared__ double s_qthr[DCR_MAX_QTHRESH];
    __shared__ WaveLds s_wave[kWavesPerBlock];
    __shared__ uint32_t s_wtab[DCR_LUT_N];
    const dcr_params *P = a.P;
    for (int i = threadIdx.x; i < DCR_LUT_N; i += kBlock) s_lut[i] = make_double2(P->match[i], P->mismatch[i]);
    if (a.t16 >= 0)
        for (int i = threadIdx.x; i < DCR_LUT_N; i += kBlock) s_wtab[i] = a.wtab[i];
    for (int i = threadIdx.x; i < DCR_MAX_QTHRESH; i += kBlock) s_qthr[i] = P->qthresh[i];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int n = a.ws.ovf_count[DUPLEX ? 1 : 0];
    int *next = a.ws.gen_next + (DUPLEX ? 1 : 0);
    // the first record of each wave by position (no atomic on the way in: most
    // general lists are shorter than the grid), then claims past the grid
    // (one record per claim: claiming 4 or 8 at a time measured slower on C3,
    // 3.85 -> 3.97 / 4.13 ms at 100 k families, the tail imbalance outweighing
    // the serialised claims)
    const int nw = gridDim.x * kWavesPerBlock;
    GStamp gs;
    for (int i = blockIdx.x * kWavesPerBlock + wave;;) {
        if (i >= n) break;
        const int v = a.ws.ovf[i];                  // bit 31: k_decide decided every column
        process_record<DUPLEX, false>(a, v & 0x7fffffff, s_wave[wave], s_lut, s_qthr, s_wtab, v < 0, lane, gs);
        if (nw >= n) break;
        // one claim per wave, by its first active lane (any lane may carry it)
        const uint64_t act = __ballot(1);
        const int leader = __ffsll((long long)act) - 1;
        int t = 0;
        if (lane == leader) t = atomicAdd(next, 1);
        i = nw + __builtin_amdgcn_readfirstlane(__shfl(t, leader, kWave));
    }
    if (DCR_GSTAMP && lane == 0)
        for (int k = 0; k < 20; ++k) atomicAdd(&a.ws.stamps[k + (DUPLEX ? 32 : 0)], (unsigned long long)gs.acc[k]);
}

// Insertion layouts by events (see run_at): one wave per general-list record
// with an insertion column, 4-wave blocks, few registers.  Writes the record's
// block (insertion mask, then every read's row of element codes over the T
// columns) into ws.lay and its offset into ws.lay_base; -1 for a record it
// does not take (no insertion, a failing read, T or R > 256, a read outside the
// model's assumptions -- more than 4 runs or one I run, fewer M + I ops than
// bases, bases ending inside or before its I run -- or no room left): the
// general kernel then lays it out column by column, reproducing the
// reference's IndexErrors.
template <bool DUPLEX>
__global__ __launch_bounds__(256, DCR_LAYOCC) void k_ins_layout(Args a) {
    __shared__ uint32_t s_scr[kWavesPerBlock][4 * kWave];   // phase A: an I read's r, need, L | bases << 16, start
    __shared__ uint32_t s_iev[kWavesPerBlock][4 * kWave];   // per read: run start | L << 9 | bases << 16 (511: none)
    __shared__ __attribute__((aligned(16))) uint32_t s_rt[kWavesPerBlock][16 * kWave];  // phase B: a chunk's read table
    __shared__ uint32_t s_wtab[DCR_LUT_N];
    if (a.t16 >= 0)
        for (int i = threadIdx.x; i < DCR_LUT_N; i += kBlock) s_wtab[i] = a.wtab[i];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int n = a.ws.ovf_count[DUPLEX ? 1 : 0];
    const int nw = gridDim.x * kWavesPerBlock;
    const int64_t lb_off = DUPLEX ? 4 * (int64_t)a.in.n_fam : 0;
    const int minbq = a.P->min_base_quality;
    uint32_t *scr = s_scr[wave];
    uint32_t *iev = s_iev[wave];
    uint32_t *rt = s_rt[wave];
    int *lnext = a.ws.lay_next + (DUPLEX ? 1 : 0);
    // single-strand: the first record of each wave by position, then one
    // claim per record (records of up to 256 reads and columns: a fixed
    // stride left the waves holding the heavy ones as the tail; C3 general
    // slot 11.98 -> 11.13 ms).  Duplex records (two reads each) keep the
    // stride: 30 k claims on one counter cost 0.27 ms there.
    auto claim = [&]() {
        const uint64_t act = __ballot(1);
        const int leader = __ffsll((long long)act) - 1;
        int t = 0;
        if (lane == leader) t = atomicAdd(lnext, 1);
        return nw + __builtin_amdgcn_readfirstlane(__shfl(t, leader, kWave));
    };
    uint64_t gacc[3] = {0, 0, 0}, gcnt[3] = {0, 0, 0}, gmax = 0;   // DCR_GSTAMP builds: ticks per record class
    for (int i = blockIdx.x * kWavesPerBlock + wave; i < n; i = DCR_LAYCLAIM && !DUPLEX ? (nw >= n ? n : claim()) : i + nw) {
        const uint64_t g0 = DCR_GSTAMP ? __builtin_amdgcn_s_memtime() : 0;
        const int vv = a.ws.ovf[i];
        if (vv < 0) continue;                         // decided by k_decide: no insertion column
        const int64_t rec = vv;
        const int R = DUPLEX ? 2 : (a.in.sub_off[rec + 1] - a.in.sub_off[rec]);
        int lay = -1;
        if (R > 0 && R <= 4 * kWave) {
            int minpos = 0x7fffffff, maxend = -0x7fffffff;
            bool up = false, ins = false;
            // the first 64 reads' references stay in registers (lane = read)
            // and their first four runs in the read table's last four words
            // (rt[16 r + 12..15], which the table leaves alone) for phase A
            // and the table
            ReadRef rd0{};
            for (int c = 0; c < R; c += kWave) {
                const int r = c + lane;
                if (r < R) {
                    const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                    if (DCR_LAYHOIST && c == 0) {
                        rd0 = rd;
                        const int kl = max(rd.ncig - 1, 0);      // every load issued at once, clamped to the read's runs
                        const uint32_t v0 = rd.cig[0], v1 = rd.cig[min(1, kl)], v2 = rd.cig[min(2, kl)],
                                       v3 = rd.cig[min(3, kl)];
                        ((uint4 *)&rt[16 * lane])[3] = make_uint4(rd.ncig > 0 ? v0 : 0u, rd.ncig > 1 ? v1 : 0u,
                                                                  rd.ncig > 2 ? v2 : 0u, rd.ncig > 3 ? v3 : 0u);
                    }
                    up |= rd.status != 0 || rd.len <= 0;
                    minpos = min(minpos, rd.pos);
                    maxend = max(maxend, rd.pos + rd.len);
                    if (!DUPLEX) {
                        ins |= a.ws.info[a.in.sub_off[rec] + r].has_ins != 0;
                    } else {
                        for (int k = 0; k < rd.ncig; ++k) ins |= (rd.cig[k] & 15u) == 1u;
                    }
                }
            }
            up = __ballot(up) != 0;
            ins = __ballot(ins) != 0;
            minpos = wave_min(minpos);
            const int T = wave_max(maxend) - minpos;
            const int64_t *col_off = DUPLEX ? a.in.ds_col_off : a.in.ss_col_off;
            const bool take = !up && ins && T > 0 && T <= kColsLds && T <= col_off[rec + 1] - col_off[rec];
            // phase A: eligibility, the I reads compacted into lanes
            int nI = 0;
            bool bad = !take;
            for (int c = 0; c < R && !bad; c += kWave) {
                const int r = c + lane;
                bool isI = false, b_r = false;
                uint32_t need = 0, L = 0, bb = 0, sr = 0;
                if (r < R) {
                    const bool reg = DCR_LAYHOIST && c == 0;
                    const ReadRef rd = reg ? rd0 : get_read<DUPLEX>(a, rec, r);
                    const uint32_t *cg0 = &rt[16 * lane + 12];
                    int nIr = 0, acc = 0, accb = 0, mi = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t v = k >= rd.ncig ? 2u : reg ? cg0[k] : rd.cig[k];   // past the runs: D of length 0
                        const int o = (int)(v & 15u), ln = (int)(v >> 4);
                        if (o == 1 && nIr == 0) {
                            need = (uint32_t)acc;
                            L = (uint32_t)ln;
                            bb = (uint32_t)accb;
                        }
                        nIr += o == 1;
                        mi += o != 2 ? ln : 0;
                        acc += ln;
                        accb += o != 2 ? ln : 0;
                    }
                    isI = nIr == 1;
                    b_r = rd.ncig > 4 || nIr > 1 || mi < rd.len || (isI && (int)(bb + L) > rd.len) || L > 127 ||
                          bb > 0xFFFF;
                    sr = (uint32_t)(rd.pos - minpos);
                    iev[r] = 511u;
                }
                const uint64_t im = __ballot(isI);
                const int slot = nI + __popcll(im & lanemask_lt(lane));
                if (isI && slot < kWave) {
                    scr[4 * slot] = (uint32_t)r;
                    scr[4 * slot + 1] = need;
                    scr[4 * slot + 2] = L | bb << 16;
                    scr[4 * slot + 3] = sr;
                }
                nI += __popcll(im);
                bad = __ballot(b_r) != 0;
            }
            uint64_t imask[4] = {0ull, 0ull, 0ull, 0ull};
            if (!bad && nI <= kWave) {
                lds_fence();
                bool pend = lane < nI;
                int need = 0, L = 0, sr = 0, rj = 0, bj = 0;
                if (pend) {
                    rj = (int)scr[4 * lane];
                    need = (int)scr[4 * lane + 1];
                    L = (int)(scr[4 * lane + 2] & 0xFFFFu);
                    bj = (int)(scr[4 * lane + 2] >> 16);
                    sr = (int)scr[4 * lane + 3];
                }
                int t = 0;
                for (int it = 0; it <= kWave; ++it) {     // each event activates at least one lane
                    const int cand = pend ? (need == 0 ? t : max(t, sr) + need) : 0x7fffffff;
                    const int tn = wave_min(cand);
                    if (tn >= T) break;
                    if (pend && need > 0) need -= max(0, tn - max(t, sr));
                    const bool act = pend && need == 0 && cand == tn;
                    const int B = wave_max(act ? L : 0);
                    const int hi = min(T, tn + B);
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const int lo2 = max(tn, 64 * w), hi2 = min(hi, 64 * w + 64);
                        if (lo2 < hi2) {
                            const int nb = hi2 - lo2;
                            imask[w] |= (nb == 64 ? ~0ull : ((1ull << nb) - 1ull)) << (lo2 - 64 * w);
                        }
                    }
                    if (act) {
                        iev[rj] = (uint32_t)tn | (uint32_t)L << 9 | (uint32_t)bj << 16;
                        pend = false;
                    }
                    t = tn + B;
                }
                lds_fence();
                // the record's mask and rows (fixed places: see Workspace::lay)
                {
                    lay = 1;
                    if (lane < 4) {
                        const uint64_t m = lane == 0 ? imask[0] : lane == 1 ? imask[1] : lane == 2 ? imask[2] : imask[3];
                        a.ws.lay_mask[4 * (lb_off + rec) + lane] = m;
                    }
                    uint16_t *rows = a.ws.lay + (DUPLEX ? (int64_t)a.in.n_reads + 2 * rec : (int64_t)a.in.sub_off[rec]) * kLayRow;
                    // phase B: lane = column, 64 at a time; per read the
                    // column-free values computed lane-parallel (lane = read).
                    // The columns' integer decision sums ride along (k_decide's
                    // bound, decide_end, insertion columns included): a record
                    // whose every column is decided is marked decided and the
                    // general kernel forms no product for it
                    bool all_dec = a.t16 >= 0 && decide_usable(a, R);
                    int32_t *cw = a.ws.cons + (DUPLEX ? a.in.ds_col_off : a.in.ss_col_off)[rec];
                    // lane = read of a chunk: everything per read that does
                    // not depend on the column, into the wave's read table
                    // (read back as uniform-address LDS loads: no readlane
                    // into scalar registers, which spilled); built once for a
                    // record of at most 64 reads, per chunk and block beyond
                    auto build_rt = [&](const int cb, const int nr) {
                    if (lane < nr) {
                        const bool reg = DCR_LAYHOIST && cb == 0;
                        const ReadRef rd = reg ? rd0 : get_read<DUPLEX>(a, rec, cb + lane);
                        const uint4 cq = ((const uint4 *)&rt[16 * lane])[3];
                        const uint32_t cg0[4] = {cq.x, cq.y, cq.z, cq.w};
                        const int sr = rd.pos - minpos;
                        int end = 0, bb = 0, ends[4], bbs[4];
                        uint32_t dm = 0;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t v = k < rd.ncig ? (reg ? cg0[k] : rd.cig[k]) : 0u;
                            const int ln = k < rd.ncig ? (int)(v >> 4) : 0;
                            const bool isd = (v & 15u) == 2u;
                            bbs[k] = bb;
                            end += ln;
                            ends[k] = end;
                            bb += isd ? 0 : ln;
                            dm |= (isd ? 1u : 0u) << k;
                        }
                        uint4 *row = (uint4 *)&rt[16 * lane];
                        row[0] = make_uint4((uint32_t)sr, (uint32_t)rd.len, (uint32_t)(sr - ins_below(imask, sr)),
                                            iev[cb + lane]);
                        row[1] = make_uint4((uint32_t)ends[0] | (uint32_t)ends[1] << 16,
                                            (uint32_t)ends[2] | (uint32_t)ends[3] << 16,
                                            (uint32_t)bbs[1] | (uint32_t)bbs[2] << 16,
                                            (uint32_t)bbs[3] | (uint32_t)bb << 16 | 0u);
                        rt[16 * lane + 8] = dm;
                        ((int64_t *)&rt[16 * lane])[5] = rd.seq_start;
                    }
                        lds_fence();
                    };
                    const bool one = DCR_LAYHOIST && R <= kWave;
                    if (one) build_rt(0, R);
                    // pass 0 decides (no rows written); the rows only when some
                    // column stays undecided (pass 1)
                    for (int pass = all_dec ? 0 : 1; pass < 2; ++pass) {
                    if (pass == 1 && all_dec) break;
                    const bool wr = pass == 1;
                    int nbase = 0;
                    for (int c0 = 0; c0 < T && (wr || all_dec); c0 += kWave) {
                        const int t2 = c0 + lane;
                        const int wq = c0 >> 6;       // no dynamic index: imask stays in registers
                        const uint64_t mw = wq == 0 ? imask[0] : wq == 1 ? imask[1] : wq == 2 ? imask[2] : imask[3];
                        const bool insc = ((mw >> lane) & 1ull) != 0;
                        const int Nt = nbase + __popcll(~mw & (lane == 0 ? 0ull : (~0ull >> (64 - lane))));
                        DecideSums D;
                        for (int cb = 0; cb < R; cb += kWave) {
                            const int nr = min(kWave, R - cb);
                            if (!one) build_rt(cb, nr);
                            const uint8_t *gb = DUPLEX ? a.ss.seq : a.in.bases;
                            const uint8_t *gq = DUPLEX ? a.ss.qual : a.in.quals;
                            constexpr int kU = DCR_LAYU;     // reads whose byte loads are in flight together
                            for (int r0 = 0; r0 < nr; r0 += kU) {
                                int64_t pu[kU];
                                uint32_t ku[kU];      // 0 base, 1 '+', 2 pad, 3 '-'
#pragma unroll
                                for (int u = 0; u < kU; ++u) {
                                    const int r = min(r0 + u, nr - 1);
                                    const uint4 f0 = ((const uint4 *)&rt[16 * r])[0];
                                    const uint4 f1 = ((const uint4 *)&rt[16 * r])[1];
                                    const uint32_t dm = rt[16 * r + 8];
                                    const int64_t ss0 = ((const int64_t *)&rt[16 * r])[5];
                                    const int sr = (int)f0.x, len = (int)f0.y, Ns = (int)f0.z;
                                    const uint32_t e0 = f0.w;
                                    const int E = (int)(e0 & 511u), L2 = (int)((e0 >> 9) & 127u), bI = (int)(e0 >> 16);
                                    const bool isI = E != 511;
                                    const bool inI = isI && t2 >= E && t2 < E + L2;
                                    const int j = Nt - Ns + ((isI && E < t2) ? L2 : 0);
                                    const int en0 = (int)(f1.x & 0xFFFFu), en1 = (int)(f1.x >> 16);
                                    const int en2 = (int)(f1.y & 0xFFFFu), en3 = (int)(f1.y >> 16);
                                    const int k = (j >= en0) + (j >= en1) + (j >= en2) + (j >= en3);
                                    const int st = k == 0 ? 0 : k == 1 ? en0 : k == 2 ? en1 : en2;
                                    const int bbk = k == 0 ? 0 : k == 1 ? (int)(f1.z & 0xFFFFu)
                                                  : k == 2 ? (int)(f1.z >> 16) : (int)(f1.w & 0xFFFFu);
                                    const bool isd = k < 4 && ((dm >> k) & 1u);
                                    const int is = k == 4 ? (int)(f1.w >> 16) : bbk + (isd ? 0 : j - st);
                                    const int cis = insc ? bI + (t2 - E) : is;
                                    ku[u] = insc ? (inI ? 0u : 1u) : (t2 < sr || is >= len) ? 2u : isd ? 3u : 0u;
                                    pu[u] = ss0 + min(max(cis, 0), len - 1);
                                }
                                uint32_t bu[kU], qu[kU];
#pragma unroll
                                for (int u = 0; u < kU; ++u) {
                                    bu[u] = gb[pu[u]];
                                    qu[u] = gq[pu[u]];
                                }
#pragma unroll
                                for (int u = 0; u < kU; ++u) {
                                    const uint32_t e = ku[u] == 0u ? make_code<DUPLEX>(bu[u], qu[u], minbq)
                                                     : ku[u] == 1u ? kPlus : ku[u] == 2u ? kPad : kDel;
                                    if (r0 + u < nr) {
                                        if (!wr) D.add(e, s_wtab);
                                        if (wr && t2 < T) rows[((int64_t)(t2 >> 5) * R + cb + r0 + u) * kTileIns + (t2 & 31)] = (uint16_t)e;
                                    }
                                }
                            }
                            if (!one) lds_fence();      // the read table is rewritten by the next chunk
                        }
                        nbase += __popcll(~mw & (T - c0 >= 64 ? ~0ull : ((1ull << (T - c0)) - 1ull)));
                        if (!wr) {
                            ColOut co;
                            if (decide_end(a, R, t2 < T, insc, D, co)) {
                                const int uc = co.ch >= 'a' ? co.ch - 32 : co.ch;
                                const uint32_t kb = uc == 'A' ? 0u : uc == 'T' ? 1u : uc == 'C' ? 2u : uc == 'G' ? 3u
                                                  : uc == '+' ? 4u : 5u;
                                if (t2 < T)
                                    cw[t2] = (int32_t)(kb | (uint32_t)co.d << 3 | (uint32_t)co.e << 15 |
                                                       (co.ch >= 'a' ? 1u : 0u) << 27);
                            } else {
                                all_dec = false;
                            }
                        }
                    }
                    }
                    if (all_dec && lane == 0) a.ws.ovf[i] = (int)rec | (int)0x80000000u;
                }
            }
        }
        if (lane == 0) a.ws.lay_base[lb_off + rec] = lay;
        if (DCR_GSTAMP) {
            const uint64_t dt = __builtin_amdgcn_s_memtime() - g0;
            const int cls = lay < 0 ? 0 : R <= kWave ? 1 : 2;
            gacc[0] += cls == 0 ? dt : 0;
            gacc[1] += cls == 1 ? dt : 0;
            gacc[2] += cls == 2 ? dt : 0;
            gcnt[0] += cls == 0;
            gcnt[1] += cls == 1;
            gcnt[2] += cls == 2;
            gmax = dt > gmax ? dt : gmax;
        }
    }
    if (DCR_GSTAMP && !DUPLEX && lane == 0) {
        for (int k = 0; k < 3; ++k) {
            atomicAdd(&a.ws.stamps[20 + k], (unsigned long long)gacc[k]);
            atomicAdd(&a.ws.stamps[23 + k], (unsigned long long)gcnt[k]);
        }
        atomicMax(&a.ws.stamps[26], (unsigned long long)gmax);
    }
}

// decision pass over the general list (decide_record), one wave per record:
// marks the records whose every column it decides (ovf entry | bit 31) and
// leaves their column words in the workspace column scratch (ws.cons)
template <bool DUPLEX>
__global__ __launch_bounds__(256) void k_decide(Args a) {
    __shared__ uint32_t s_wtab[DCR_LUT_N];
    __shared__ __attribute__((aligned(16))) uint16_t s_stage[kWavesPerBlock][kStageElems];
    if (a.t16 < 0) return;
    for (int i = threadIdx.x; i < DCR_LUT_N; i += kBlock) s_wtab[i] = a.wtab[i];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int n = a.ws.ovf_count[DUPLEX ? 1 : 0];
    const int nw = gridDim.x * kWavesPerBlock;
    for (int i = blockIdx.x * kWavesPerBlock + wave; i < n; i += nw) {
        const int64_t rec = a.ws.ovf[i];
        const int R = DUPLEX ? 2 : (a.in.sub_off[rec + 1] - a.in.sub_off[rec]);
        if (R <= 0) continue;
        if (!DUPLEX && R >= kDeepReads) {            // the block-cooperative pass below
            if (lane == 0) a.ws.deep[atomicAdd(a.ws.deep_count, 1)] = i;
            continue;
        }
        int minpos = 0x7fffffff, maxend = -0x7fffffff, up = 0;
        for (int c = 0; c < R; c += kWave) {
            const int r = c + lane;
            if (r < R) {
                const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                up |= rd.status != 0 || rd.len <= 0;
                if (!DUPLEX) up |= a.ws.info[a.in.sub_off[rec] + r].has_ins;
                minpos = min(minpos, rd.pos);
                maxend = max(maxend, rd.pos + rd.len);
            }
        }
        if (__ballot(up)) continue;
        minpos = wave_min(minpos);
        const int T = wave_max(maxend) - minpos;          // :458-459
        const int64_t *col_off = DUPLEX ? a.in.ds_col_off : a.in.ss_col_off;
        const int64_t off = col_off[rec];
        if (T > col_off[rec + 1] - off) continue;
        if (decide_record<DUPLEX>(a, rec, R, T, minpos, a.ws.cons + off, s_stage[wave], s_wtab, lane) && lane == 0)
            a.ws.ovf[i] = (int)rec | (int)0x80000000u;
    }
}

// k_decide for deep single-strand records (R >= kDeepReads, queued by
// k_decide): one 8-wave block per record, two blocks per CU.  Wave w adds the
// rows of reads [R w / 8, R (w + 1) / 8) (decide_accumulate with the packed
// row table, its own LDS stage); the integer partial sums meet in LDS
// (ds_add_u32, exact: the sums are order-free) and wave 0 decides.  A
// 1,000-read subfamily no longer sets the pass's length on one wave (C4).
template <int NT, class Mark>
__device__ void decide_deep_record(const Args &a, const int i, const int64_t rec, const int R, const int T,
                                   const int minpos, uint16_t *stage, const uint32_t *s_wtab, const uint8_t *tab,
                                   uint32_t *s_acc, int *s_fail, const int wave, const int lane, Mark mark) {
    DecideAcc A[NT];
    const int r0 = (int)((int64_t)R * wave / kDeepWaves), r1 = (int)((int64_t)R * (wave + 1) / kDeepWaves);
    const bool ok = decide_accumulate_tab<NT>(a, rec, r0, r1, T, minpos, stage, tab, s_acc, lane);
    if (!ok && lane == 0) *s_fail = 1;
    mark();
    __syncthreads();
    if (wave == 0 && *s_fail == 0) {
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
            const uint32_t *c = s_acc + 64 * tt + lane;
#pragma unroll
            for (int k = 0; k < 5; ++k) A[tt].s[k] = c[256 * k];
#pragma unroll
            for (int k = 0; k < 6; ++k) A[tt].n[k] = c[256 * (5 + k)];
            A[tt].z = c[256 * 11];
        }
        const int64_t off = a.in.ss_col_off[rec];
        if (decide_columns<NT>(a, R, T, A, a.ws.cons + off, lane) && lane == 0) a.ws.ovf[i] = (int)rec | (int)0x80000000u;
    }
}

__global__ __launch_bounds__(kDeepWaves * kWave, 2 * kDeepWaves / 4) void k_decide_deep(Args a) {
    __shared__ uint32_t s_wtab[DCR_LUT_N];
    __shared__ __attribute__((aligned(16))) uint16_t s_stage[kDeepWaves][kStageElems];
    __shared__ uint32_t s_acc[12 * 256];        // per column: s[5], n[6], z
    __shared__ int s_red[4];                    // min pos, max end, unusable read, failed wave
    __shared__ __attribute__((aligned(16))) uint8_t s_tab[kTabBytes];
    if (a.t16 < 0) return;
    for (int i = threadIdx.x; i < DCR_LUT_N; i += blockDim.x) s_wtab[i] = a.wtab[i];
    {
        const int minbq = a.P->min_base_quality;
        for (int i = threadIdx.x; i < kTabBytes / 32; i += blockDim.x) deep_tab_row(s_tab, i, a.wtab, minbq);
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int n = *a.ws.deep_count;
    const bool aligned = ((((uintptr_t)a.in.bases) | ((uintptr_t)a.in.quals)) & 3) == 0;
    uint64_t st_acc[4] = {0, 0, 0, 0}, st_t = 0;           // DCR_STAMP builds: cycles per phase
    auto stamp = [&](int ph) {
        if (DCR_STAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (ph > 0) st_acc[ph - 1] += now - st_t;
            st_t = now;
        }
    };
    for (int k = blockIdx.x; k < n; k += gridDim.x) {
        stamp(0);
        const int i = a.ws.deep[k];
        const int64_t rec = a.ws.ovf[i];
        const int g0 = a.in.sub_off[rec];
        const int R = a.in.sub_off[rec + 1] - g0;
        for (int j = threadIdx.x; j < 12 * 256; j += blockDim.x) s_acc[j] = 0;
        if (threadIdx.x == 0) {
            s_red[0] = 0x7fffffff;
            s_red[1] = -0x7fffffff;
            s_red[2] = 0;
            s_red[3] = 0;
        }
        __syncthreads();
        // k_decide's checks over the whole block (:458-459 for T)
        int minpos = 0x7fffffff, maxend = -0x7fffffff, up = 0;
        for (int r = threadIdx.x; r < R; r += blockDim.x) {
            const ReadRef rd = get_read<false>(a, rec, r);
            up |= rd.status != 0 || rd.len <= 0 || a.ws.info[g0 + r].has_ins;
            minpos = min(minpos, rd.pos);
            maxend = max(maxend, rd.pos + rd.len);
        }
        minpos = wave_min(minpos);
        maxend = wave_max(maxend);
        const bool wup = __ballot(up) != 0;
        if (lane == 0) {
            atomicMin(&s_red[0], minpos);
            atomicMax(&s_red[1], maxend);
            if (wup) s_red[2] = 1;
        }
        __syncthreads();
        const int mp = s_red[0];
        const int T = s_red[1] - mp;
        const int64_t off = a.in.ss_col_off[rec];
        const bool take = !s_red[2] && aligned && R <= 4095 && T > 0 && T <= 256 && T <= a.in.ss_col_off[rec + 1] - off;
        stamp(1);                               // [0] checks over the reads
        if (take) {                             // block-uniform
            uint16_t *st = s_stage[wave];
            auto mk = [&]() { stamp(2); };      // [1] the wave's rows (decide_accumulate_tab)
            if (T <= 64) decide_deep_record<1>(a, i, rec, R, T, mp, st, s_wtab, s_tab, s_acc, &s_red[3], wave, lane, mk);
            else if (T <= 128) decide_deep_record<2>(a, i, rec, R, T, mp, st, s_wtab, s_tab, s_acc, &s_red[3], wave, lane, mk);
            else if (T <= 192) decide_deep_record<3>(a, i, rec, R, T, mp, st, s_wtab, s_tab, s_acc, &s_red[3], wave, lane, mk);
            else decide_deep_record<4>(a, i, rec, R, T, mp, st, s_wtab, s_tab, s_acc, &s_red[3], wave, lane, mk);
        }
        __syncthreads();                        // s_acc / s_red reused by the next record
        stamp(3);                               // [2] the rest (the decision on wave 0, barriers)
    }
    if (DCR_STAMP && lane == 0)
        for (int q = 0; q < 3; ++q) atomicAdd(&a.ws.stamps[26 + q], (unsigned long long)st_acc[q]);
}

template __global__ void k_recmeta<false>(Args);
template __global__ void k_recmeta<true>(Args);
template __global__ void k_consensus_fast<false, false>(FastArgs);
template __global__ void k_consensus_fast<true, false>(FastArgs);
template __global__ void k_consensus_fast<false, true>(FastArgs);
template __global__ void k_consensus_fast<true, true>(FastArgs);
template __global__ void k_consensus_general<false>(Args);
template __global__ void k_decide<false>(Args);
template __global__ void k_decide<true>(Args);
template __global__ void k_ins_layout<false>(Args);
template __global__ void k_ins_layout<true>(Args);
template __global__ void k_consensus_general<true>(Args);

}  // namespace dcr
