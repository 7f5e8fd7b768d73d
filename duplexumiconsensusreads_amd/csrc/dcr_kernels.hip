// dcr_kernels.hip — gfx950 (MI355X) kernels of the duplex-consensus hot path.
//
// Reference: /root/reference/DuplexUMIConsensusReads.py (":line" below).
//
//   k_prep       one lane per read: remove_clipping / mask / trim_3prime_N
//                (:191-325) -> kept sequence window + normalised M/I/D runs.
//   k_consensus  one wavefront per consensus record (single-strand: one
//                subfamily; duplex: one A1+B2 / B1+A2 pair).  Phases:
//                  1. column layout of reconstruct_alignment (:430-547)
//                  2. per-column likelihood products in read order + posterior,
//                     masking and output quality (:550-712)
//                  3. field layout: trims, CIGAR, seq/qual (:716-871),
//                     depth/errors and their pairwise mean (:970-1021), MAPQ
//                     (:874-889).
// All arithmetic is IEEE binary64 in the reference's operation order; build
// with -ffp-contract=off (no FMA contraction).  No transcendental is
// evaluated on device: p', thresholds and the phred rounding boundaries are
// host tables (params.py).
//
// Data flow per wave (lane = column for phase 2/3; lane = read for setup and
// for the insertion-aware layout of phase 1):
//   fast layout  (no I op in the record): element (r, t) is computed directly
//                from the read's M/D runs — no per-column simulation;
//   ins layout   (some read has an I op): the reference's column loop is run
//                with lane = read and a wave ballot per column deciding
//                insertion columns (:476-478), materialising a 64x64 tile of
//                (class, LUT row) codes in LDS that phase 2 consumes by column.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dcr.h"

namespace dcr {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// element code: bits 0..8 LUT row (quality 0..255, 256 '+', 257 '-'), bits 9..11 class
// class: 0 A, 1 T, 2 C, 3 G, 4 '+', 5 '-', 6 N/n, 7 invalid character (:580-591)
constexpr uint32_t kPad = (6u << 9) | 2u;          // 'N' with quality 2 (:509-510, :543-544)
constexpr uint32_t kPlus = (4u << 9) | DCR_LUT_PLUS;
constexpr uint32_t kDel = (5u << 9) | DCR_LUT_DEL;

struct Workspace {
    dcr_read_info *info;    // [n_reads]
    uint32_t *norm_cig;     // [n_cigar] normalised runs (M/I/D)
    int32_t *cons;          // [cols] consensus char | quality << 8 (pre-layout)
    double *et;             // [cols] e/d per kept column
    uint8_t *insflag;       // [ss cols] insertion-column flags (R > 64 layout)
    int4 *state;            // [n_reads] layout state (R > 64)
    int *err;               // [1] capacity error flag
};

struct Args {
    dcr_batch in;
    const dcr_params *P;
    Workspace ws;
    dcr_out ss;
    dcr_out ds;
    int64_t n_rec;
};

__device__ __forceinline__ uint32_t base_class(uint8_t b) {
    switch (b) {
    case 'A': return 0;
    case 'T': return 1;
    case 'C': return 2;
    case 'G': return 3;
    case 'N': return 6;
    default: return 7;
    }
}

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

__device__ __forceinline__ int wave_min(int v) {
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ long long wave_sum(long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// wave-local ordering of global/LDS traffic between phases of one wavefront
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ k_prep
// remove_clipping (:191-265): drop H; drop S with its bases (5'/3' ends);
// mask_low_quality_bases (:268-289): base -> 'N' if qual < min_base_quality
// (applied lazily by the consumer); trim_3prime_N (:292-325): drop trailing
// 'N' and cut as many entries from the END of the expanded CIGAR.
__global__ __launch_bounds__(256) void k_prep(dcr_batch in, const dcr_params *P, Workspace ws) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n_reads) return;
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

// ------------------------------------------------------------ read access
struct ReadRef {
    int pos, len, ncig, mapq, status;
    const uint32_t *cig;
    const uint8_t *seq, *qual;
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
        rd.seq = a.ss.seq + off;
        rd.qual = a.ss.qual + off;
    }
    return rd;
}

// element of read rd at seq index is (M op): class + LUT row; masking only
// for single-strand input reads (mask_low_quality_bases :280)
template <bool DUPLEX>
__device__ __forceinline__ uint32_t base_elem(const ReadRef &rd, int is, int minbq) {
    const uint32_t b = rd.seq[is];
    const uint32_t q = rd.qual[is];
    uint32_t cls = base_class((uint8_t)b);
    if (!DUPLEX && (int)q < minbq) cls = 6;
    return (cls << 9) | q;
}

// ------------------------------------------------ reconstruct_alignment state
// lane = read.  Mirrors idx_cigar / idx_seq (:465-466) with run-length CIGAR.
struct Sim {
    int k, o, is, curop, curlen;
};

__device__ __forceinline__ void sim_load_run(Sim &s, const ReadRef &rd) {
    if (s.k < rd.ncig) {
        const uint32_t v = rd.cig[s.k];
        s.curop = v & 15;
        s.curlen = v >> 4;
    } else {
        s.curop = -1;     // exhausted: get_current_CIGAR_operations reports 0 (:424-425)
        s.curlen = 0;
    }
}
__device__ __forceinline__ void sim_advance(Sim &s, const ReadRef &rd) {
    if (++s.o == s.curlen) {
        ++s.k;
        s.o = 0;
        sim_load_run(s, rd);
    }
}

// one column of :473-545 for one read; returns the element code
template <bool DUPLEX>
__device__ __forceinline__ uint32_t sim_step(Sim &s, const ReadRef &rd, int p, bool ins_col,
                                             int minbq, bool &idx_err) {
    uint32_t e;
    if (ins_col) {                                   // :478-499
        if (s.curop == 1) {
            if (s.is >= rd.len) { idx_err = true; return kPad; }
            e = base_elem<DUPLEX>(rd, s.is, minbq);
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
            e = base_elem<DUPLEX>(rd, s.is, minbq);
            ++s.is;
        }
        sim_advance(s, rd);
    } else {                                         // :540-544
        e = kPad;
    }
    return e;
}

// element (r, t) of a record without insertion columns: the read's op index
// at column t is j = t - (pos - min_pos); its seq index is the number of M
// ops before j.  Once that reaches len the read pads (:514, :540).
template <bool DUPLEX>
__device__ __forceinline__ uint32_t direct_elem(const ReadRef &rd, int j, int minbq) {
    if (j < 0) return kPad;
    int is;
    int op;
    if (rd.ncig == 1) {
        op = rd.cig[0] & 15;
        is = j;
        if (j >= (int)(rd.cig[0] >> 4)) return kPad;
    } else {
        int acc = 0, accis = 0;
        op = -1;
        is = 0;
        for (int k = 0; k < rd.ncig; ++k) {
            const uint32_t v = rd.cig[k];
            const int ln = v >> 4, o = v & 15;
            if (op < 0 && j < acc + ln) {
                op = o;
                is = accis + (o == 0 ? j - acc : 0);
            }
            acc += ln;
            if (o == 0) accis += ln;
        }
        if (op < 0) return kPad;
        if (op == 2 && accis == 0) { /* deletion before any base: is = 0 */ }
    }
    if (is >= rd.len) return kPad;
    if (op == 2) return kDel;
    return base_elem<DUPLEX>(rd, is, minbq);
}

// --------------------------------------------------------------- phase 2
struct Acc {
    double L0, L1, L2, L3, L4, L5;
    int c0, c1, c2, c3, c4, c5, c6;
    int bad;
};

__device__ __forceinline__ void acc_init(Acc &A) {
    A.L0 = A.L1 = A.L2 = A.L3 = A.L4 = A.L5 = 1.0;
    A.c0 = A.c1 = A.c2 = A.c3 = A.c4 = A.c5 = A.c6 = 0;
    A.bad = 0;
}

// most_likely_nucleotide (:594-600): likelihoods multiplied in read order
__device__ __forceinline__ void acc_add(Acc &A, uint32_t e, const double2 *lut) {
    const uint32_t cls = e >> 9;
    const double2 f = lut[e & 511];
    A.L0 *= (cls == 0) ? f.x : f.y;
    A.L1 *= (cls == 1) ? f.x : f.y;
    A.L2 *= (cls == 2) ? f.x : f.y;
    A.L3 *= (cls == 3) ? f.x : f.y;
    A.L4 *= (cls == 4) ? f.x : f.y;
    A.L5 *= (cls == 5) ? f.x : f.y;
    A.c0 += (cls == 0);
    A.c1 += (cls == 1);
    A.c2 += (cls == 2);
    A.c3 += (cls == 3);
    A.c4 += (cls == 4);
    A.c5 += (cls == 5);
    A.c6 += (cls == 6);
    A.bad |= (cls == 7);
}

struct ColOut {
    int ch, q, d, e;
    bool overflow;
};

// posterior, mask, output quality (:603-621, :699-709), depth/errors (:1001-1012)
__device__ __forceinline__ ColOut finalize(const Acc &A, int R, bool ins_col, const dcr_params *P,
                                           const double *qthr) {
    ColOut o;
    double S = A.L0 + A.L1;                      // np.sum of 6: left to right (:608)
    S = S + A.L2;
    S = S + A.L3;
    S = S + A.L4;
    S = S + A.L5;
    const double p[6] = {A.L0 / S, A.L1 / S, A.L2 / S, A.L3 / S, A.L4 / S, A.L5 / S};
    int best = 0;                                // np.argmax: first NaN, else first max
    double pm = p[0];
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
    const bool has_plus = A.c4 > 0;              // '+' in nucleotides (:613, :618)
    int ch = "ATCG+-"[best];
    if (has_plus && best < 4) ch += 32;
    if (pm < P->post_threshold) ch = has_plus ? 'n' : 'N';
    // consensus quality (:700-709)
    const double e = 1.0 - pm;
    const double pre = (double)P->error_rate_pre_labeling;
    const double post = (double)P->error_rate_post_labeling;
    const double x = pre * (1.0 - e) + (1.0 - post) * e + pre * e * 4.0 / 5.0;
    int q = P->max_base_quality;
    o.overflow = false;
    if (x > 0.0) {
        if (__builtin_isinf(x)) {
            o.overflow = true;
        } else {
            int lo = 0, hi = P->n_qthresh;       // qthr decreasing: first i with qthr[i] <= x
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (qthr[mid] <= x) hi = mid; else lo = mid + 1;
            }
            q = P->max_base_quality - (P->n_qthresh - lo);
        }
    }
    o.ch = ch;
    o.q = q;
    // depth: rows not in {N, n, +}; errors: rows != consensus char (case-sensitive)
    o.d = R - A.c6 - A.c4;
    int kc;
    switch (ch) {
    case 'A': case 'a': kc = 0; break;
    case 'T': case 't': kc = 1; break;
    case 'C': case 'c': kc = 2; break;
    case 'G': case 'g': kc = 3; break;
    case '+': kc = 4; break;
    case '-': kc = 5; break;
    default: kc = 6; break;
    }
    const bool lower = ch >= 'a';
    int match = 0;
    const int cnt[7] = {A.c0, A.c1, A.c2, A.c3, A.c4, A.c5, A.c6};
    // row characters: insertion columns hold lowercase bases / 'n' / '+',
    // normal columns uppercase bases / 'N' / '-'
    if (kc == 4) match = cnt[4];
    else if (kc == 5) match = ins_col ? 0 : cnt[5];
    else match = (lower == ins_col) ? cnt[kc] : 0;
    o.e = R - match;
    return o;
}

// ------------------------------------------------------------ k_consensus
template <bool DUPLEX>
__global__ __launch_bounds__(kBlock) void k_consensus(Args a) {
    __shared__ double2 s_lut[DCR_LUT_N];
    __shared__ double s_qthr[DCR_MAX_QTHRESH];
    __shared__ uint16_t s_tile[kWavesPerBlock][kWave][kWave];

    const dcr_params *P = a.P;
    for (int i = threadIdx.x; i < DCR_LUT_N; i += kBlock) s_lut[i] = make_double2(P->match[i], P->mismatch[i]);
    for (int i = threadIdx.x; i < DCR_MAX_QTHRESH; i += kBlock) s_qthr[i] = P->qthresh[i];
    __syncthreads();

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t rec = (int64_t)blockIdx.x * kWavesPerBlock + wave;
    if (rec >= a.n_rec) return;

    dcr_out &O = DUPLEX ? a.ds : a.ss;
    const int64_t* col_off = DUPLEX ? a.in.ds_col_off : a.in.ss_col_off;
    const int64_t off = col_off[rec];
    const int64_t cap = col_off[rec + 1] - off;
    const int minbq = P->min_base_quality;
    uint16_t(*tile)[kWave] = s_tile[wave];

    const int R = DUPLEX ? 2 : (a.in.sub_off[rec + 1] - a.in.sub_off[rec]);

    // ---- setup: lane = read
    int minpos = 0x7fffffff, maxend = -0x7fffffff, up = 0, empty = 0, ins = 0;
    long long msum = 0;
    for (int c = 0; c < R; c += kWave) {
        const int r = c + lane;
        if (r < R) {
            const ReadRef rd = get_read<DUPLEX>(a, rec, r);
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
    if (R == 0 || up) { write_status(DCR_ST_UPSTREAM); return; }
    if (empty) { write_status(DCR_ST_TYPE_ERROR); return; }     // list(None) at :402
    const int T = maxend - minpos;                                  // :458-459
    if (T > cap) {
        if (lane == 0) atomicOr(a.ws.err, 1);
        write_status(255);
        return;
    }

    int32_t *cons = a.ws.cons + off;
    double *et = a.ws.et + off;
    uint16_t *od = O.d + off;
    uint16_t *oe = O.e + off;

    bool idx_err = false;      // IndexError inside reconstruct_alignment
    int bad = 0;               // invalid nucleotide somewhere (:582)
    int n_de = 0, Dmax = -1, Dmin = 0x7fffffff;
    int first = -1, last = -1;
    bool qoverflow = false;    // int(-inf) consensus quality

    // R > 64 with insertion columns: precompute the insertion-column flags
    // (all reads must be consulted per column, :476-478) and keep per-read
    // layout state in global scratch between column tiles.
    const bool big = R > kWave;
    uint8_t *insflag = a.ws.insflag + off;
    int4 *gstate = DUPLEX ? nullptr : a.ws.state + a.in.sub_off[rec];
    if (ins && big && !DUPLEX) {
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
    ReadRef myrd;
    if (ins && !big) {
        if (lane < R) {
            myrd = get_read<DUPLEX>(a, rec, lane);
            sim_load_run(sim, myrd);
        }
    }

    // ---- phases 1+2: column tiles (lane = column)
    for (int c0 = 0; c0 < T; c0 += kWave) {
        const int t = c0 + lane;
        const bool live = t < T;
        const int ncol = min(kWave, T - c0);
        Acc A;
        acc_init(A);
        bool ins_col = false;
        if (!ins) {
            for (int r = 0; r < R; ++r) {
                const ReadRef rd = get_read<DUPLEX>(a, rec, r);
                const uint32_t e = live ? direct_elem<DUPLEX>(rd, t - (rd.pos - minpos), minbq) : kPad;
                acc_add(A, e, s_lut);
            }
        } else if (!big) {
            uint64_t insmask = 0;
            for (int tt = 0; tt < ncol; ++tt) {
                const bool isI = lane < R && sim.curop == 1;
                const bool any = __ballot(isI) != 0;
                insmask |= (uint64_t)any << tt;
                if (lane < R) tile[lane][tt] = (uint16_t)sim_step<DUPLEX>(sim, myrd, minpos + c0 + tt, any, minbq, idx_err);
            }
            wave_fence();
            ins_col = (insmask >> lane) & 1;
            for (int r = 0; r < R; ++r) acc_add(A, live ? tile[r][lane] : kPad, s_lut);
            wave_fence();
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
                        tile[lane][tt] = (uint16_t)sim_step<DUPLEX>(s, rd, minpos + c0 + tt, insflag[c0 + tt] != 0,
                                                                    minbq, idx_err);
                    gstate[r] = make_int4(s.k, s.o, s.is, 0);
                }
                wave_fence();
                for (int rr = 0; rr < nr; ++rr) acc_add(A, live ? tile[rr][lane] : kPad, s_lut);
                wave_fence();
            }
        }
        bad |= A.bad && live;
        const ColOut co = finalize(A, R, ins_col, P, s_qthr);
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
        }
        n_de += __popcll(km);
        Dmax = max(Dmax, wave_max(keep ? co.d : -1));
        Dmin = min(Dmin, wave_min(keep ? co.d : 0x7fffffff));
        // 5'/3' trims count uppercase 'N' only (:770-784)
        const uint64_t nn = __ballot(live && co.ch != 'N');
        if (nn) {
            if (first < 0) first = c0 + __builtin_ctzll(nn);
            last = c0 + 63 - __builtin_clzll(nn);
        }
    }
    idx_err = __ballot(idx_err) != 0;
    bad = __ballot(bad) != 0;
    qoverflow = __ballot(qoverflow) != 0;
    if (idx_err) { write_status(DCR_ST_INDEX_ERROR); return; }
    if (bad) { write_status(DCR_ST_EXIT_BADCHAR); return; }
    wave_fence();

    // ---- phase 3: adjust_consensus_fields (:745-871) over [first, last]
    const int lo = first < 0 ? T : first;
    const int hi = first < 0 ? T : last + 1;
    uint8_t *oseq = O.seq + off;
    uint8_t *oqual = O.qual + off;
    uint32_t *ocig = O.cigar + off;
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
            ocig[ri] = ((uint32_t)oi << 4) | (uint32_t)op;        // run start, converted below
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
    if (kept_overflow || qoverflow) { write_status(DCR_ST_OVERFLOW_ERROR); return; }
    wave_fence();
    for (int i0 = 0; i0 < nruns; i0 += kWave) {
        const int i = i0 + lane;
        uint32_t v = 0, nx = 0;
        if (i < nruns) {
            v = ocig[i];
            nx = i + 1 < nruns ? (ocig[i + 1] >> 4) : (uint32_t)nops;
        }
        wave_fence();
        if (i < nruns) ocig[i] = ((nx - (v >> 4)) << 4) | (v & 15);
    }

    // ---- E = round(mean(e/d), 3) with numpy's pairwise summation (:1015-1018)
    wave_fence();
    double total;
    {
        // explicit-stack form of numpy's pairwise_sum recursion (blocks of <= 128,
        // 8 accumulators, split at n/2 rounded down to a multiple of 8)
        int st_off[24], st_n[24], st_stage[24];
        double st_left[24];
        int sp = 0;
        st_off[0] = 0; st_n[0] = n_de; st_stage[0] = 0; st_left[0] = 0.0;
        double ret = 0.0;
        while (sp >= 0) {
            const int fo = st_off[sp], fn = st_n[sp];
            if (fn <= 128) {
                double res;
                if (fn < 8) {
                    res = -0.0;
                    for (int i = 0; i < fn; ++i) res += et[fo + i];
                } else {
                    const int body = fn - (fn % 8);
                    double r = 0.0;
                    if (lane < 8) {
                        r = et[fo + lane];
                        for (int i = 8; i < body; i += 8) r += et[fo + i + lane];
                    }
                    const double r0 = __shfl(r, 0), r1 = __shfl(r, 1), r2 = __shfl(r, 2), r3 = __shfl(r, 3);
                    const double r4 = __shfl(r, 4), r5 = __shfl(r, 5), r6 = __shfl(r, 6), r7 = __shfl(r, 7);
                    res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
                    for (int i = body; i < fn; ++i) res += et[fo + i];
                }
                ret = res;
                --sp;
                continue;
            }
            int n2 = fn / 2;
            n2 -= n2 % 8;
            if (st_stage[sp] == 0) {
                st_stage[sp] = 1;
                ++sp;
                st_off[sp] = fo; st_n[sp] = n2; st_stage[sp] = 0;
            } else if (st_stage[sp] == 1) {
                st_left[sp] = ret;
                st_stage[sp] = 2;
                ++sp;
                st_off[sp] = fo + n2; st_n[sp] = fn - n2; st_stage[sp] = 0;
            } else {
                ret = st_left[sp] + ret;
                --sp;
            }
        }
        total = 0.0 + ret;
    }
    const double mean = total / (double)n_de;
    const double E = __builtin_rint(mean * 1000.0) / 1000.0;

    if (lane == 0) {
        O.status[rec] = DCR_ST_OK;
        O.pos[rec] = minpos + lo;                   // :790
        O.mapq[rec] = (int)(msum / R);              // trunc(np.mean) (:887, :1377)
        O.len[rec] = nlen;
        O.n_cig[rec] = nruns;
        O.n_de[rec] = n_de;
        O.D[rec] = Dmax;
        O.M[rec] = Dmin;
        O.E[rec] = E;
    }
}

template __global__ void k_consensus<false>(Args);
template __global__ void k_consensus<true>(Args);

}  // namespace dcr
