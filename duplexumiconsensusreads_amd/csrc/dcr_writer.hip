// dcr_writer.hip — the record writer on the GPU: the two duplex BAM records
// of every family of a batch formatted straight from the kernel outputs in
// HBM, the failure scan, and the BGZF compression of the record stream
// (dcr_deflate.h), so that only compressed blocks cross PCIe.
//
// Reference (/root/reference/DuplexUMIConsensusReads.py): record fields
// make_consensus_read :1352-1384, names / flags :892-968, duplex tags
// add_tags :1076-1120, mate fields fix_paired_end_fields :1390-1419.  The
// byte layout is exactly the host formatter's (csrc/dcr_format.cpp), which
// tests/test_cli_e2e.py pins to the Python record codec.
#include <hip/hip_runtime.h>

#include "dcr_deflate.h"
#include "dcr_internal.h"
#include "dcr_writer.h"

namespace dcrw {

constexpr int kW = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kW - 1); }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < kW; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, kW);
        if (l >= d) v += t;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kW);
    return v;
}

__device__ __forceinline__ uint32_t ndigits(uint32_t v) {
    return v < 10 ? 1 : v < 100 ? 2 : v < 1000 ? 3 : v < 10000 ? 4 : v < 100000 ? 5 : v < 1000000 ? 6 : 10;
}
__device__ __forceinline__ uint32_t int_tag_bytes(int64_t v) {
    if (v < 0) return v >= -128 ? 4 : v >= -32768 ? 5 : 7;
    return v <= 255 ? 4 : v <= 65535 ? 5 : 7;
}

__device__ __forceinline__ int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

__device__ __forceinline__ uint8_t nt_code(uint8_t c) {
    // "=ACMGRSVTWYHKDBN" (either case), unknown letters 15
    switch (c | 0x20) {
        case 'a': return 1; case 'c': return 2; case 'm': return 3; case 'g': return 4; case 'r': return 5;
        case 's': return 6; case 'v': return 7; case 't': return 8; case 'w': return 9; case 'y': return 10;
        case 'h': return 11; case 'k': return 12; case 'd': return 13; case 'b': return 14; case 'n': return 15;
        default: return c == '=' ? 0 : 15;
    }
}

__device__ __forceinline__ uint32_t dstrlen(const char *s) {
    uint32_t n = 0;
    while (s[n]) ++n;
    return n;
}

// text bytes of a "[1, 2, 3]" list (digits and separators only)
__device__ uint32_t list_body(const uint16_t *v, int32_t n) {
    uint32_t t = 0;
    for (int32_t i = lane_id(); i < n; i += kW) t += ndigits(v[i]);
    t = wave_sum(t);
    return t + (n > 0 ? 2u * (uint32_t)(n - 1) : 0u);
}

struct Rec {
    int32_t k, f, j, a, b;
    int32_t L, nc, tid, pos, opos, tlen, mapq;
    int64_t ro, ao, bo;
    const char *code, *rx;
    uint32_t lc, lr;
    int32_t a0, a1, b0, b1;
};

__device__ void rec_setup(const FmtArgs &A, int32_t k, Rec &r) {
    r.k = k;
    r.f = k >> 1;
    r.j = k & 1;
    r.a = 4 * r.f + 2 * r.j;
    r.b = r.a + 1;
    r.L = A.ds.len[k];
    r.nc = A.ds.n_cig[k];
    r.tid = A.fam_tid[r.f];
    r.pos = A.ds.pos[k];
    r.opos = A.ds.pos[2 * r.f + 1 - r.j];
    const int32_t t = A.ds.pos[2 * r.f + 1] + A.ds.len[2 * r.f + 1] - A.ds.pos[2 * r.f];
    r.tlen = r.j == 0 ? t : -t;
    r.mapq = A.ds.mapq[k];
    r.ro = A.ds_col_off[k];
    r.ao = A.ss_col_off[r.a];
    r.bo = A.ss_col_off[r.b];
    r.code = A.names + A.fam_code[r.f];
    r.rx = A.names + A.fam_rx[2 * r.f + r.j];
    r.lc = dstrlen(r.code);
    r.lr = dstrlen(r.rx);
    r.a0 = A.sub_off[r.a];
    r.a1 = A.sub_off[r.a + 1];
    r.b0 = A.sub_off[r.b];
    r.b1 = A.sub_off[r.b + 1];
}

__device__ uint32_t rec_size(const FmtArgs &A, const Rec &r) {
    const dcr_out &ss = A.ss, &ds = A.ds;
    uint32_t n = 36 + 16 + r.lc + 12 + 1 + 4u * (uint32_t)r.nc + (uint32_t)((r.L + 1) >> 1) + (uint32_t)r.L;
    n += 3 + r.lc + 1 + 3 + r.lr + 1;                                  // MI, RX
    n += 8 + (uint32_t)(r.a1 - r.a0) + 8 + (uint32_t)(r.b1 - r.b0) + 8 + 2;   // aQ bQ cQ
    const uint16_t *dl[3] = {ss.d + r.ao, ss.d + r.bo, ds.d + r.ro};
    const uint16_t *el[3] = {ss.e + r.ao, ss.e + r.bo, ds.e + r.ro};
    const int32_t nn[3] = {ss.n_de[r.a], ss.n_de[r.b], ds.n_de[r.k]};
    for (int i = 0; i < 3; ++i) n += 6 + list_body(dl[i], nn[i]);
    for (int i = 0; i < 3; ++i) n += 6 + list_body(el[i], nn[i]);
    n += int_tag_bytes(ss.D[r.a]) + int_tag_bytes(ss.D[r.b]) + int_tag_bytes(ds.D[r.k]);
    n += int_tag_bytes(ss.M[r.a]) + int_tag_bytes(ss.M[r.b]) + int_tag_bytes(ds.M[r.k]);
    n += 3 * 7;
    n += 2 * (4 + (uint32_t)ss.len[r.a]) + 2 * (4 + (uint32_t)ss.len[r.b]);   // ac bc aq bq
    return n;
}

// byte writer: scalar pieces by lane 0, arrays by the whole wave
struct Out {
    uint8_t *o;
    uint32_t p;
    __device__ void b1(uint32_t v) {
        if (lane_id() == 0) o[p] = (uint8_t)v;
        p += 1;
    }
    __device__ void u16(uint32_t v) {
        if (lane_id() == 0) { o[p] = (uint8_t)v; o[p + 1] = (uint8_t)(v >> 8); }
        p += 2;
    }
    __device__ void u32(uint32_t v) {
        if (lane_id() == 0)
            for (int i = 0; i < 4; ++i) o[p + i] = (uint8_t)(v >> (8 * i));
        p += 4;
    }
    __device__ void str(const char *s, uint32_t n) {
        for (uint32_t i = lane_id(); i < n; i += kW) o[p + i] = (uint8_t)s[i];
        p += n;
    }
    __device__ void bytes(const uint8_t *s, uint32_t n) {
        for (uint32_t i = lane_id(); i < n; i += kW) o[p + i] = s[i];
        p += n;
    }
    __device__ void tag(char a, char b, char t) { b1((uint8_t)a); b1((uint8_t)b); b1((uint8_t)t); }
    __device__ void int_tag(char a, char b, int64_t v) {
        b1((uint8_t)a);
        b1((uint8_t)b);
        if (v < 0) {
            if (v >= -128) { b1('c'); b1((uint8_t)(int8_t)v); }
            else if (v >= -32768) { b1('s'); u16((uint16_t)(int16_t)v); }
            else { b1('i'); u32((uint32_t)(int32_t)v); }
        } else if (v <= 255) { b1('C'); b1((uint32_t)v); }
        else if (v <= 65535) { b1('S'); u16((uint32_t)v); }
        else { b1('I'); u32((uint32_t)v); }
    }
    __device__ void float_tag(char a, char b, double v) {
        b1((uint8_t)a);
        b1((uint8_t)b);
        b1('f');
        const float f = (float)v;
        u32(__float_as_uint(f));
    }
    __device__ void list(char a, char b, const uint16_t *v, int32_t n) {
        tag(a, b, 'Z');
        b1('[');
        for (int32_t c0 = 0; c0 < n; c0 += kW) {
            const int32_t i = c0 + lane_id();
            uint32_t x = 0, len = 0;
            if (i < n) {
                x = v[i];
                len = ndigits(x) + (i > 0 ? 2u : 0u);
            }
            const uint32_t incl = wave_incl_scan(len);
            const uint32_t tot = __shfl(incl, kW - 1, kW);
            if (i < n) {
                uint8_t *q = o + p + (incl - len);
                if (i > 0) { q[0] = ','; q[1] = ' '; q += 2; }
                const uint32_t nd = ndigits(x);
                for (int d = (int)nd - 1; d >= 0; --d) { q[d] = (uint8_t)('0' + x % 10); x /= 10; }
            }
            p += tot;
        }
        b1(']');
        b1(0);
    }
};

__device__ void rec_write(const FmtArgs &A, const Rec &r, uint8_t *o, uint32_t total) {
    const dcr_out &ss = A.ss, &ds = A.ds;
    Out w{o, 0};
    w.u32(total - 4);
    w.u32((uint32_t)r.tid);
    w.u32((uint32_t)r.pos);
    w.b1(16 + r.lc + 12 + 1);
    w.b1((uint32_t)(r.mapq & 0xff));
    const uint32_t *cg = ds.cigar + r.ro;
    int64_t rl = 0;
    if (lane_id() == 0)
        for (int32_t i = 0; i < r.nc; ++i) {
            const uint32_t op = cg[i] & 15;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += cg[i] >> 4;
        }
    w.u16(r.pos >= 0 ? (uint32_t)reg2bin(r.pos, r.pos + (rl > 0 ? rl : 1)) : 4680u);
    w.u16((uint32_t)r.nc);
    w.u16(r.j == 0 ? 99u : 147u);
    w.u32((uint32_t)r.L);
    w.u32((uint32_t)r.tid);
    w.u32((uint32_t)r.opos);
    w.u32((uint32_t)r.tlen);
    w.str("consensus_family", 16);
    w.str(r.code, r.lc);
    w.str(r.j == 0 ? "_paired-end1" : "_paired-end2", 12);
    w.b1(0);
    for (int32_t i = lane_id(); i < r.nc; i += kW) {
        const uint32_t v = cg[i];
        for (int b = 0; b < 4; ++b) o[w.p + 4 * i + b] = (uint8_t)(v >> (8 * b));
    }
    w.p += 4u * (uint32_t)r.nc;
    const uint8_t *sq = ds.seq + r.ro;
    const int32_t nb = (r.L + 1) >> 1;
    for (int32_t i = lane_id(); i < nb; i += kW) {
        const uint8_t hi = nt_code(sq[2 * i]);
        const uint8_t lo = (2 * i + 1 < r.L) ? nt_code(sq[2 * i + 1]) : 0;
        o[w.p + i] = (uint8_t)((hi << 4) | lo);
    }
    w.p += (uint32_t)nb;
    w.bytes(ds.qual + r.ro, (uint32_t)r.L);
    w.tag('M', 'I', 'Z');
    w.str(r.code, r.lc);
    w.b1(0);
    w.tag('R', 'X', 'Z');
    w.str(r.rx, r.lr);
    w.b1(0);
    w.tag('a', 'Q', 'B'); w.b1('C'); w.u32((uint32_t)(r.a1 - r.a0)); w.bytes(A.read_mapq + r.a0, (uint32_t)(r.a1 - r.a0));
    w.tag('b', 'Q', 'B'); w.b1('C'); w.u32((uint32_t)(r.b1 - r.b0)); w.bytes(A.read_mapq + r.b0, (uint32_t)(r.b1 - r.b0));
    w.tag('c', 'Q', 'B'); w.b1('C'); w.u32(2); w.b1((uint32_t)ss.mapq[r.a] & 0xff); w.b1((uint32_t)ss.mapq[r.b] & 0xff);
    w.list('a', 'd', ss.d + r.ao, ss.n_de[r.a]);
    w.list('b', 'd', ss.d + r.bo, ss.n_de[r.b]);
    w.list('c', 'd', ds.d + r.ro, ds.n_de[r.k]);
    w.int_tag('a', 'D', ss.D[r.a]); w.int_tag('b', 'D', ss.D[r.b]); w.int_tag('c', 'D', ds.D[r.k]);
    w.int_tag('a', 'M', ss.M[r.a]); w.int_tag('b', 'M', ss.M[r.b]); w.int_tag('c', 'M', ds.M[r.k]);
    w.list('a', 'e', ss.e + r.ao, ss.n_de[r.a]);
    w.list('b', 'e', ss.e + r.bo, ss.n_de[r.b]);
    w.list('c', 'e', ds.e + r.ro, ds.n_de[r.k]);
    w.float_tag('a', 'E', ss.E[r.a]); w.float_tag('b', 'E', ss.E[r.b]); w.float_tag('c', 'E', ds.E[r.k]);
    w.tag('a', 'c', 'Z'); w.bytes(ss.seq + r.ao, (uint32_t)ss.len[r.a]); w.b1(0);
    w.tag('b', 'c', 'Z'); w.bytes(ss.seq + r.bo, (uint32_t)ss.len[r.b]); w.b1(0);
    w.tag('a', 'q', 'Z');
    for (int32_t i = lane_id(); i < ss.len[r.a]; i += kW) o[w.p + i] = (uint8_t)(ss.qual[r.ao + i] + 33);
    w.p += (uint32_t)ss.len[r.a];
    w.b1(0);
    w.tag('b', 'q', 'Z');
    for (int32_t i = lane_id(); i < ss.len[r.b]; i += kW) o[w.p + i] = (uint8_t)(ss.qual[r.bo + i] + 33);
    w.p += (uint32_t)ss.len[r.b];
    w.b1(0);
}

// one wave per duplex record; records of failing families get size 0
__global__ __launch_bounds__(256) void k_fmt_size(FmtArgs A) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kW;
    const int64_t nw = (int64_t)gridDim.x * blockDim.x / kW;
    for (int64_t k = wave; k < 2LL * A.n_fam; k += nw) {
        uint32_t n = 0;
        if (A.fam_fail[k >> 1] == 0) {
            Rec r;
            rec_setup(A, (int32_t)k, r);
            n = rec_size(A, r);
        }
        if (lane_id() == 0) A.rec_size[k] = n;
    }
}

__global__ __launch_bounds__(256) void k_fmt_write(FmtArgs A) {
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kW;
    const int64_t nw = (int64_t)gridDim.x * blockDim.x / kW;
    for (int64_t k = wave; k < 2LL * A.n_fam; k += nw) {
        const int64_t o = A.rec_off[k], n = A.rec_off[k + 1] - o;
        if (n == 0) continue;
        Rec r;
        rec_setup(A, (int32_t)k, r);
        rec_write(A, r, A.stream + o, (uint32_t)n);
    }
}

// the reference's outcome per family, in its execution order (dcr_fmt_scan)
__global__ __launch_bounds__(256) void k_famfail(FmtArgs A) {
    const int32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= A.n_fam) return;
    int32_t kind = 0, which = -1;
    // preprocessing of every read comes first (:1272-1283): the first
    // subfamily holding a failing read (DCR_ST_PREP | its status)
    for (int k = 0; k < 4 && !kind; ++k) {
        const int st = A.ss.status[4 * f + k];
        if (st & DCR_ST_PREP) { kind = st & 15; which = 8 + k; }
    }
    auto st_fail = [](int st) { return st != 0 && st != DCR_ST_UPSTREAM; };
    for (int k = 0; k < 4 && !kind; ++k) {
        const int st = A.ss.status[4 * f + k];
        if (st_fail(st)) { kind = st; which = k; }
    }
    for (int j = 0; j < 2 && !kind; ++j) {
        const int st = A.ds.status[2 * f + j];
        if (st_fail(st)) { kind = st; which = 4 + j; break; }
        for (int s = 4 * f + 2 * j; s < 4 * f + 2 * j + 2 && !kind; ++s) {
            const int64_t o = A.ss_col_off[s];
            for (int32_t i = 0; i < A.ss.len[s]; ++i)
                if (A.ss.qual[o + i] >= 95) { kind = 7; which = 4 + j; break; }   // pysam force_bytes(ascii)
        }
    }
    A.fam_fail[f] = kind ? (kind | (which << 8)) : 0;
    A.ds_len_out[2 * f] = A.ds.len[2 * f];
    A.ds_len_out[2 * f + 1] = A.ds.len[2 * f + 1];
}

// dfl::p4_scan across the workgroup: wave scans of the lanes' bit counts,
// xor of their CRC registers; zeroes the words two lanes share
__device__ __forceinline__ void p4_scan_wg(dfl::Shared &s, uint32_t n, int lane, uint32_t *slot) {
    const uint32_t b = s.lane_bits[lane];
    const uint32_t inc = wave_incl_scan(b);
    uint32_t cx = s.lane_crc[lane];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cx ^= __shfl_xor(cx, d, kW);
    const int w = lane >> 6;
    if ((lane & (kW - 1)) == kW - 1) s.wave_sum[w] = inc;
    if ((lane & (kW - 1)) == 0) s.wave_crc[w] = cx;
    __syncthreads();
    uint32_t base = 3 * 8 * 6 + s.hdr_bits;
    for (int k = 0; k < w; ++k) base += s.wave_sum[k];
    const uint32_t off = base + inc - b;
    s.lane_off[lane] = off;
    if (lane && (off & 31)) {
        slot[off >> 5] = 0;
        if ((off >> 5) < sizeof(s.stage) / 4) s.stage[off >> 5] = 0;
    }
    if (lane == dfl::kT - 1) {
        dfl::decide(s, n, off + b);
        uint32_t c = dfl::multmodp(dfl::x8nmodp(n), 0xffffffffu);
        for (int k = 0; k < dfl::kT / kW; ++k) c ^= s.wave_crc[k];
        s.crc = ~c;
    }
}

// dfl::p3c_header on wave 0 (lanes 0..63): the same greedy run-length
// code of the code lengths, built in parallel.  Runs start where a length
// differs from the one before it (ballots over five chunks of 64 positions);
// each run's lane counts its symbols, an exclusive scan in run order gives
// its offset in rle[], and it writes them; the symbol counts go in by LDS
// atomics.  Lane 0 then finishes as the serial code does (p3c_header_post).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void p3c_header_wave(dfl::Shared &s, int lane) {
    const uint32_t last_lit = s.last_lit, last_dist = s.last_dist;
    const int nlit = last_lit + 1 > 257 ? (int)last_lit + 1 : 257;
    const int ndist = (int)last_dist + 1;
    const int N = nlit + ndist;                       // <= 316: five chunks
    auto L = [&](int i) -> uint32_t { return i < nlit ? s.lit_len[i] : s.dist_len[i - nlit]; };
    uint32_t *clf = s.t0_clf;
    if (lane < 19) clf[lane] = 0;
    if (lane == 0) {
        dfl::first_codes_from_counts(s.num_lit, s.next_code[0]);
        dfl::first_codes_from_counts(s.num_dist, s.next_code[1]);
        s.hlit = (uint32_t)(nlit - 257);
        s.hdist = (uint32_t)(ndist - 1);
    }
    constexpr int kC = 5;
    uint32_t v[kC];
    uint64_t st[kC];                                  // run starts per chunk (uniform)
#pragma unroll
    for (int c = 0; c < kC; ++c) {
        const int i = 64 * c + lane;
        v[c] = i < N ? L(i) : 0xffu;
        const uint32_t pv = (i > 0 && i <= N) ? L(i - 1) : 0xfeu;
        st[c] = __ballot(i < N && v[c] != pv);
    }
    wave_lds_sync();                                  // clf zeroed before the atomics
    uint32_t base = 0;
#pragma unroll
    for (int c = 0; c < kC; ++c) {
        const int i = 64 * c + lane;
        const bool start = (st[c] >> lane) & 1u;
        // the next run start after i: in this chunk above the lane, else in a later chunk, else N
        int nxt = N;
        const uint64_t above = lane == 63 ? 0ull : st[c] & (~0ull << (lane + 1));
        if (above) nxt = 64 * c + (int)__builtin_ctzll(above);
        else {
#pragma unroll
            for (int d = kC - 1; d > c; --d)
                if (st[d]) nxt = 64 * d + (int)__builtin_ctzll(st[d]);
        }
        int run = nxt - i;
        uint32_t ns = 0, n18 = 0, n17 = 0, n16 = 0, nv = 0;
        const uint32_t val = v[c];
        if (start) {
            int r = run;
            if (val == 0) {
                while (r >= 11) { r -= r < 138 ? r : 138; ++n18; }
                if (r >= 3) { ++n17; r = 0; }
                nv = (uint32_t)r;
                ns = n18 + n17 + nv;
            } else {
                --r;
                nv = 1;
                while (r >= 3) { r -= r < 6 ? r : 6; ++n16; }
                nv += (uint32_t)r;
                ns = 1 + n16 + (uint32_t)r;
            }
        }
        const uint32_t inc = wave_incl_scan(ns);
        uint32_t off = base + inc - ns;
        base += __shfl(inc, 63, kW);
        if (start) {
            int r = run;
            if (val == 0) {
                while (r >= 11) { const int t = r < 138 ? r : 138; s.rle[off++] = (uint16_t)(18 | ((t - 11) << 8)); r -= t; }
                if (r >= 3) { s.rle[off++] = (uint16_t)(17 | ((r - 3) << 8)); r = 0; }
                while (r-- > 0) s.rle[off++] = 0;
            } else {
                s.rle[off++] = (uint16_t)val;
                --r;
                while (r >= 3) { const int t = r < 6 ? r : 6; s.rle[off++] = (uint16_t)(16 | ((t - 3) << 8)); r -= t; }
                while (r-- > 0) s.rle[off++] = (uint16_t)val;
            }
            if (n18) atomicAdd(&clf[18], n18);
            if (n17) atomicAdd(&clf[17], n17);
            if (n16) atomicAdd(&clf[16], n16);
            if (nv) atomicAdd(&clf[val], nv);
        }
    }
    wave_lds_sync();
    if (lane == 0) {
        s.n_rle = base;
        dfl::p3c_header_post(s);
    }
}

#ifndef DFL_STAGE4
#define DFL_STAGE4 1      // stage a block 16 bytes per lane per load, four loads in flight
#endif
// one workgroup (256 lanes) per BGZF block of the record stream
__global__ __launch_bounds__(dfl::kT) void k_deflate(DflArgs D) {
    extern __shared__ __align__(16) uint8_t smem[];
    dfl::Shared &s = *reinterpret_cast<dfl::Shared *>(smem);
    const int lane = threadIdx.x;
    const int64_t total = *D.stream_bytes;
    const int64_t nb = (total + dfl::kMaxIn - 1) / dfl::kMaxIn;
    const bool st = D.stamps != nullptr;
    uint32_t *tok = D.tok + (size_t)blockIdx.x * dfl::kTokWords;
    // phase stamps (dcr_deflate_probe): accumulated in LDS by lane 0, not
    // in per-lane registers
    __shared__ uint64_t t[12];
    uint64_t t0 = 0;
    if (st && lane < 12) t[lane] = 0;
#if DFL_CRCS
    static_assert(DFL_CRCS == 4 || DFL_CRCS == 8, "CRC32 slices: 4 or 8");
    // slice-by-N CRC32 tables, once per workgroup: t[0] the byte table,
    // t[k][i] = t[k-1][i] >> 8 ^ t[0][t[k-1][i] & 255]
    for (int i = lane; i < 256; i += dfl::kT) s.crc_t[0][i] = dfl::crc_byte((uint32_t)i);
    __syncthreads();
    for (int k = 1; k < DFL_CRCS; ++k) {
        for (int i = lane; i < 256; i += dfl::kT) {
            const uint32_t v = s.crc_t[k - 1][i];
            s.crc_t[k][i] = (v >> 8) ^ s.crc_t[0][v & 255];
        }
        __syncthreads();
    }
#endif
    auto stamp = [&](int k) {
        if (st && lane == 0) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            t[k] += now - t0;
            t0 = now;
        }
    };
    // blocks claimed one at a time when a counter is given: in the pipeline
    // the grid's workgroups start as inflate workgroups leave their CUs, and
    // a fixed stride left the late starters' blocks as the launch's tail
    __shared__ int64_t s_claim;
    auto claim = [&](int64_t fixed) -> int64_t {
        if (!D.claim) return fixed;
        __syncthreads();                 // every lane has read the previous claim
        if (lane == 0) s_claim = (int64_t)atomicAdd(D.claim, 1ull);
        __syncthreads();
        return s_claim;
    };
    for (int64_t b = claim(blockIdx.x); b < nb; b = claim(b + gridDim.x)) {
        if (st && lane == 0) t0 = __builtin_amdgcn_s_memtime();
        const int64_t off = b * (int64_t)dfl::kMaxIn;
        const uint32_t n = (uint32_t)((total - off) < (int64_t)dfl::kMaxIn ? (total - off) : dfl::kMaxIn);
        uint32_t *slot = reinterpret_cast<uint32_t *>(D.slots + b * (int64_t)dfl::kSlot);
        // stage the block as dwords (block starts are dword-aligned; the
        // record stream's allocation is padded), zero bytes past n
        {
#if DFL_STAGE4
            // 16 bytes per lane per load, four loads in flight (block starts
            // are 16-byte aligned: 0xff00 = 16 * 4080)
            static_assert(dfl::kMaxIn % 16 == 0 && sizeof(s.in) % 16 == 0, "16-byte staging");
            const uint4 *src = reinterpret_cast<const uint4 *>(D.stream + off);
            uint4 *dst = reinterpret_cast<uint4 *>(s.in);
            const uint32_t nq = (n + 15) / 16, pq = (uint32_t)sizeof(s.in) / 16;
            auto mask = [&](uint32_t w, uint32_t byte0) -> uint32_t {     // bytes of w at or past n zeroed
                return byte0 + 4 <= n ? w : byte0 >= n ? 0u : w & ((1u << (8 * (n - byte0))) - 1);
            };
            for (uint32_t i0 = lane; i0 < pq; i0 += 4 * dfl::kT) {
                uint4 v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t i = i0 + (uint32_t)k * dfl::kT;
                    v[k] = (i < nq) ? src[i] : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t i = i0 + (uint32_t)k * dfl::kT;
                    if (i >= pq) continue;
                    uint4 w = v[k];
                    if (16 * i + 16 > n) {
                        w.x = mask(w.x, 16 * i);
                        w.y = mask(w.y, 16 * i + 4);
                        w.z = mask(w.z, 16 * i + 8);
                        w.w = mask(w.w, 16 * i + 12);
                    }
                    dst[i] = w;
                }
            }
#else
            const uint32_t *src = reinterpret_cast<const uint32_t *>(D.stream + off);
            uint32_t *dst = reinterpret_cast<uint32_t *>(s.in);
            const uint32_t nw = (n + 3) / 4, pw = (uint32_t)sizeof(s.in) / 4;
            for (uint32_t i = lane; i < pw; i += dfl::kT) {
                uint32_t v = 0;
                if (i < nw) {
                    v = src[i];
                    const uint32_t rem = n - 4 * i;
                    if (rem < 4) v &= (1u << (8 * rem)) - 1;
                }
                dst[i] = v;
            }
#endif
        }
        dfl::p0_clear(s, lane);
        __syncthreads();
        stamp(0);
        dfl::p1_hash(s, n, lane);
        __syncthreads();
        stamp(1);
        dfl::p2_count(s, n, lane, tok);
        __syncthreads();
        stamp(2);
        dfl::p3a_keys(s, lane);
        __syncthreads();
        dfl::p3b_rank(s, lane);
        __syncthreads();
        stamp(3);
        dfl::p3c_trees(s, lane);
#if DFL_CRC_LATE
        // waves 2 and 3 are idle while lanes 0 and 64 build the two codes:
        // the sub-block CRCs (two per lane) go there
        static_assert(dfl::kT == 256, "DFL_CRC_LATE assumes four waves");
        if (lane >= 128) {
            s.lane_crc[lane - 128] = dfl::sub_crc(s, n, lane - 128);
            s.lane_crc[lane] = dfl::sub_crc(s, n, lane);
        }
#endif
        __syncthreads();
        stamp(4);
        dfl::p3c_assign(s, lane);
        __syncthreads();
        stamp(10);
        if (lane < kW) p3c_header_wave(s, lane);
#if DFL_CODES_EARLY
        else dfl::p3d_codes_litdist(s, lane - kW, dfl::kT - kW);   // waves 1-3, idle during the header
#endif
        __syncthreads();
        stamp(11);
#if DFL_CODES_EARLY
        if (lane < 19) s.cl_code[lane] = dfl::code_of(s.cl_len, lane, s.next_code[2]);
#else
        dfl::p3d_codes(s, lane);
#endif
        __syncthreads();
        stamp(5);
        dfl::p4_bits(s, n, lane, tok);
        __syncthreads();
        stamp(6);
        p4_scan_wg(s, n, lane, slot);
        __syncthreads();
        stamp(7);
#ifndef DFL_ABL_NOEMIT
        dfl::p5_emit(s, n, lane, tok, slot);
#endif
        __syncthreads();
        dfl::p6_copy(s, lane, slot);
        stamp(8);
        if (lane == 0) D.sizes[b] = dfl::p6_frame(s, n, slot);
        __syncthreads();
        stamp(9);
    }
    if (st && lane == 0)
        for (int k = 0; k < 12; ++k) atomicAdd(&D.stamps[k], (unsigned long long)t[k]);
}

// compressed blocks into one contiguous buffer (offsets from an exclusive scan)
__global__ __launch_bounds__(256) void k_compact(CompactArgs C) {
    const int64_t total = *C.stream_bytes;
    const int64_t nb = (total + dfl::kMaxIn - 1) / dfl::kMaxIn;
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t n = (uint32_t)C.sizes[b];
        const int64_t o = C.offs[b];
        const uint8_t *src = C.slots + b * (int64_t)dfl::kSlot;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) C.out[o + i] = src[i];
        if (b == nb - 1 && threadIdx.x == 0) {
            C.totals[0] = o + n;        // compressed bytes
            C.totals[1] = total;        // formatted bytes
            C.totals[2] = nb;           // blocks
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && nb == 0) {
        C.totals[0] = 0;
        C.totals[1] = 0;
        C.totals[2] = 0;
    }
}


// ---- exclusive prefix sums of int64 (record sizes -> record offsets, block
// sizes -> block offsets).  Tiles of 2,048 values per 256-lane workgroup: each
// lane sums its 8 consecutive values, the workgroup scans the lane sums (wave
// shuffles, then the four wave totals through LDS) and writes the tile's
// exclusive prefixes; tile totals go to `part`.  More than one tile: one
// workgroup scans the tile totals, and every tile after the first adds its
// prefix.  Plain launches, no inter-workgroup waiting.
constexpr int kScanT = 256, kScanPer = 8, kScanTile = kScanT * kScanPer;

__device__ __forceinline__ int64_t wg_excl_scan(int64_t v, int64_t &total, int64_t *wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int64_t before = 0;
    for (int k = 0; k < w; ++k) before += wsum[k];
    total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return before + x - v;
}

__global__ __launch_bounds__(kScanT) void k_scan_tiles(const int64_t *in, int64_t *out, int64_t *part, int n) {
    __shared__ int64_t wsum[4];
    const int64_t t0 = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    int64_t v[kScanPer], s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        v[k] = t0 + k < n ? in[t0 + k] : 0;
        s += v[k];
    }
    int64_t total;
    int64_t run = wg_excl_scan(s, total, wsum);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        if (t0 + k < n) out[t0 + k] = run;
        run += v[k];
    }
    if (part && threadIdx.x == 0) part[blockIdx.x] = total;
}

// one workgroup: exclusive scan of the tile totals in place
__global__ __launch_bounds__(kScanT) void k_scan_part(int64_t *part, int nt) {
    __shared__ int64_t wsum[4];
    int64_t carry = 0;
    for (int base = 0; base < nt; base += kScanT) {
        const int i = base + (int)threadIdx.x;
        const int64_t v = i < nt ? part[i] : 0;
        int64_t total;
        const int64_t e = wg_excl_scan(v, total, wsum);
        if (i < nt) part[i] = carry + e;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanT) void k_scan_add(int64_t *out, const int64_t *part, int n) {
    const int64_t add = part[blockIdx.x + 1];
    const int64_t t0 = (int64_t)(blockIdx.x + 1) * kScanTile;
    for (int k = (int)threadIdx.x; k < kScanTile; k += kScanT)
        if (t0 + k < n) out[t0 + k] += add;
}

size_t scan_tmp_bytes(int n) { return 8 * (size_t)((n + kScanTile - 1) / kScanTile + 1); }

hipError_t scan_excl_i64(const int64_t *in, int64_t *out, int n, int64_t *tmp, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int nt = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)nt), dim3(kScanT), 0, s, in, out, nt > 1 ? tmp : nullptr, n);
    if (nt > 1) {
        hipLaunchKernelGGL(k_scan_part, dim3(1), dim3(kScanT), 0, s, tmp, nt);
        hipLaunchKernelGGL(k_scan_add, dim3((unsigned)(nt - 1)), dim3(kScanT), 0, s, out, (const int64_t *)tmp, n);
    }
    return hipGetLastError();
}

}  // namespace dcrw
