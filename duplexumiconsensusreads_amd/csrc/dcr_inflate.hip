// dcr_inflate.hip — BGZF inflate on gfx950 (include/dcr_inflate.h): the
// input side of the whole-node pipeline.  The reference reads its BAM through
// pysam (DuplexUMIConsensusReads.py:1476, :1519); the native ingest
// (csrc/dcr_ingest.cpp) cuts the file into chunks of whole BGZF members and,
// with the hook set, hands each chunk's members to this kernel instead of
// inflating them on its host pool.
//
// k_inflate: one wavefront per member (a 64-thread workgroup, ~9.3 KB of LDS,
// about 17 per CU).  Huffman decoding is serial within a member, so the
// wave decodes it as one scalar stream (bit buffer, positions and tables'
// results are wave-uniform, held in SGPRs) and uses its 64 lanes for
// everything around that stream:
//   - decode tables built lane-parallel in LDS (counts by ballot, canonical
//     first codes by a lane scan, symbols sorted by (length, symbol), every
//     10-bit root entry resolved by its own lane); literal/length root
//     entries hold two literals when both codes fit the 10 bits;
//   - the input read as 256-byte windows, one dword per lane (loaded when the
//     bit buffer reaches them); the bit buffer refilled by v_readlane;
//   - literals collected one per lane and written 64 at a time, matches
//     copied by all lanes (a distance below 64 by its period);
//   - the last kRing bytes of output (4 KiB) kept in an LDS ring, the source
//     of every match that reaches no further (older ones read HBM); the ring
//     is written to HBM in pieces of half its size with dword stores, and the
//     CRC32 of each piece is formed on the way (a stripe per lane, raw CRCs
//     shifted by x^(8n) mod P and xor-reduced;
//     zlib's crc32_combine algebra, dcr_deflate.h multmodp);
//   - ISIZE and CRC32 checked against the member trailer on the device.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dcr_inflate.h"
#include "dcr_deflate.h"
#include "dcr_internal.h"
#include "dcr_span_stream.h"

#ifndef DINF_STAMP
#define DINF_STAMP 0      // diagnostic builds: per-phase s_memtime cycles and token counts in Args::dbg
#endif

namespace dinf {

// diagnostic phase clock (DINF_STAMP builds): dbg[16 mi + k]
struct IStamp {
    uint64_t t = 0;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void start() {
        if (DINF_STAMP) t = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void lap(int k) {
        if (DINF_STAMP) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            acc[k] += (uint32_t)(now - t);
            t = now;
        }
    }
    __device__ __forceinline__ void count(int k, uint32_t v = 1) {
        if (DINF_STAMP) cnt[k] += v;
    }
};

// LDS per wave sets the waves per CU, and a member's decode is latency-bound:
// a 4 KiB ring and a 9-bit root table (9.3 KB, 17 waves per CU instead of 10
// at 8 KiB / 10 bits) inflate a 4,096-member span in 5.65 ms instead of 9.09
// (35.2 -> 47.5 GB/s over all members in one launch; profiles/r04e)
#ifndef DINF_WG_PER_CU
#define DINF_WG_PER_CU 16 // k_inflate launch grid cap per CU (0: one workgroup per member)
#endif
#ifndef DINF_CU_SHARE
#define DINF_CU_SHARE 0   // diagnostic builds: the streaming inflate on DINF_CU_SHARE of every 8 CUs (0: all)
#endif
#ifndef DINF_RING
#define DINF_RING 4096    // LDS output history per member (bytes)
#endif
#ifndef DINF_LB
#define DINF_LB 9         // literal/length root table bits
#endif
constexpr int kW = 64;
constexpr int kLB = DINF_LB;               // literal/length root table bits
constexpr int kDB = 8;                     // distance root table bits
constexpr int kCB = 7;                     // code-length code (all codes <= 7 bits)
constexpr uint32_t kRing = DINF_RING;      // output history in LDS
constexpr uint32_t kRM = kRing - 1;
constexpr uint32_t kPiece = kRing / 2;     // ring -> HBM write unit
constexpr uint32_t kStripe = kPiece / kW;  // CRC stripe per lane in a piece
static_assert((kRing & (kRing - 1)) == 0 && kRing >= 2048, "ring: a power of two");
// bytes not yet in HBM stay in the ring: [gpos, opos) spans < kPiece + 322
// (a match of <= 258 and <= 63 literals between keep_room calls) and a step
// writes <= 320 bytes past opos
static_assert(kPiece + 322 + 320 <= kRing, "the ring holds the unwritten bytes");
constexpr int kPad = 1024;                 // readable bytes past the last member (window prefetch)

// root entry: bits 0-4 bits to consume (0: a longer code, canonical slow path),
// 5-7 kind, 8-15 literal / extra bits, 16-31 second literal / base
enum : uint32_t { K_LIT = 0, K_PAIR = 1, K_LEN = 2, K_EOB = 3, K_DIST = 4, K_BAD = 7 };

enum : uint8_t { ST_OK = 0, ST_STREAM = 1, ST_SIZE = 2, ST_CRC = 3, ST_GUARD = 4 };
// iterations of the block / header / symbol loops per member (a member has
// at most 65,536 output bytes and 65,536 input bytes): every wave ends
constexpr uint32_t kGuard = 1u << 21;

struct alignas(16) WaveLds {
    uint32_t lit[1 << kLB];               // literal/length root table
    uint32_t dist[1 << kDB];              // distance root table (the code-length table while a header is read)
    uint8_t ring[kRing];                  // output history
    uint32_t crc_tab[256];
    uint16_t lsym[288], dsym[32];         // symbols sorted by (code length, symbol)
    uint16_t lcnt[16], dcnt[16];          // codes per length
    uint8_t lens[320];                    // HLIT + HDIST code lengths
    uint8_t cl_lens[20];
};

struct Args {
    const uint8_t *in;
    uint8_t *out;
    const dcr_bgzf_member *m;
    uint8_t *status;
    uint32_t *dbg;                        // [4 n]: failing loop, bits used, output bytes, iterations (may be null)
    int32_t n;
    uint32_t x8n_piece;                   // x^(8 kPiece) mod P
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kW - 1)); }
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// literal/length symbol -> root entry payload (without the bit count)
__device__ __forceinline__ uint32_t lit_entry(uint32_t sym) {
    if (sym < 256) return (K_LIT << 5) | (sym << 8);
    if (sym == 256) return K_EOB << 5;
    if (sym < 286) return (K_LEN << 5) | ((uint32_t)dfl::kLenExtra[sym - 257] << 8) | ((uint32_t)dfl::kLenBase[sym - 257] << 16);
    return K_BAD << 5;
}
__device__ __forceinline__ uint32_t dist_entry(uint32_t sym) {
    if (sym < 30) return (K_DIST << 5) | ((uint32_t)dfl::kDistExtra[sym] << 8) | ((uint32_t)dfl::kDistBase[sym] << 16);
    return K_BAD << 5;
}

// Canonical decode tables from code lengths lens[0, n) (n <= 288), built by
// the whole wave.  kind: 0 literal/length, 1 distance, 2 code-length code.
// Returns false for an over-subscribed code.  Entries of codes longer than
// TB bits are 0; an incomplete code leaves K_BAD entries.
template <int TB, int KIND>
__device__ __noinline__ bool build_table(const uint8_t *lens, int n, uint32_t *tab, uint16_t *cnt_out, uint16_t *sym_out) {
    const int lane = lane_id();
    const uint64_t lt = (1ull << lane) - 1;
    // codes per length: lane L holds cnt[L]
    uint32_t mycnt = 0;
    for (int c0 = 0; c0 < n; c0 += kW) {
        const int i = c0 + lane;
        const uint32_t l = i < n ? lens[i] : 0;
#pragma unroll
        for (int L = 1; L <= 15; ++L) {
            const uint32_t k = (uint32_t)__popcll(__ballot(l == (uint32_t)L));
            if (lane == L) mycnt += k;
        }
    }
    if (lane == 0) mycnt = 0;
    // Kraft sum: sum cnt[L] 2^(15-L) <= 2^15
    uint32_t kr = lane >= 1 && lane <= 15 ? mycnt << (15 - lane) : 0;
    for (int d = 32; d >= 1; d >>= 1) kr += __shfl_xor(kr, d, kW);
    if (uni(kr) > 32768u) return false;
    // offsets (symbols of shorter codes) and canonical first codes
    uint32_t offs = 0, first = 0;
#pragma unroll
    for (int l = 1; l <= 15; ++l) {
        const uint32_t cl = lane_read(mycnt, l);
        if (l < lane && lane < 16) {
            offs += cl;
            first += cl << (lane - l);
        }
    }
    if (lane < 16) cnt_out[lane] = (uint16_t)mycnt;
    // symbols sorted by (length, symbol)
    uint32_t run = offs;          // lane L: next slot of length L
    for (int c0 = 0; c0 < n; c0 += kW) {
        const int i = c0 + lane;
        const uint32_t l = i < n ? lens[i] : 0;
#pragma unroll
        for (int L = 1; L <= 15; ++L) {
            const uint64_t m = __ballot(l == (uint32_t)L);
            const uint32_t base = lane_read(run, L);
            if (l == (uint32_t)L) sym_out[base + __popcll(m & lt)] = (uint16_t)i;
            if (lane == L) run += (uint32_t)__popcll(m);
        }
    }
    // root entries, one lane per entry: the MSB-first TB-bit code of index e
    // is bitrev(e); it lies in length L's range [first_L, first_L + cnt_L)
    uint32_t fL[TB + 1], cL[TB + 1], oL[TB + 1];
#pragma unroll
    for (int L = 1; L <= TB; ++L) {
        fL[L] = lane_read(first, L);
        cL[L] = lane_read(mycnt, L);
        oL[L] = lane_read(offs, L);
    }
    bool any_long = false;
    {
        uint32_t longer = 0;
        for (int l = TB + 1; l <= 15; ++l) longer += lane_read(mycnt, l);
        any_long = longer != 0;
    }
    for (int e = lane; e < (1 << TB); e += kW) {
        const uint32_t c = __builtin_bitreverse32((uint32_t)e) >> (32 - TB);
        uint32_t ent = any_long ? 0u : (K_BAD << 5);
#pragma unroll
        for (int L = 1; L <= TB; ++L) {
            const uint32_t v = (c >> (TB - L)) - fL[L];
            if (v < cL[L]) {
                const uint32_t sym = sym_out[oL[L] + v];
                const uint32_t pay = KIND == 0 ? lit_entry(sym) : KIND == 1 ? dist_entry(sym) : (sym << 8);
                ent = pay | (uint32_t)L;
            }
        }
        tab[e] = ent;
    }
    if (KIND == 0) {
        // pairs: a literal of n1 < TB bits followed by a literal whose code
        // fits the remaining TB - n1 bits of the index
        uint32_t pr[(1 << TB) / kW];
#pragma unroll
        for (int k = 0; k < (1 << TB) / kW; ++k) {
            const int e = lane + k * kW;
            const uint32_t e1 = tab[e];
            const uint32_t n1 = e1 & 31;
            pr[k] = e1;
            if (n1 != 0 && ((e1 >> 5) & 7) == K_LIT && n1 < TB) {
                const uint32_t e2 = tab[e >> n1];
                const uint32_t n2 = e2 & 31;
                if (n2 != 0 && ((e2 >> 5) & 7) == K_LIT && n1 + n2 <= TB)
                    pr[k] = (n1 + n2) | (K_PAIR << 5) | (e1 & 0xff00u) | (((e2 >> 8) & 0xffu) << 16);
            }
        }
#pragma unroll
        for (int k = 0; k < (1 << TB) / kW; ++k) tab[lane + k * kW] = pr[k];
    }
    return true;
}

// the wave's decoder state (all wave-uniform)
struct Dec {
    __amdgpu_buffer_rsrc_t rs; // member input from a dword-aligned base; loads past its end read 0
    uint32_t win;             // this lane's dword of the current 256-byte window
    uint32_t wbase;           // dword index of the current window
    uint32_t wi;              // next dword to enter the bit buffer
    uint64_t bb;
    uint32_t nb;
    uint32_t skip;            // bits of the first dword before the stream start
    uint32_t off;             // bits of the member consumed before the current base
    const uint8_t *base;      // the dword-aligned base
};

// start reading at p (the member's input ends at end; the buffer is readable
// kPad bytes past every member)
__device__ __forceinline__ void dec_start(Dec &d, const uint8_t *p, const uint8_t *end, uint32_t off_bits) {
    const uintptr_t a = (uintptr_t)p;
    d.base = (const uint8_t *)(a & ~(uintptr_t)3);
    d.skip = (uint32_t)(a & 3) * 8;
    d.off = off_bits;
    const uint32_t extent = (uint32_t)(end - d.base) + 512;
    d.rs = __builtin_amdgcn_make_buffer_rsrc((void *)d.base, (short)0, (int)extent, 0x00020000);
    const int lane = lane_id();
    d.win = __builtin_amdgcn_raw_buffer_load_b32(d.rs, 4 * lane, 0, 0);
    d.wbase = 0;
    d.wi = 0;
    d.bb = 0;
    d.nb = 0;
}
__device__ __forceinline__ void refill(Dec &d) {
    while (d.nb <= 32) {
        const uint32_t w = lane_read(d.win, d.wi - d.wbase);
        d.bb |= (uint64_t)w << d.nb;
        d.nb += 32;
        ++d.wi;
        if (d.wi - d.wbase == kW) {
            // the next window on demand (~300 tokens per window): a
            // prefetched register would be copied at every loop back edge
            // while in flight, i.e. a vmcnt(0) wait per token
            d.wbase += kW;
            d.win = __builtin_amdgcn_raw_buffer_load_b32(d.rs, 4 * (d.wbase + lane_id()), 0, 0);
        }
    }
}
// drop the bits in front of the stream start (after dec_start)
__device__ __forceinline__ void dec_prime(Dec &d) {
    refill(d);
    d.bb >>= d.skip;
    d.nb -= d.skip;
}
__device__ __forceinline__ uint32_t getbits(Dec &d, uint32_t k) {   // k <= 24
    if (d.nb < k) refill(d);
    const uint32_t v = (uint32_t)d.bb & ((1u << k) - 1);
    d.bb >>= k;
    d.nb -= k;
    return v;
}
// bits of the member consumed so far
__device__ __forceinline__ uint32_t bits_used(const Dec &d) { return d.off + d.wi * 32 - d.nb - d.skip; }

// canonical slow path for codes longer than the root (puff's decode)
__device__ __forceinline__ int slow_decode(Dec &d, const uint16_t *cnt, const uint16_t *sym, uint32_t &nbits) {
    uint32_t code = 0, first = 0, index = 0;
    for (uint32_t L = 1; L <= 15; ++L) {
        code |= (uint32_t)(d.bb >> (L - 1)) & 1u;
        const uint32_t c = uni(cnt[L]);      // LDS reads stay wave-uniform (else the whole decoder turns divergent)
        if (code - first < c) {
            nbits = L;
            return (int)uni(sym[index + code - first]);
        }
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

struct Out {
    uint8_t *g;               // member output in HBM
    uint32_t isize;
    uint32_t opos;            // bytes produced (ring holds [opos - kRing, opos))
    uint32_t gpos;            // bytes written to HBM
    uint32_t crc;             // raw CRC (init 0) of [0, gpos)
    uint32_t lbuf;            // pending literal of this lane
    uint32_t nlit;
};

__device__ __forceinline__ uint32_t crc_stripe(const WaveLds &s, uint32_t from, uint32_t n) {
    uint32_t c = 0;
    for (uint32_t i = 0; i < n; ++i) c = s.crc_tab[(c ^ s.ring[(from + i) & kRM]) & 0xff] ^ (c >> 8);
    return c;
}

extern __shared__ __align__(16) unsigned char smem[];

// write ring bytes [g0, g0 + m) to HBM (m <= kPiece) and fold them into the
// raw CRC; one out-of-line copy (called every kPiece bytes) keeps the decode loop small
__device__ __noinline__ uint32_t write_piece(uint8_t *g, uint32_t g0, uint32_t m, uint32_t crc, uint32_t lane_shift,
                                             uint32_t x8n_piece) {
    const WaveLds &s = *reinterpret_cast<const WaveLds *>(smem);
    const int lane = lane_id();
    uint8_t *dst = g + g0;
    if (((uintptr_t)dst & 3) == 0 && (g0 & 3) == 0) {
        const uint32_t *rw = reinterpret_cast<const uint32_t *>(s.ring);
        uint32_t *dw = reinterpret_cast<uint32_t *>(dst);
        const uint32_t nd = m >> 2;
        for (uint32_t k = lane; k < nd; k += kW) dw[k] = rw[((g0 >> 2) + k) & (kRM >> 2)];
        for (uint32_t k = (nd << 2) + lane; k < m; k += kW) dst[k] = s.ring[(g0 + k) & kRM];
    } else {
        for (uint32_t k = lane; k < m; k += kW) dst[k] = s.ring[(g0 + k) & kRM];
    }
    const uint32_t lo = min(m, (uint32_t)lane * kStripe), hi = min(m, (uint32_t)lane * kStripe + kStripe);
    uint32_t c = hi > lo ? crc_stripe(s, g0 + lo, hi - lo) : 0;
    if (hi > lo) c = dfl::multmodp(m == kPiece ? lane_shift : dfl::x8nmodp(m - hi), c);
    for (int d = 32; d >= 1; d >>= 1) c ^= __shfl_xor(c, d, kW);
    const uint32_t shift = m == kPiece ? x8n_piece : dfl::x8nmodp(m);
    return uni(dfl::multmodp(shift, crc) ^ c);
}

// Ring writes past the bytes produced are harmless: positions in
// [opos, opos + 64) are rewritten before anything reads them, and their ring
// slots alias bytes older than opos + 64 - kRing, which no match reads
// (distances from the ring stay <= kRingDist) and which are already in HBM
// (gpos > opos - kPiece - 322).  So literal flushes and match copies store all
// 64 lanes, with no exec masking.
constexpr uint32_t kRingDist = kRing - kW;

__device__ __forceinline__ void flush_lits(WaveLds &s, Out &o) {
    s.ring[(o.opos + lane_id()) & kRM] = (uint8_t)o.lbuf;
    o.opos += o.nlit;
    o.nlit = 0;
}
__device__ __forceinline__ void keep_room(Out &o, const Args &a, uint32_t lane_shift) {
    while (o.gpos + kPiece <= o.opos) {
        o.crc = uni(write_piece(o.g, o.gpos, kPiece, o.crc, lane_shift, a.x8n_piece));   // call results count as divergent
        o.gpos += kPiece;
    }
}

// one member, decoded by the calling wave
__device__ __forceinline__ void inflate_one(const Args &a, WaveLds &s, const int mi, const uint32_t lsh) {
    const int lane = lane_id();
    const dcr_bgzf_member M = a.m[mi];

    Out o;
    o.g = a.out + M.out_off;
    o.isize = M.isize;
    o.opos = o.gpos = o.crc = 0;
    o.lbuf = 0;
    o.nlit = 0;
    uint8_t st = ST_OK;
    const uint8_t *mstart = a.in + M.in_off, *mend = mstart + M.in_len;
    Dec d;
    dec_start(d, mstart, mend, 0);
    dec_prime(d);

    bool last = false;
    uint32_t guard = 0, where = 0;
    IStamp sp;
    sp.start();
    while (!last && st == ST_OK) {
        if (++guard > kGuard) { st = ST_GUARD; where = 1; break; }
        if (bits_used(d) > (M.in_len + 4) * 8) { st = ST_STREAM; break; }
        last = getbits(d, 1) != 0;
        const uint32_t type = getbits(d, 2);
        if (type == 0) {                                  // stored
            const uint32_t k = d.nb & 7;
            d.bb >>= k;
            d.nb -= k;
            const uint32_t len = getbits(d, 16), nlen = getbits(d, 16);
            if ((len ^ 0xffffu) != nlen) { st = ST_STREAM; break; }
            const uint32_t bytepos = (d.wi * 32 - d.nb) >> 3;     // next unread byte, from d.base
            const uint8_t *src = d.base + bytepos;
            if (src + len > mend || o.opos + len > o.isize) { st = ST_STREAM; break; }
            for (uint32_t c0 = 0; c0 < len; c0 += kW) {
                const uint32_t m = min((uint32_t)kW, len - c0);
                if (lane < (int)m) s.ring[(o.opos + lane) & kRM] = src[c0 + lane];
                o.opos += m;
                keep_room(o, a, lsh);
            }
            // the bit reader restarts after the stored bytes
            dec_start(d, src + len, mend, (uint32_t)(src + len - mstart) * 8);
            dec_prime(d);
            continue;
        }
        if (type == 3) { st = ST_STREAM; break; }
        if (type == 1) {                                  // fixed codes
            for (int i = lane; i < 288; i += kW) s.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
            build_table<kLB, 0>(s.lens, 288, s.lit, s.lcnt, s.lsym);
            for (int i = lane; i < 32; i += kW) s.lens[i] = 5;
            build_table<kDB, 1>(s.lens, 32, s.dist, s.dcnt, s.dsym);
        } else {                                          // dynamic codes
            const uint32_t hlit = getbits(d, 5) + 257, hdist = getbits(d, 5) + 1, hclen = getbits(d, 4) + 4;
            if (hlit > 286 || hdist > 30) { st = ST_STREAM; break; }
            if (lane < 20) s.cl_lens[lane] = 0;
            for (uint32_t i = 0; i < hclen; ++i) {
                const uint32_t v = getbits(d, 3);
                if (lane == 0) s.cl_lens[dfl::kClOrder[i]] = (uint8_t)v;
            }
            // the code-length table lives in dist[] while the lengths are read
            if (!uni(build_table<kCB, 2>(s.cl_lens, 19, s.dist, s.dcnt, s.dsym))) { st = ST_STREAM; break; }
            const uint32_t total = hlit + hdist;
            uint32_t i = 0;
            while (i < total) {
                if (++guard > kGuard) { st = ST_GUARD; where = 2; break; }
                if (d.nb < 16) refill(d);
                const uint32_t e = uni(s.dist[(uint32_t)d.bb & ((1u << kCB) - 1)]);
                const uint32_t n = e & 31;
                if (n == 0 || ((e >> 5) & 7) == K_BAD) { st = ST_STREAM; break; }
                d.bb >>= n;
                d.nb -= n;
                const uint32_t sym = e >> 8;
                uint32_t rep = 1, val = sym;
                if (sym == 16) {
                    if (i == 0) { st = ST_STREAM; break; }
                    val = uni(s.lens[i - 1]);
                    rep = 3 + getbits(d, 2);
                } else if (sym == 17) {
                    val = 0;
                    rep = 3 + getbits(d, 3);
                } else if (sym == 18) {
                    val = 0;
                    rep = 11 + getbits(d, 7);
                }
                if (i + rep > total) { st = ST_STREAM; break; }
                for (uint32_t r = lane; r < rep; r += kW) s.lens[i + r] = (uint8_t)val;
                i += rep;
            }
            if (st != ST_OK) break;
            if (uni(s.lens[256]) == 0) { st = ST_STREAM; break; }
            if (!uni(build_table<kLB, 0>(s.lens, (int)hlit, s.lit, s.lcnt, s.lsym))) { st = ST_STREAM; break; }
            if (!uni(build_table<kDB, 1>(s.lens + hlit, (int)hdist, s.dist, s.dcnt, s.dsym))) { st = ST_STREAM; break; }
        }
        sp.lap(0);                                        // block header, tables
        // Huffman-coded data
        // (bounded without a guard: every symbol emits output, checked
        // against ISIZE at least every 63 literals and at every match)
        for (;;) {
            if (d.nb < 32) refill(d);
            uint32_t e = uni(s.lit[(uint32_t)d.bb & ((1u << kLB) - 1)]);
            uint32_t n = e & 31;
            if (n == 0) {
                const int sym = slow_decode(d, s.lcnt, s.lsym, n);
                if (sym < 0) { st = ST_STREAM; break; }
                e = lit_entry((uint32_t)sym) | n;
            }
            d.bb >>= n;
            d.nb -= n;
            const uint32_t kind = (e >> 5) & 7;
            if (kind == K_LIT || kind == K_PAIR) {
                sp.count(kind == K_PAIR ? 1 : 0);
                o.lbuf = lane == (int)o.nlit ? (e >> 8) & 0xff : o.lbuf;
                ++o.nlit;
                if (kind == K_PAIR) {
                    o.lbuf = lane == (int)o.nlit ? (e >> 16) & 0xff : o.lbuf;
                    ++o.nlit;
                }
                if (o.nlit >= kW - 1) {
                    if (o.opos + o.nlit > o.isize) { st = ST_SIZE; break; }
                    sp.lap(1);
                    flush_lits(s, o);
                    keep_room(o, a, lsh);
                    sp.lap(4);
                }
                continue;
            }
            if (kind == K_EOB) break;
            if (kind != K_LEN) { st = ST_STREAM; break; }
            const uint32_t ex = (e >> 8) & 7;
            const uint32_t len = (e >> 16) + ((uint32_t)d.bb & ((1u << ex) - 1));
            d.bb >>= ex;
            d.nb -= ex;
            if (d.nb < 32) refill(d);
            uint32_t de = uni(s.dist[(uint32_t)d.bb & ((1u << kDB) - 1)]);
            uint32_t dn = de & 31;
            if (dn == 0) {
                const int sym = slow_decode(d, s.dcnt, s.dsym, dn);
                if (sym < 0) { st = ST_STREAM; break; }
                de = dist_entry((uint32_t)sym) | dn;
            }
            if (((de >> 5) & 7) != K_DIST) { st = ST_STREAM; break; }
            d.bb >>= dn;
            d.nb -= dn;
            const uint32_t dex = (de >> 8) & 15;
            const uint32_t dist = (de >> 16) + ((uint32_t)d.bb & ((1u << dex) - 1));
            d.bb >>= dex;
            d.nb -= dex;
            if (o.opos + o.nlit + len > o.isize) { st = ST_SIZE; break; }
            sp.lap(2);
            sp.count(2);
            sp.count(3, len);
            flush_lits(s, o);
            if (dist > o.opos) { st = ST_STREAM; break; }
            if (dist >= kW && dist <= kRingDist) {
                // no overlap inside a 64-byte step: sources precede the step
                for (uint32_t c0 = 0; c0 < len; c0 += kW) {
                    const uint32_t i = c0 + lane;
                    const uint8_t v = s.ring[(o.opos - dist + i) & kRM];
                    s.ring[(o.opos + i) & kRM] = v;
                }
            } else if (dist < kW) {
                // a period below the wave: byte i repeats byte i mod dist
                // lane mod dist and the largest multiple of dist <= 64 by a
                // float reciprocal (exact here: (x + 0.5) / dist is >= 0.5 / 63
                // away from an integer), not an integer division sequence
                const float rd = __builtin_amdgcn_rcpf((float)dist);
                const uint32_t rep = (uint32_t)lane - dist * (uint32_t)(((float)lane + 0.5f) * rd);
                const uint32_t step = dist * uni((uint32_t)(((float)kW + 0.5f) * rd));   // a multiple of dist
                const uint8_t v = s.ring[(o.opos - dist + rep) & kRM];
                for (uint32_t c0 = 0; c0 < len; c0 += step) s.ring[(o.opos + c0 + lane) & kRM] = v;
            } else {
                // older than the ring: already in HBM (written by this wave)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                for (uint32_t c0 = 0; c0 < len; c0 += kW) {
                    const uint32_t i = c0 + lane;
                    if (i < len) s.ring[(o.opos + i) & kRM] = o.g[o.opos - dist + i];
                }
            }
            o.opos += len;
            sp.lap(3);
            keep_room(o, a, lsh);
            sp.lap(4);
        }
        sp.lap(1);
        if (st != ST_OK) break;
        if (o.opos + o.nlit > o.isize) { st = ST_SIZE; break; }
        flush_lits(s, o);
        keep_room(o, a, lsh);
    }
    if (st == ST_OK && (bits_used(d) + 7) / 8 > M.in_len) st = ST_STREAM;
    if (st == ST_OK && o.opos != o.isize) st = ST_SIZE;
    if (st == ST_OK) {
        while (o.gpos < o.opos) {
            const uint32_t m = min(kPiece, o.opos - o.gpos);
            o.crc = uni(write_piece(o.g, o.gpos, m, o.crc, lsh, a.x8n_piece));
            o.gpos += m;
        }
        const uint32_t crc = ~(dfl::multmodp(dfl::x8nmodp(o.isize), 0xffffffffu) ^ o.crc);
        if (o.isize == 0) {
            if (M.crc != 0) st = ST_CRC;
        } else if (crc != M.crc) {
            st = ST_CRC;
        }
    }
    sp.lap(5);
    if (DINF_STAMP && lane == 0 && a.dbg) {
        for (int k = 0; k < 6; ++k) a.dbg[16 * mi + k] = sp.acc[k];
        for (int k = 0; k < 4; ++k) a.dbg[16 * mi + 8 + k] = sp.cnt[k];
        a.dbg[16 * mi + 12] = guard;
        a.dbg[16 * mi + 13] = o.opos;
    }
    if (lane == 0) {
        a.status[mi] = st;
        if (a.dbg && !DINF_STAMP) {
            a.dbg[4 * mi] = st | where << 8;
            a.dbg[4 * mi + 1] = bits_used(d);
            a.dbg[4 * mi + 2] = o.opos;
            a.dbg[4 * mi + 3] = guard;
        }
    }
}

// Wave w takes members w, w + gridDim.x, ...  The grid is capped at
// DINF_WG_PER_CU workgroups per CU.  The member decode is latency-bound: 4 or
// 2 waves per CU starved the inflate (117 -> 266 / 390 ms of kernel time per
// pass) and the whole node lost (357 -> 268 / 204 M consensus bases/s,
// profiles/r05r); 12 per CU beat the uncapped grid in round 5 (profiles/r05ab:
// 429 vs 419 M at level 1, 470 vs 422 M at level 6).  With round 6's pass
// bound by the batch stream, 16 per CU (every workgroup whose LDS fits)
// decodes a pass in 92 instead of 120 ms of kernel time and the whole node
// gains (ten interleaved pairs, profiles/r06wg: 400.8 vs 391.8 M at level 1,
// 449.6 vs 423.6 M at level 6); 6, 8 and 10 per CU were slower or level.
__global__ __launch_bounds__(64) void k_inflate(Args a) {
    WaveLds &s = *reinterpret_cast<WaveLds *>(smem);
    const int lane = lane_id();
    for (int i = lane; i < 256; i += kW) s.crc_tab[i] = dfl::crc_byte((uint32_t)i);
    // x^(8 (kPiece - kStripe (l + 1))) mod P: the shift of lane l's stripe to a piece's end
    const uint32_t lsh = dfl::x8nmodp(kPiece - kStripe * (uint32_t)(lane + 1));
    for (int mi = (int)blockIdx.x; mi < a.n; mi += (int)gridDim.x) inflate_one(a, s, mi, lsh);
}

}  // namespace dinf

// ---- host side ---------------------------------------------------------------
struct InflSlots {
    static constexpr int kSlots = 4;
    uint8_t *d_in[kSlots] = {}, *d_out[kSlots] = {}, *d_st[kSlots] = {};
    dcr_bgzf_member *d_m[kSlots] = {};
    size_t cap_in[kSlots] = {}, cap_out[kSlots] = {}, cap_m[kSlots] = {}, cap_dst[kSlots] = {};
    uint8_t *h_stage[kSlots] = {}, *h_st[kSlots] = {};
    size_t cap_stage[kSlots] = {}, cap_hst[kSlots] = {};
    hipStream_t s_k = nullptr, s_out = nullptr;
    bool busy = false;
    void release() {
        for (int i = 0; i < kSlots; ++i) {
            if (d_in[i]) (void)hipFree(d_in[i]);
            if (d_out[i]) (void)hipFree(d_out[i]);
            if (d_st[i]) (void)hipFree(d_st[i]);
            if (d_m[i]) (void)hipFree(d_m[i]);
            if (h_stage[i]) (void)hipHostFree(h_stage[i]);
            if (h_st[i]) (void)hipHostFree(h_st[i]);
        }
        if (s_k) (void)hipStreamDestroy(s_k);
        if (s_out) (void)hipStreamDestroy(s_out);
    }
};

struct dcr_inflater {
    int device = 0;
    int grid_cap = 1 << 30;           // k_inflate workgroups per launch (resident waves)
    int n_cu = 1;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    uint8_t *d_in = nullptr, *d_out = nullptr, *d_st = nullptr;
    dcr_bgzf_member *d_m = nullptr;
    uint32_t *d_dbg = nullptr;
    size_t cap_in = 0, cap_out = 0, cap_m = 0, cap_dbg = 0;
    size_t cap_st = 0;
    dinf::Args base{};
    float last_ms = 0;
    int32_t last_n = 0;
    double tot[4] = {0, 0, 0, 0};     // kernel ms, runs, members, output bytes
    double stamp[16] = {};            // DINF_STAMP builds: summed dbg words
    struct InflSlots *slots = nullptr;  // the streaming buffers (kept across streams)
    std::mutex mu;
    std::unordered_multimap<size_t, void *> free_host;   // page-locked buffers kept for later ingests
    std::unordered_map<void *, size_t> live_host;
};

namespace {
template <class T>
hipError_t grow(T *&p, size_t &cap, size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc((void **)&p, n * sizeof(T));
    if (e == hipSuccess) cap = n;
    return e;
}
int hip_fail(hipError_t e, const char *what) {
    return dcr::set_error(DCR_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

extern "C" {

dcr_inflater *dcr_inflater_create(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        dcr::set_error(DCR_ENODEV, "dcr_inflater_create: no such device");
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        dcr::set_error(DCR_ENODEV, "dcr_inflater_create: not a gfx950 device");
        return nullptr;
    }
    auto *h = new dcr_inflater;
    h->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
        hipFuncSetAttribute((const void *)dinf::k_inflate, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(dinf::WaveLds)) != hipSuccess) {
        dcr::set_error(DCR_EHIP, "dcr_inflater_create: HIP setup failed");
        dcr_inflater_destroy(h);
        return nullptr;
    }
    h->base.x8n_piece = dfl::x8nmodp(dinf::kPiece);
    h->n_cu = std::max(1, prop.multiProcessorCount);
    if (DINF_WG_PER_CU > 0) h->grid_cap = DINF_WG_PER_CU * h->n_cu * (DINF_CU_SHARE > 0 ? DINF_CU_SHARE : 8) / 8;
    return h;
}

void dcr_inflater_destroy(dcr_inflater *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->d_in) (void)hipFree(h->d_in);
    if (h->d_out) (void)hipFree(h->d_out);
    if (h->d_st) (void)hipFree(h->d_st);
    if (h->d_m) (void)hipFree(h->d_m);
    if (h->d_dbg) (void)hipFree(h->d_dbg);
    for (auto &kv : h->free_host) (void)hipHostFree(kv.second);
    for (auto &kv : h->live_host) (void)hipHostFree(kv.first);
    if (h->slots) {
        h->slots->release();
        delete h->slots;
    }
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int dcr_inflater_run(dcr_inflater *h, const uint8_t *in, int64_t in_bytes, const dcr_bgzf_member *m, int32_t n,
                     uint8_t *out, int64_t out_bytes) {
    if (!h || n < 0 || in_bytes < 0 || out_bytes < 0 || (n && (!in || !m || !out)))
        return -dcr::set_error(DCR_EARG, "dcr_inflater_run: bad arguments");
    if (n == 0) return 0;
    for (int32_t i = 0; i < n; ++i)
        if (m[i].in_off < 0 || m[i].in_off + (int64_t)m[i].in_len > in_bytes || m[i].isize > 65536 ||
            m[i].out_off < 0 || m[i].out_off + (int64_t)m[i].isize > out_bytes)
            return -dcr::set_error(DCR_EARG, "dcr_inflater_run: member " + std::to_string(i) + " outside the buffers");
    std::lock_guard<std::mutex> g(h->mu);
    hipError_t e;
    if ((e = hipSetDevice(h->device)) != hipSuccess) return -hip_fail(e, "hipSetDevice");
    if ((e = grow(h->d_in, h->cap_in, (size_t)in_bytes + dinf::kPad)) != hipSuccess ||
        (e = grow(h->d_out, h->cap_out, (size_t)out_bytes + 16)) != hipSuccess ||
        (e = grow(h->d_m, h->cap_m, (size_t)n)) != hipSuccess ||
        (e = grow(h->d_st, h->cap_st, (size_t)n)) != hipSuccess ||
        (e = grow(h->d_dbg, h->cap_dbg, (size_t)n * (DINF_STAMP ? 16 : 4))) != hipSuccess)
        return -hip_fail(e, "dcr_inflater_run: device buffers");
    std::vector<uint8_t> st((size_t)n);
    hipStream_t s = h->stream;
    if ((e = hipMemcpyAsync(h->d_in, in, (size_t)in_bytes, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(h->d_m, m, (size_t)n * sizeof(dcr_bgzf_member), hipMemcpyHostToDevice, s)) != hipSuccess)
        return -hip_fail(e, "dcr_inflater_run: upload");
    dinf::Args a = h->base;
    a.in = h->d_in;
    a.out = h->d_out;
    a.m = h->d_m;
    a.status = h->d_st;
    a.dbg = h->d_dbg;
    a.n = n;
    (void)hipEventRecord(h->ev0, s);
    hipLaunchKernelGGL(dinf::k_inflate, dim3((unsigned)std::min(n, h->grid_cap)), dim3(64), sizeof(dinf::WaveLds), s,
                       a);
    if ((e = hipGetLastError()) != hipSuccess) return -hip_fail(e, "k_inflate launch");
    (void)hipEventRecord(h->ev1, s);
    if ((e = hipMemcpyAsync(out, h->d_out, (size_t)out_bytes, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipMemcpyAsync(st.data(), h->d_st, (size_t)n, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return -hip_fail(e, "dcr_inflater_run: download");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return -hip_fail(e, "dcr_inflater_run: sync");
    (void)hipEventElapsedTime(&h->last_ms, h->ev0, h->ev1);
    h->last_n = n;
    h->tot[0] += h->last_ms;
    h->tot[1] += 1;
    h->tot[2] += n;
    h->tot[3] += (double)out_bytes;
    if (DINF_STAMP) {
        std::vector<uint32_t> dbg((size_t)n * 16);
        (void)hipMemcpy(dbg.data(), h->d_dbg, dbg.size() * 4, hipMemcpyDeviceToHost);
        for (int32_t i = 0; i < n; ++i)
            for (int k = 0; k < 16; ++k) h->stamp[k] += dbg[(size_t)i * 16 + k];
    }
    for (int32_t i = 0; i < n; ++i)
        if (st[(size_t)i] != dinf::ST_OK) {
            uint32_t dbg[4] = {0, 0, 0, 0};
            (void)hipMemcpy(dbg, h->d_dbg + 4 * (size_t)i, sizeof(dbg), hipMemcpyDeviceToHost);
            const int k = st[(size_t)i];
            dcr::set_error(DCR_EARG, "BGZF member " + std::to_string(i) +
                                         (k == dinf::ST_CRC    ? ": CRC32 mismatch"
                                          : k == dinf::ST_SIZE ? ": ISIZE mismatch"
                                          : k == dinf::ST_GUARD ? ": decoder iteration guard"
                                                                : ": invalid deflate stream") +
                                         " (loop " + std::to_string(dbg[0] >> 8) + ", input bits " +
                                         std::to_string(dbg[1]) + ", output " + std::to_string(dbg[2]) +
                                         ", iterations " + std::to_string(dbg[3]) + ")");
            return i + 1;
        }
    return 0;
}

int dcr_inflater_last(dcr_inflater *h, float *kernel_ms, int32_t *n_members) {
    if (!h) return dcr::set_error(DCR_EARG, "dcr_inflater_last: null inflater");
    if (kernel_ms) *kernel_ms = h->last_ms;
    if (n_members) *n_members = h->last_n;
    return 0;
}

int dcr_inflater_totals(dcr_inflater *h, double *out4, int reset) {
    if (!h || !out4) return dcr::set_error(DCR_EARG, "dcr_inflater_totals: null argument");
    std::lock_guard<std::mutex> g(h->mu);
    for (int i = 0; i < 4; ++i) out4[i] = h->tot[i];
    if (reset)
        for (double &t : h->tot) t = 0;
    return 0;
}

// diagnostic (not in include/dcr_inflate.h): the summed phase stamps of a
// DINF_STAMP build (0 otherwise)
extern "C" int dcr_inflater_stamps(dcr_inflater *h, double *out16, int reset) {
    if (!h || !out16) return dcr::set_error(DCR_EARG, "dcr_inflater_stamps: null argument");
    std::lock_guard<std::mutex> g(h->mu);
    for (int i = 0; i < 16; ++i) out16[i] = h->stamp[i];
    if (reset)
        for (double &t : h->stamp) t = 0;
    return DINF_STAMP;
}

// ---- streaming: spans of members launched ahead of the reader ---------------
// The protocol (spans, slots, when a slot is reused) is csrc/dcr_span_stream.h;
// this backend copies a span's compressed bytes from page-locked staging to
// the device, launches k_inflate into the slot's device output and DMAs
// fetched ranges into the caller's page-locked chunk buffer.  The slots'
// device and page-locked buffers belong to the inflater and outlive a stream.
namespace {
hipError_t pinned_grow(uint8_t *&p, size_t &cap, size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc((void **)&p, n, hipHostMallocDefault);
    if (e == hipSuccess) cap = n;
    return e;
}

struct HipSpanBackend {
    using Event = hipEvent_t;
    dcr_inflater *h;
    InflSlots &S;
    bool new_events(Event &start, Event &done) {
        return hipEventCreateWithFlags(&done, hipEventBlockingSync) == hipSuccess &&
               hipEventCreate(&start) == hipSuccess;
    }
    void free_events(Event &start, Event &done) {
        if (start) (void)hipEventDestroy(start);
        if (done) (void)hipEventDestroy(done);
        start = done = nullptr;
    }
    bool ensure(int slot, size_t nin, size_t nout, int32_t n) {
        (void)hipSetDevice(h->device);
        return pinned_grow(S.h_stage[slot], S.cap_stage[slot], nin + 16) == hipSuccess &&
               pinned_grow(S.h_st[slot], S.cap_hst[slot], (size_t)n) == hipSuccess &&
               grow(S.d_in[slot], S.cap_in[slot], nin + dinf::kPad) == hipSuccess &&
               grow(S.d_out[slot], S.cap_out[slot], nout + 16) == hipSuccess &&
               grow(S.d_m[slot], S.cap_m[slot], (size_t)n) == hipSuccess &&
               grow(S.d_st[slot], S.cap_dst[slot], (size_t)n) == hipSuccess;
    }
    uint8_t *stage(int slot) { return S.h_stage[slot]; }
    bool launch(int slot, const dcr_bgzf_member *rel, int32_t n, size_t nin, Event start, Event done) {
        dinf::Args a = h->base;
        a.in = S.d_in[slot];
        a.out = S.d_out[slot];
        a.m = S.d_m[slot];
        a.status = S.d_st[slot];
        a.dbg = nullptr;
        a.n = n;
        // rel is the producer's per-slot copy: it is rewritten only after
        // this span is done (the protocol waits for `done` before reusing)
        if (hipMemcpyAsync(S.d_in[slot], S.h_stage[slot], nin, hipMemcpyHostToDevice, S.s_k) != hipSuccess ||
            hipMemcpyAsync(S.d_m[slot], rel, (size_t)n * sizeof(dcr_bgzf_member), hipMemcpyHostToDevice, S.s_k) !=
                hipSuccess ||
            hipEventRecord(start, S.s_k) != hipSuccess)
            return false;
        hipLaunchKernelGGL(dinf::k_inflate, dim3((unsigned)std::min(n, h->grid_cap)), dim3(64), sizeof(dinf::WaveLds),
                           S.s_k, a);
        return hipGetLastError() == hipSuccess &&
               hipMemcpyAsync(S.h_st[slot], S.d_st[slot], (size_t)n, hipMemcpyDeviceToHost, S.s_k) == hipSuccess &&
               hipEventRecord(done, S.s_k) == hipSuccess;
    }
    bool wait(Event start, Event done, float *ms) {
        if (hipEventSynchronize(done) != hipSuccess) return false;
        if (ms) {
            *ms = 0;
            (void)hipEventElapsedTime(ms, start, done);
        }
        return true;
    }
    const uint8_t *status(int slot) { return S.h_st[slot]; }
    bool copy_out(uint8_t *dst, int slot, int64_t off, int64_t n) {
        return hipMemcpyAsync(dst, S.d_out[slot] + off, (size_t)n, hipMemcpyDeviceToHost, S.s_out) == hipSuccess;
    }
    bool sync_out() { return hipStreamSynchronize(S.s_out) == hipSuccess; }
    void drain() {
        (void)hipSetDevice(h->device);
        if (S.s_k) (void)hipStreamSynchronize(S.s_k);
        if (S.s_out) (void)hipStreamSynchronize(S.s_out);
    }
    void account(float ms, int32_t members, int64_t bytes) {
        std::lock_guard<std::mutex> g(h->mu);
        if (members) {
            h->tot[0] += ms;
            h->tot[1] += 1;
            h->tot[2] += members;
        }
        h->tot[3] += (double)bytes;
    }
    void error(const std::string &msg) { dcr::set_error(DCR_EARG, msg); }
};
}  // namespace

static_assert(InflSlots::kSlots == dcr_span::kSlots, "one device slot per protocol slot");

struct dcr_inflate_stream {
    HipSpanBackend be;
    dcr_span::Stream<HipSpanBackend> s;
    dcr_inflate_stream(dcr_inflater *h, const uint8_t *file) : be{h, *h->slots}, s(be, file) {}
};

extern "C" dcr_inflate_stream *dcr_inflate_stream_open(dcr_inflater *h, const uint8_t *file) {
    if (!h || !file) {
        dcr::set_error(DCR_EARG, "dcr_inflate_stream_open: bad arguments");
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> g(h->mu);
        if (!h->slots) h->slots = new InflSlots;
        if (h->slots->busy) {            // one stream per inflater at a time
            dcr::set_error(DCR_EARG, "dcr_inflate_stream_open: the inflater's stream is in use");
            return nullptr;
        }
        h->slots->busy = true;
    }
    InflSlots &S = *h->slots;
    (void)hipSetDevice(h->device);
    auto make_k = [&]() {
        if (DINF_CU_SHARE <= 0) return hipStreamCreateWithFlags(&S.s_k, hipStreamNonBlocking);
        std::vector<uint32_t> mask((size_t)(h->n_cu + 31) / 32, 0u);
        for (int i = 0; i < h->n_cu; ++i)
            if (i % 8 < DINF_CU_SHARE) mask[(size_t)i / 32] |= 1u << (i % 32);
        return hipExtStreamCreateWithCUMask(&S.s_k, (uint32_t)mask.size(), mask.data());
    };
    if ((!S.s_k && make_k() != hipSuccess) ||
        (!S.s_out && hipStreamCreateWithFlags(&S.s_out, hipStreamNonBlocking) != hipSuccess)) {
        std::lock_guard<std::mutex> g(h->mu);
        S.busy = false;
        dcr::set_error(DCR_EHIP, "dcr_inflate_stream_open: HIP setup failed");
        return nullptr;
    }
    auto *st = new dcr_inflate_stream(h, file);
    st->s.start();
    return st;
}

extern "C" int dcr_inflate_stream_add(dcr_inflate_stream *st, const dcr_bgzf_member *m, int32_t n, int32_t last) {
    if (!st || n < 0 || (n && !m)) return dcr::set_error(DCR_EARG, "dcr_inflate_stream_add: bad arguments");
    for (int32_t i = 0; i < n; ++i)
        if (m[i].isize > 65536 || m[i].in_off < 0 || m[i].out_off < 0)
            return dcr::set_error(DCR_EARG, "dcr_inflate_stream_add: member out of range");
    return st->s.add(m, n, last);
}

extern "C" int dcr_inflate_stream_fetch(dcr_inflate_stream *st, int64_t out_off, int64_t n, uint8_t *dst) {
    if (!st || n < 0 || (n && !dst)) return -1;
    (void)hipSetDevice(st->be.h->device);
    return st->s.fetch(out_off, n, dst);
}

extern "C" void dcr_inflate_stream_close(dcr_inflate_stream *st) {
    if (!st) return;
    st->s.close();
    dcr_inflater *h = st->be.h;
    delete st;
    std::lock_guard<std::mutex> g(h->mu);
    h->slots->busy = false;
}

static void *hook_stream_open(void *u, const uint8_t *file) {
    return dcr_inflate_stream_open((dcr_inflater *)u, file);
}
static int hook_stream_add(void *s, const dcr_bgzf_member *m, int32_t n, int32_t last) {
    return dcr_inflate_stream_add((dcr_inflate_stream *)s, m, n, last);
}
static int hook_stream_fetch(void *s, int64_t off, int64_t n, uint8_t *dst) {
    return dcr_inflate_stream_fetch((dcr_inflate_stream *)s, off, n, dst);
}
static void hook_stream_close(void *s) { dcr_inflate_stream_close((dcr_inflate_stream *)s); }

static int hook_run(void *u, const uint8_t *in, int64_t in_bytes, const dcr_bgzf_member *m, int32_t n, uint8_t *out,
                    int64_t out_bytes) {
    const int r = dcr_inflater_run((dcr_inflater *)u, in, in_bytes, m, n, out, out_bytes);
    return r < 0 ? -1 : r;
}
static void *hook_alloc(void *u, size_t bytes) {
    auto *h = (dcr_inflater *)u;
    std::lock_guard<std::mutex> g(h->mu);
    auto it = h->free_host.find(bytes);
    void *p = nullptr;
    if (it != h->free_host.end()) {
        p = it->second;
        h->free_host.erase(it);
    } else {
        (void)hipSetDevice(h->device);
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    }
    h->live_host[p] = bytes;
    return p;
}
static void hook_free(void *u, void *p) {
    auto *h = (dcr_inflater *)u;
    std::lock_guard<std::mutex> g(h->mu);
    auto it = h->live_host.find(p);
    if (it == h->live_host.end()) return;
    h->free_host.emplace(it->second, p);
    h->live_host.erase(it);
}

int dcr_inflater_hook(dcr_inflater *h, dcr_inflate_hook *hook) {
    if (!h || !hook) return dcr::set_error(DCR_EARG, "dcr_inflater_hook: null argument");
    hook->user = h;
    hook->run = hook_run;
    hook->host_alloc = hook_alloc;
    hook->host_free = hook_free;
    hook->stream_open = hook_stream_open;
    hook->stream_add = hook_stream_add;
    hook->stream_fetch = hook_stream_fetch;
    hook->stream_close = hook_stream_close;
    return 0;
}

}  // extern "C"
