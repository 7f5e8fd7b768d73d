// dcr_deflate.h — BGZF block compressor for gfx950: one 256-lane workgroup
// per block of <= 0xff00 input bytes, producing one RFC 1951 dynamic-Huffman
// block (or a stored block when that is smaller) inside an RFC 1952 member
// with the BGZF "BC" extra field (SAM spec v1.6 §4.1), CRC32 and ISIZE.
//
// The same phase functions run as the device kernel (dcr_writer.hip, one
// lane per thread, barriers between phases) and as a sequential lane-by-lane
// emulation on the host (dcr_deflate_emulate in libdcr_io.so), so the CPU
// tests can check the GPU's algorithm against zlib / libdeflate inflate.
//
// Algorithm (per block):
//   P0  stage the block in LDS, clear the tables / histograms
//   P1  hash every 4-byte position: earliest position per hash in each 32 KiB
//       half and latest in the first half (LDS atomics)
//   P2  each lane greedily parses its contiguous sub-block (256 sub-blocks per
//       block; matches end at the sub-block end) against those candidates and
//       distances 1..4, counting literal/length and distance symbols and
//       keeping its tokens (one word per match, literals by run length) in a
//       per-workgroup token buffer; every lane: the CRC32 of its sub-block
//   P3  symbol ranks (all lanes), then thread 0: Huffman code lengths
//       (in-place minimum-redundancy code of Moffat & Katajainen, lengths
//       limited to 15 / 7) and the run-length-coded header; canonical codes
//   P4  each lane replays its tokens and counts its bits; exclusive scan,
//       CRC combine, stored-or-compressed decision
//   P5  each lane replays its tokens and writes its bits (plain stores for
//       the words it owns, atomic or for the one or two it shares with its
//       neighbours, which the scan zeroed); lane 0 writes the gzip / BGZF
//       header and the Huffman header ahead of its tokens, the last lane
//       end of block, CRC32 and ISIZE after its own.  A stored block (when
//       that is smaller) is written with plain byte stores instead.
#pragma once
#include <stdint.h>
#include <type_traits>
#include <string.h>

#if defined(__HIPCC__)
#define DFL_HD __host__ __device__
#else
#define DFL_HD
#endif

#if defined(__clang__)
#define DFL_UNROLL _Pragma("unroll")
#else
#define DFL_UNROLL
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define DFL_DEVICE 1
#else
#define DFL_DEVICE 0
#endif

namespace dfl {

#ifndef DFL_T
#define DFL_T 256
#endif
#ifndef DFL_LS
#define DFL_LS 32
#endif
#ifndef DFL_MW
#define DFL_MW 4                           // dwords per side per match-extension step
#endif
constexpr int kT = DFL_T;                 // lanes per block
#ifndef DFL_MAXIN
#define DFL_MAXIN 0xff00
#endif
constexpr uint32_t kMaxIn = DFL_MAXIN;    // input bytes per BGZF block
#ifndef DFL_HB
#define DFL_HB 11
#endif
#ifndef DFL_CRCS
#define DFL_CRCS 8                         // device CRC32 slice-by-N from LDS tables, N = 4 or 8 (0: bit by bit)
#endif
#ifndef DFL_SPEC
#define DFL_SPEC 1                         // device parse: batched table warm-up, p + 1 preloaded (parse_dev)
#endif
#ifndef DFL_P1W
#define DFL_P1W 1                          // device block hash: one dword load per four positions
#endif
#ifndef DFL_CODES_EARLY
#define DFL_CODES_EARLY 1                  // device: literal / distance codes on waves 1-3 during the header
#endif
#ifndef DFL_CRC_LATE
#define DFL_CRC_LATE 1                     // device: sub-block CRCs on the waves the code-length phase leaves idle
#endif
#ifndef DFL_XQ
#define DFL_XQ 1                           // device match extension: one candidate queue per lane (0: candidate by candidate)
#endif
constexpr int kHB = DFL_HB;
constexpr int kHN = 1 << kHB;
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kSlot = 65536;         // output slot bytes (one BGZF block at most)
constexpr uint32_t kMaxDeflate = kSlot - 26;
constexpr int kLS = DFL_LS;               // lane-private recency table: sets x 2 ways
// tokens per lane: <= 63 matches (>= 4 bytes each in <= 255 bytes) and the
// tail literal run; entry e of lane l at tok[e * kT + l]:
//   bit 31 tail | bits 23..30 literal run before | 15..22 length - 4 | 0..14 distance - 1
constexpr int kTokE = 64;
constexpr uint32_t kTokWords = (uint32_t)kTokE * kT;

struct alignas(16) Shared {
    uint8_t in[kMaxIn + 4 * DFL_MW + 32];   // zero padding: match_len reads past the end
    union {
        struct {
            uint32_t a_min[kHN], a_max[kHN], b_min[kHN];   // positions (a_max: position + 1, 0 none)
            uint16_t lt[kT][2 * kLS];     // per lane: latest positions + 1 per hash set (2 ways)
        };
        uint32_t stage[(3 * kHN * 4 + kT * 2 * kLS * 2) / 4];   // P5: the compressed member (after P2)
    };
#if DFL_CRCS
    uint32_t crc_t[DFL_CRCS][256];        // slice-by-N CRC32 tables, filled once per workgroup (k_deflate)
#endif
    uint32_t lit_freq[288], dist_freq[32];
    uint8_t lit_len[288], dist_len[32], cl_len[19];
    uint16_t lit_code[288], dist_code[32], cl_code[19];   // bit-reversed (LSB-first) codes
    uint32_t lit_cl[288], dist_cl[32];    // code | length << 16: one LDS load per symbol in P4 / P5
    uint32_t lane_bits[kT];
    uint32_t lane_off[kT];
    uint32_t lane_crc[kT];
    uint32_t wave_sum[kT / 64], wave_crc[kT / 64];   // device scan
    uint32_t extra_bits;                  // extra bits of all matches (pass P2)
    uint32_t sort_a[320];                 // literal/length frequencies by rank, then code lengths; scratch
    uint32_t sort_d[32];                  // the same for distances
    uint32_t num_lit[33], num_dist[33];   // codes per length (length-limited)
    uint32_t last_lit, last_dist;         // highest symbol with a code
    uint32_t key_lit[288], key_dist[32];  // (freq << 9 | symbol), 0 = unused; then sorted ascending
    uint32_t srt_lit[288], srt_dist[32];  // sorted keys, then in-place code lengths
    uint32_t m_lit, m_dist;               // used symbols
    uint32_t next_code[3][16];            // canonical first codes per length: lit, dist, cl
    uint32_t t0_num[33], t0_cnt[16], t0_clf[19];   // thread-0 scratch (kept out of private memory)
    uint16_t rle[320];                    // header: code-length symbol | extra << 8
    uint32_t n_rle;
    uint32_t hlit, hdist, hclen;
    uint32_t hdr_bits, body_bits;
    uint32_t stored;
    uint32_t use_stage;                   // the member is assembled in stage[] (LDS)
    uint32_t crc;
};

// ---- tables -------------------------------------------------------------
#if DFL_DEVICE
#define DFL_CONST __constant__
#else
#define DFL_CONST static const
#endif
DFL_CONST uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99,
                                   115, 131, 163, 195, 227, 258};
DFL_CONST uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
DFL_CONST uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                    1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
DFL_CONST uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12,
                                    12, 13, 13};
DFL_CONST uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ---- atomics (host emulation: plain operations) -------------------------------
DFL_HD inline void amin(uint32_t *a, uint32_t v) {
#if DFL_DEVICE
    atomicMin(a, v);
#else
    if (v < *a) *a = v;
#endif
}
DFL_HD inline void amax(uint32_t *a, uint32_t v) {
#if DFL_DEVICE
    atomicMax(a, v);
#else
    if (v > *a) *a = v;
#endif
}
DFL_HD inline void aadd(uint32_t *a, uint32_t v) {
#if DFL_DEVICE
    atomicAdd(a, v);
#else
    *a += v;
#endif
}
DFL_HD inline void aor(uint32_t *a, uint32_t v) {
#if DFL_DEVICE
    atomicOr(a, v);
#else
    *a |= v;
#endif
}

// ---- CRC32 (reflected, 0xEDB88320), zlib's multmodp / x2nmodp ----------------
DFL_HD inline uint32_t crc_byte(uint32_t c) {
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
    return c;
}
DFL_HD inline uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (; m; m >>= 1) {          // a = 0 (never passed) ends after 32 steps
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
// x^(8 * 2^k) mod P, k = 0..16 (reflected), by repeated squaring of x^8
DFL_CONST uint32_t kX8Pow2[17] = {0x00800000u, 0x00008000u, 0xedb88320u, 0xb1e6b092u, 0xa06a2517u, 0xed627daeu,
                                  0x88d14467u, 0xd7bbfe6au, 0xec447f11u, 0x8e7ea170u, 0x6427800eu, 0x4d47bae0u,
                                  0x09fe548fu, 0x83852d0fu, 0x30362f1au, 0x7b5a9cc3u, 0x31fec169u};
// x^(8n) mod P (n <= 65536, a BGZF member's ISIZE at most): the register shift of n zero bytes
DFL_HD inline uint32_t x8nmodp(uint32_t n) {
    uint32_t p = 1u << 31;         // 1
    for (int k = 0; n; ++k, n >>= 1)
        if (n & 1) p = multmodp(kX8Pow2[k], p);
    return p;
}

// ---- input access -------------------------------------------------------------
DFL_HD inline uint32_t ld32(const Shared &s, uint32_t p) {
#if DFL_DEVICE
    // two aligned LDS dwords and a byte funnel shift
    const uint32_t *w = reinterpret_cast<const uint32_t *>(s.in);
    return __builtin_amdgcn_alignbyte(w[(p >> 2) + 1], w[p >> 2], p & 3);
#else
    return (uint32_t)s.in[p] | ((uint32_t)s.in[p + 1] << 8) | ((uint32_t)s.in[p + 2] << 16) |
           ((uint32_t)s.in[p + 3] << 24);
#endif
}
DFL_HD inline uint32_t hash4(uint32_t v) { return (v * 0x9E3779B1u) >> (32 - kHB); }

DFL_HD inline void lane_range(uint32_t n, int lane, uint32_t &lo, uint32_t &hi) {
    const uint32_t S = (n + kT - 1) / kT;
    lo = (uint32_t)lane * S;
    if (lo > n) lo = n;
    hi = lo + S;
    if (hi > n) hi = n;
}

// length of the common prefix of in[c..] and in[p..], at most lim (reads
// stay below p + lim + 4 * kMW + 4 <= n + 4 * kMW + 4, inside the zero padding of in[])
DFL_HD inline uint32_t match_len(const Shared &s, uint32_t c, uint32_t p, uint32_t lim) {
#if DFL_DEVICE
    // kMW * 4 bytes per step: kMW new aligned LDS dwords per side issued
    // together (one LDS round trip), byte funnel shifts, the first
    // differing byte from the lowest set bit of the xor.  The workgroup is
    // alone on its CU (LDS), so registers are plentiful and a wide step
    // shortens the longest match of a wave, which every lane waits for.
    constexpr int kMW = DFL_MW;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(s.in);
    uint32_t ia = c >> 2, ib = p >> 2;
    const uint32_t sa = c & 3, sb = p & 3;
    uint32_t a0 = w[ia], b0 = w[ib], l = 0;
    while (l < lim) {
        uint32_t a[kMW + 1], b[kMW + 1], x[kMW];
        a[0] = a0;
        b[0] = b0;
DFL_UNROLL
        for (int k = 1; k <= kMW; ++k) { a[k] = w[ia + k]; b[k] = w[ib + k]; }
        uint32_t any = 0;
DFL_UNROLL
        for (int k = 0; k < kMW; ++k) {
            x[k] = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sa) ^ __builtin_amdgcn_alignbyte(b[k + 1], b[k], sb);
            any |= x[k];
        }
        if (any) {
            uint32_t kk = kMW - 1, xx = x[kMW - 1];
DFL_UNROLL
            for (int k = kMW - 2; k >= 0; --k)
                if (x[k]) { kk = (uint32_t)k; xx = x[k]; }
            l += 4 * kk + ((uint32_t)__builtin_ctz(xx) >> 3);
            break;
        }
        l += 4 * kMW;
        ia += kMW;
        ib += kMW;
        a0 = a[kMW];
        b0 = b[kMW];
    }
    return l < lim ? l : lim;
#else
    uint32_t l = 0;
    while (l < lim && s.in[c + l] == s.in[p + l]) ++l;
    return l;
#endif
}

// Length / distance symbols by arithmetic (RFC 1951 3.2.5; the tables above
// are its listing): the tables are in global memory on the device, and a
// binary search over them was a chain of dependent loads per match in each
// of the three passes over the tokens.
struct Sym {
    uint32_t sym, nb, ev;   // symbol (0-based), extra bits, extra value
};
DFL_HD inline uint32_t log2u(uint32_t x) { return 31u - (uint32_t)__builtin_clz(x); }
DFL_HD inline Sym len_code(uint32_t len) {     // len 3..258 -> symbol 257 + sym
    const uint32_t x = len - 3;
    if (x < 8) return {x, 0, 0};
    if (len == 258) return {28, 0, 0};
    const uint32_t e = log2u(x);               // 3..7
    return {4 * (e - 1) + ((x >> (e - 2)) & 3), e - 2, x & ((1u << (e - 2)) - 1)};
}
DFL_HD inline Sym dist_code(uint32_t d) {      // d 1..32768
    const uint32_t x = d - 1;
    if (x < 4) return {x, 0, 0};
    const uint32_t e = log2u(x);               // 2..14
    return {2 * e + ((x >> (e - 1)) & 1), e - 1, x & ((1u << (e - 1)) - 1)};
}

// lane-private recency table (deterministic: one lane, positions in order)
DFL_HD inline void lt_insert(uint16_t *t, uint32_t h, uint32_t p) {
    const uint32_t set = (h & (kLS - 1)) * 2;
    t[set + 1] = t[set];
    t[set] = (uint16_t)(p + 1);
}

// candidate i for a lane-varying i: c0..c3 from the tables, then p - 1 .. p - 4
// (a select tree: a chain of selects over an array became an indexed load
// from private memory)
DFL_HD inline uint32_t cand_at(uint32_t i, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t p) {
    const uint32_t lo = i & 1 ? c1 : c0, hi = i & 1 ? c3 : c2;
    const uint32_t t = i & 2 ? hi : lo;
    return i < 4 ? t : p + 3 - i;
}

// greedy parse of [lo, hi): v.lit(byte) / v.match(len, dist).  Candidates
// for position p, in this order: the lane's two latest positions with the
// same hash set (its table holds the previous sub-block and its own
// positions so far), the earliest / latest block positions with the same
// hash (P1), and distances 1..4; the first longest match wins.
// Positions inside a match are not inserted into the lane's table: lanes
// of a wave would wait for the longest match of every step (measured: a
// quarter of the kernel), and the table keeps older, equally useful
// positions instead (slightly better ratio on record streams).
//
// Per position the candidate positions are loaded together and their first
// four bytes compared together (one LDS round trip each), so a literal costs
// three round trips; only candidates that match >= 4 bytes are extended, in
// candidate order, skipping any that cannot beat the best so far.
#if DFL_DEVICE && DFL_SPEC
// The device parse: the same decisions as parse() below, scheduled for
// fewer dependent LDS round trips per lane.
//  - The recency table is warmed 8 positions per round trip: the 8 sets'
//    dwords are loaded together and a set repeated within the batch takes
//    the earlier position in registers (the stores then go out in order).
//  - The dwords around p stay in registers (W0..W3: dwords pi-1 .. pi+2);
//    a literal step shifts them by a dword at most, loading the next one
//    ahead, so only a match reloads them.
//  - Each step also loads the set dword and the block-hash candidates of
//    p + 1; after a literal they are the next step's (the set dword with
//    this step's insert forwarded when p + 1 falls in the same set), so a
//    literal run costs one round trip per position (its candidates' bytes).
template <class V>
DFL_HD inline void parse_dev(Shared &s, uint32_t n, int lane, uint32_t lo, uint32_t hi, V &v) {
    uint16_t *t = s.lt[lane];
    uint32_t *t32 = reinterpret_cast<uint32_t *>(t);
    const uint32_t *wi = reinterpret_cast<const uint32_t *>(s.in);
DFL_UNROLL
    for (int i = 0; i < kLS; ++i) t32[i] = 0;
    {
        const uint32_t S = hi - lo;
#ifdef DFL_ABL_NOWARM                      // ablation: no table warm-up
        for (uint32_t qb = lo; qb < lo; qb += 8) {
#else
        for (uint32_t qb = lo >= S ? lo - S : 0; qb < lo; qb += 8) {
#endif
            const uint32_t di = qb >> 2, o = qb & 3;
            const uint32_t D0 = wi[di], D1 = wi[di + 1], D2 = wi[di + 2], D3 = wi[di + 3];
            const uint32_t E[3] = {__builtin_amdgcn_alignbyte(D1, D0, o), __builtin_amdgcn_alignbyte(D2, D1, o),
                                   __builtin_amdgcn_alignbyte(D3, D2, o)};
            uint32_t set[8], old[8];
            bool on[8];
DFL_UNROLL
            for (int j = 0; j < 8; ++j) {
                const uint32_t q = qb + (uint32_t)j;
                const uint32_t vq = (j & 3) ? __builtin_amdgcn_alignbyte(E[(j >> 2) + 1], E[j >> 2], (uint32_t)(j & 3))
                                            : E[j >> 2];
                on[j] = q < lo && q + 4 <= n;
                set[j] = hash4(vq) & (kLS - 1);
                old[j] = t32[set[j]];
            }
DFL_UNROLL
            for (int j = 0; j < 8; ++j) {
                uint32_t w0 = old[j] & 0xffff;
DFL_UNROLL
                for (int i = 0; i < j; ++i) w0 = (on[i] && set[i] == set[j]) ? qb + (uint32_t)i + 1 : w0;
                if (on[j]) t32[set[j]] = (w0 << 16) | (qb + (uint32_t)j + 1);
            }
        }
    }
    uint32_t p = lo, pi = p >> 2;
    uint32_t W0 = pi ? wi[pi - 1] : 0u, W1 = wi[pi], W2 = wi[pi + 1], W3 = wi[pi + 2];
    bool pre = false;
    uint32_t tw = 0, ca = kNone, cb = kNone;    // preloaded for p: set dword, block candidates
    while (p < hi) {
        const uint32_t lim = (hi - p) < 258 ? (hi - p) : 258;
        const bool hashed = p + 4 <= n;
        const uint32_t sh = p & 3;
        const uint32_t vp = __builtin_amdgcn_alignbyte(W2, W1, sh);
        const uint32_t h = hashed ? hash4(vp) : 0;
        const uint32_t set = h & (kLS - 1);
        if (!pre) {
            tw = t32[set];
            if (p >= 32768) {
                ca = s.b_min[h];
                const uint32_t am = s.a_max[h];
                cb = am ? am - 1 : kNone;
            } else {
                ca = s.a_min[h];
                cb = kNone;
            }
        }
        // p + 1, speculatively (its bytes are in W1..W3)
        const uint32_t q = p + 1;
        const uint32_t vq = sh < 3 ? __builtin_amdgcn_alignbyte(W2, W1, sh + 1) : W2;
        const uint32_t hq = q + 4 <= n ? hash4(vq) : 0;
        const uint32_t setq = hq & (kLS - 1);
        const uint32_t twq = t32[setq];
        uint32_t caq, cbq;
        if (q >= 32768) {
            caq = s.b_min[hq];
            const uint32_t am = s.a_max[hq];
            cbq = am ? am - 1 : kNone;
        } else {
            caq = s.a_min[hq];
            cbq = kNone;
        }
        uint32_t best = 0, bd = 0;
        const uint32_t t0 = tw & 0xffff, t1 = tw >> 16;
        if (lim >= 4) {
            uint32_t c[8];
            c[0] = t0 ? t0 - 1 : kNone;
            c[1] = t1 ? t1 - 1 : kNone;
            c[2] = ca;
            c[3] = cb;
DFL_UNROLL
            for (int k = 1; k <= 4; ++k) c[3 + k] = p >= (uint32_t)k ? p - (uint32_t)k : kNone;
            uint32_t ok = 0;
DFL_UNROLL
            for (int i = 0; i < 4; ++i)
                if (c[i] != kNone && c[i] < p && p - c[i] <= 32768 && ld32(s, c[i]) == vp) ok |= 1u << i;
DFL_UNROLL
            for (int k = 1; k <= 4; ++k) {
                const uint32_t off = 4 + sh - (uint32_t)k;
                const uint32_t vk = off < 4 ? __builtin_amdgcn_alignbyte(W1, W0, off)
                                            : __builtin_amdgcn_alignbyte(W2, W1, off - 4);
                if (p >= (uint32_t)k && vk == vp) ok |= 1u << (3 + k);
            }
            if (ok) {      // the candidate queue (see parse() below)
                constexpr int kMW = DFL_MW;
                const uint32_t lim4 = lim - 4;
                uint32_t rem = ok & (ok - 1);
                uint32_t cc = cand_at((uint32_t)__builtin_ctz(ok), c[0], c[1], c[2], c[3], p), l = 0;
                bool act = true;
                while (act) {
                    const uint32_t xa = cc + 4 + l, xb = p + 4 + l;
                    const uint32_t ia = xa >> 2, ib = xb >> 2, sa = xa & 3, sb = xb & 3;
                    uint32_t a[kMW + 1], b[kMW + 1];
DFL_UNROLL
                    for (int k = 0; k <= kMW; ++k) { a[k] = wi[ia + k]; b[k] = wi[ib + k]; }
                    uint32_t kk = kMW, xx = 0;
DFL_UNROLL
                    for (int k = kMW - 1; k >= 0; --k) {
                        const uint32_t x = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sa) ^
                                           __builtin_amdgcn_alignbyte(b[k + 1], b[k], sb);
                        if (x) { kk = (uint32_t)k; xx = x; }
                    }
                    uint32_t L = l + 4 * kMW;
                    bool fin = L >= lim4;
                    if (kk < (uint32_t)kMW) { L = l + 4 * kk + ((uint32_t)__builtin_ctz(xx) >> 3); fin = true; }
                    l += 4 * kMW;
                    if (fin) {
                        if (L > lim4) L = lim4;
                        if (4 + L > best) { best = 4 + L; bd = p - cc; }
                        if (rem && best < lim) {
                            cc = cand_at((uint32_t)__builtin_ctz(rem), c[0], c[1], c[2], c[3], p);
                            rem &= rem - 1;
                            l = 0;
                        } else {
                            act = false;
                        }
                    }
                }
            }
        }
        const uint32_t ins = (t0 << 16) | (p + 1);
        if (hashed) t32[set] = ins;
        if (best >= 4) {
            v.match(best, bd);
            p += best;
            pi = p >> 2;
            W0 = pi ? wi[pi - 1] : 0u;
            W1 = wi[pi];
            W2 = wi[pi + 1];
            W3 = wi[pi + 2];
            pre = false;
        } else {
            v.lit((uint8_t)vp);
            p = q;
            tw = (hashed && setq == set) ? ins : twq;
            ca = caq;
            cb = cbq;
            pre = true;
            if ((q >> 2) != pi) {
                pi = q >> 2;
                W0 = W1;
                W1 = W2;
                W2 = W3;
                W3 = wi[pi + 2];
            }
        }
    }
}
#endif

template <class V>
DFL_HD inline void parse(Shared &s, uint32_t n, int lane, uint32_t lo, uint32_t hi, V &v) {
#if DFL_DEVICE && DFL_SPEC
    parse_dev(s, n, lane, lo, hi, v);
    return;
#endif
    uint16_t *t = s.lt[lane];
    for (int i = 0; i < 2 * kLS; ++i) t[i] = 0;
    const uint32_t S = hi - lo;
    for (uint32_t q = lo >= S ? lo - S : 0; q < lo; ++q)
        if (q + 4 <= n) lt_insert(t, hash4(ld32(s, q)), q);
    uint32_t p = lo;
    while (p < hi) {
        const uint32_t lim = (hi - p) < 258 ? (hi - p) : 258;
        const bool hashed = p + 4 <= n;
#if DFL_DEVICE
        // the dwords around p: the bytes at p (vp) and at p - 1 .. p - 4
        // (the distance 1-4 candidates) without further loads
        const uint32_t *wi = reinterpret_cast<const uint32_t *>(s.in);
        const uint32_t pi = p >> 2, sh = p & 3;
        const uint32_t W0 = pi ? wi[pi - 1] : 0u, W1 = wi[pi], W2 = wi[pi + 1];
        const uint32_t vp = __builtin_amdgcn_alignbyte(W2, W1, sh);
#else
        const uint32_t vp = ld32(s, p);
#endif
        const uint32_t h = hashed ? hash4(vp) : 0;
        const uint32_t set = (h & (kLS - 1)) * 2;
        uint32_t best = 0, bd = 0;
        // the set's two ways in one dword (t0 the latest)
#if DFL_DEVICE
        const uint32_t tw = *reinterpret_cast<const uint32_t *>(t + set);
#else
        const uint32_t tw = t[set] | (uint32_t)t[set + 1] << 16;
#endif
        const uint32_t t0 = tw & 0xffff, t1 = tw >> 16;
        if (lim >= 4) {
            uint32_t c[8];
            c[0] = t0 ? t0 - 1 : kNone;
            c[1] = t1 ? t1 - 1 : kNone;
            if (p >= 32768) {
                c[2] = s.b_min[h];
                const uint32_t am = s.a_max[h];
                c[3] = am ? am - 1 : kNone;
            } else {
                c[2] = s.a_min[h];
                c[3] = kNone;
            }
DFL_UNROLL
            for (int k = 1; k <= 4; ++k) c[3 + k] = p >= (uint32_t)k ? p - (uint32_t)k : kNone;
            uint32_t ok = 0;
DFL_UNROLL
            for (int i = 0; i < 4; ++i)
                if (c[i] != kNone && c[i] < p && p - c[i] <= 32768 && ld32(s, c[i]) == vp) ok |= 1u << i;
DFL_UNROLL
            for (int k = 1; k <= 4; ++k) {
#if DFL_DEVICE
                // bytes p - k .. p - k + 3 from W0 W1 W2 (offset 4 + sh - k in W0)
                const uint32_t off = 4 + sh - (uint32_t)k;
                const uint32_t vk = off < 4 ? __builtin_amdgcn_alignbyte(W1, W0, off)
                                            : __builtin_amdgcn_alignbyte(W2, W1, off - 4);
#else
                const uint32_t vk = p >= (uint32_t)k ? ld32(s, p - (uint32_t)k) : 0u;
#endif
                if (p >= (uint32_t)k && vk == vp) ok |= 1u << (3 + k);
            }
#if DFL_DEVICE && DFL_XQ
            // The candidates with >= 4 matching bytes are extended through one
            // queue per lane: each iteration is one kMW-dword step of the
            // lane's current candidate, so a wave runs as many iterations as
            // its busiest lane needs, not the sum over candidate slots of the
            // most any lane needs there.  The first longest candidate wins, as
            // in the loop below (which also skips, by one byte, candidates that
            // cannot beat the best so far; here they run to their mismatch).
            if (ok) {
                constexpr int kMW = DFL_MW;
                const uint32_t *w = reinterpret_cast<const uint32_t *>(s.in);
                const uint32_t lim4 = lim - 4;
                uint32_t rem = ok & (ok - 1);
                uint32_t cc = cand_at((uint32_t)__builtin_ctz(ok), c[0], c[1], c[2], c[3], p), l = 0;
                bool act = true;
                while (act) {
                    const uint32_t xa = cc + 4 + l, xb = p + 4 + l;
                    const uint32_t ia = xa >> 2, ib = xb >> 2, sa = xa & 3, sb = xb & 3;
                    uint32_t a[kMW + 1], b[kMW + 1];
DFL_UNROLL
                    for (int k = 0; k <= kMW; ++k) { a[k] = w[ia + k]; b[k] = w[ib + k]; }
                    uint32_t kk = kMW, xx = 0;
DFL_UNROLL
                    for (int k = kMW - 1; k >= 0; --k) {
                        const uint32_t x = __builtin_amdgcn_alignbyte(a[k + 1], a[k], sa) ^
                                           __builtin_amdgcn_alignbyte(b[k + 1], b[k], sb);
                        if (x) { kk = (uint32_t)k; xx = x; }
                    }
                    uint32_t L = l + 4 * kMW;
                    bool fin = L >= lim4;
                    if (kk < (uint32_t)kMW) { L = l + 4 * kk + ((uint32_t)__builtin_ctz(xx) >> 3); fin = true; }
                    l += 4 * kMW;
                    if (fin) {
                        if (L > lim4) L = lim4;
                        if (4 + L > best) { best = 4 + L; bd = p - cc; }
                        if (rem && best < lim) {
                            cc = cand_at((uint32_t)__builtin_ctz(rem), c[0], c[1], c[2], c[3], p);
                            rem &= rem - 1;
                            l = 0;
                        } else {
                            act = false;
                        }
                    }
                }
            }
#else
DFL_UNROLL
            for (int i = 0; i < 8; ++i) {
                if (!((ok >> i) & 1) || best >= lim) continue;
                if (best && s.in[c[i] + best] != s.in[p + best]) continue;   // not longer than best
                const uint32_t l = 4 + match_len(s, c[i] + 4, p + 4, lim - 4);
                if (l > best) { best = l; bd = p - c[i]; }
            }
#endif
        }
        if (hashed) {                                       // lt_insert(t, h, p)
#if DFL_DEVICE
            *reinterpret_cast<uint32_t *>(t + set) = (t0 << 16) | (p + 1);
#else
            t[set + 1] = (uint16_t)t0;
            t[set] = (uint16_t)(p + 1);
#endif
        }
        if (best >= 4) {
            v.match(best, bd);
            p += best;
        } else {
            v.lit((uint8_t)vp);   // the byte at p (vp's low byte, also past n: zero padding)
            ++p;
        }
    }
}

struct CountV {            // P2: symbol histogram, extra bits
    Shared &s;
    uint32_t extra = 0;
#ifdef DFL_ABL_NOCNT                       // ablation (invalid members): the histogram atomics spread over bins
    int lane;
    DFL_HD void lit(uint8_t b) { aadd(&s.lit_freq[(b + (uint32_t)lane) & 255], 1); }
    DFL_HD void match(uint32_t len, uint32_t d) {
        const Sym L = len_code(len), D = dist_code(d);
        aadd(&s.lit_freq[257 + (L.sym + (uint32_t)lane) % 29], 1);
        aadd(&s.dist_freq[(D.sym + (uint32_t)lane) % 30], 1);
        extra += L.nb + D.nb;
    }
#else
    DFL_HD void lit(uint8_t b) { aadd(&s.lit_freq[b], 1); }
    DFL_HD void match(uint32_t len, uint32_t d) {
        const Sym L = len_code(len), D = dist_code(d);
        aadd(&s.lit_freq[257 + L.sym], 1);
        aadd(&s.dist_freq[D.sym], 1);
        extra += L.nb + D.nb;
    }
#endif
};

struct TokV {              // P2: the lane's tokens (kTokE layout)
    uint32_t *t;
    int lane;
    uint32_t e = 0, run = 0;
    DFL_HD void lit(uint8_t) { ++run; }
    DFL_HD void match(uint32_t len, uint32_t d) {
        t[e * kT + lane] = (run << 23) | ((len - 4) << 15) | (d - 1);
        ++e;
        run = 0;
    }
    DFL_HD void finish() { t[e * kT + lane] = (1u << 31) | (run << 23); }
};

struct CountTokV {         // P2: both
    CountV c;
    TokV t;
    DFL_HD void lit(uint8_t b) { c.lit(b); t.lit(b); }
    DFL_HD void match(uint32_t len, uint32_t d) { c.match(len, d); t.match(len, d); }
};

// the tokens of a lane again, from the token buffer
#ifndef DFL_TOKPF
#define DFL_TOKPF 4                        // token entries in flight during a replay (1 or 4)
#endif
template <class V>
DFL_HD inline void replay(const Shared &s, const uint32_t *t, int lane, uint32_t lo, V &v) {
    uint32_t p = lo;
#if DFL_TOKPF == 4
    // four entries in flight (the token buffer is in HBM / L2): a ring
    // shifted by one per entry (entries past the tail hold stale words,
    // never used)
    uint32_t x1 = t[lane], x2 = t[kT + lane], x3 = t[2 * kT + lane], x4 = t[3 * kT + lane];
    for (int e = 0; e < kTokE; ++e) {
        const uint32_t x = x1;
        x1 = x2;
        x2 = x3;
        x3 = x4;
        if (e + 4 < kTokE) x4 = t[(e + 4) * kT + lane];
#else
    uint32_t xn = t[lane];
    for (int e = 0; e < kTokE; ++e) {
        // the next entry's load is in flight while this one is replayed
        // (entries past the tail hold stale words, never used)
        const uint32_t x = xn;
        if (e + 1 < kTokE) xn = t[(e + 1) * kT + lane];
#endif
        const uint32_t run = (x >> 23) & 255;
        v.lits(p, run);
        p += run;
        if (x >> 31) break;
        const uint32_t len = ((x >> 15) & 255) + 4;
        v.match(len, (x & 0x7fff) + 1);
        p += len;
    }
}

// A literal run of a replay, four bytes per step: one unaligned dword of
// the block, then the four symbols' table entries loaded together.
template <class F>
DFL_HD inline void lit_run(const Shared &s, uint32_t p, uint32_t run, F &&f) {
    uint32_t q = 0;
    for (; q + 4 <= run; q += 4) {
        const uint32_t w = ld32(s, p + q);
        const uint32_t e0 = s.lit_cl[w & 255], e1 = s.lit_cl[(w >> 8) & 255], e2 = s.lit_cl[(w >> 16) & 255],
                       e3 = s.lit_cl[w >> 24];
        f(e0);
        f(e1);
        f(e2);
        f(e3);
    }
    for (; q < run; ++q) f(s.lit_cl[s.in[p + q]]);
}

struct BitsV {             // P4: bits of a lane's tokens
    const Shared &s;
    uint32_t bits = 0;
    DFL_HD void lits(uint32_t p, uint32_t run) {
        lit_run(s, p, run, [&](uint32_t e) { bits += e >> 16; });
    }
    DFL_HD void match(uint32_t len, uint32_t d) {
        const Sym L = len_code(len), D = dist_code(d);
        bits += (s.lit_cl[257 + L.sym] >> 16) + L.nb + (s.dist_cl[D.sym] >> 16) + D.nb;
    }
};

// LSB-first bit writer over a word array.  A word shared with the previous
// writer (first word, start not word-aligned) or the next one (last word,
// unless own_last) is or-ed atomically into a word zeroed beforehand; the
// words in between belong to this writer alone and are stored.
struct BitOut {
    uint32_t *w;
    uint64_t acc = 0;
    uint32_t nacc;          // bits in acc
    uint32_t word;          // index of acc's first word
    bool first = true, shared_first, own_last;
    DFL_HD BitOut(uint32_t *words, uint32_t bitpos, bool own_last_word)
        : w(words), nacc(bitpos & 31), word(bitpos >> 5), shared_first((bitpos & 31) != 0), own_last(own_last_word) {}
    DFL_HD uint32_t pos() const { return word * 32 + nacc; }
    DFL_HD void put(uint32_t v, uint32_t nb) {
        if (!nb) return;
        acc |= (uint64_t)v << nacc;
        nacc += nb;
        if (nacc >= 32) {
            if (first && shared_first) aor(&w[word], (uint32_t)acc);
            else w[word] = (uint32_t)acc;
            first = false;
            ++word;
            acc >>= 32;
            nacc -= 32;
        }
    }
    DFL_HD void flush() {
        if (nacc) {
            if ((first && shared_first) || !own_last) aor(&w[word], (uint32_t)acc);
            else w[word] = (uint32_t)acc;
        }
        acc = 0;
        nacc = 0;
    }
};

// The same writer without a branch per symbol (P5 into stage[]): every put
// stores one word, the completed one or, when none completed, a throwaway
// into `dummy` (a word of the lane's own nobody reads); a first word shared
// with the previous lane is kept in a register and or-ed in at flush.
struct BitOut2 {
    uint32_t *w, *dummy;
    uint64_t acc = 0;
    uint32_t nacc, word, w0, fw = 0;
    bool pend, shared_first, own_last;    // pend: the shared first word is not complete yet
    DFL_HD BitOut2(uint32_t *words, uint32_t bitpos, bool own_last_word, uint32_t *dummy_word)
        : w(words), dummy(dummy_word), nacc(bitpos & 31), word(bitpos >> 5), w0(bitpos >> 5),
          pend((bitpos & 31) != 0), shared_first((bitpos & 31) != 0), own_last(own_last_word) {}
    DFL_HD uint32_t pos() const { return word * 32 + nacc; }
    DFL_HD void put(uint32_t v, uint32_t nb) {     // nb <= 32, v < 2^nb
        acc |= (uint64_t)v << nacc;
        nacc += nb;
        const bool full = nacc >= 32;
        const uint32_t lo = (uint32_t)acc;
        *(full && !pend ? &w[word] : dummy) = lo;
        fw = full && pend ? lo : fw;
        pend = pend && !full;
        word += full ? 1u : 0u;
        acc = full ? acc >> 32 : acc;
        nacc -= full ? 32u : 0u;
    }
    DFL_HD void flush() {
        if (shared_first && !pend) aor(&w[w0], fw);
        if (nacc) {
            if (pend || !own_last) aor(&w[word], (uint32_t)acc);
            else w[word] = (uint32_t)acc;
        }
        acc = 0;
        nacc = 0;
    }
};

// P5 with BitOut2: two literal codes (<= 15 bits each) per put, a length or
// distance code with its extra bits in one put
struct EmitV2 {
    const Shared &s;
    BitOut2 &o;
    DFL_HD void lits(uint32_t p, uint32_t run) {
        uint32_t q = 0;
        for (; q + 4 <= run; q += 4) {
            const uint32_t w = ld32(s, p + q);
            const uint32_t e0 = s.lit_cl[w & 255], e1 = s.lit_cl[(w >> 8) & 255], e2 = s.lit_cl[(w >> 16) & 255],
                           e3 = s.lit_cl[w >> 24];
            o.put((e0 & 0xffff) | (e1 & 0xffff) << (e0 >> 16), (e0 >> 16) + (e1 >> 16));
            o.put((e2 & 0xffff) | (e3 & 0xffff) << (e2 >> 16), (e2 >> 16) + (e3 >> 16));
        }
        for (; q < run; ++q) {
            const uint32_t e = s.lit_cl[s.in[p + q]];
            o.put(e & 0xffff, e >> 16);
        }
    }
    DFL_HD void match(uint32_t len, uint32_t d) {
        const Sym L = len_code(len), D = dist_code(d);
        const uint32_t le = s.lit_cl[257 + L.sym], de = s.dist_cl[D.sym];
        o.put((le & 0xffff) | L.ev << (le >> 16), (le >> 16) + L.nb);
        o.put((de & 0xffff) | D.ev << (de >> 16), (de >> 16) + D.nb);
    }
};

struct EmitV {             // P5: write a lane's tokens
    const Shared &s;
    BitOut &o;
    DFL_HD void lits(uint32_t p, uint32_t run) {
        lit_run(s, p, run, [&](uint32_t e) { o.put(e & 0xffff, e >> 16); });
    }
    DFL_HD void match(uint32_t len, uint32_t d) {
        const Sym L = len_code(len), D = dist_code(d);
        const uint32_t le = s.lit_cl[257 + L.sym], de = s.dist_cl[D.sym];
        o.put(le & 0xffff, le >> 16);
        o.put(L.ev, L.nb);
        o.put(de & 0xffff, de >> 16);
        o.put(D.ev, D.nb);
    }
};

// ---- Huffman code lengths (one wave) ----------------------------------------------
// The serial code below runs on one lane.  DFL_SERIAL_WAVE=1 runs it on a
// whole wave with the same data in every lane instead: each LDS read goes
// through DFL_U() (readfirstlane), so indices and loop bounds live in scalar
// registers and the branches are scalar; every lane stores the same value to
// the same address.  That measured slower (readfirstlane after each LDS
// load), so one lane it is.  The host emulation runs it once (lane 0).
#ifndef DFL_SERIAL_WAVE
#define DFL_SERIAL_WAVE 0      // 1: a whole wave with readfirstlane reads (measured slower: 6.95 vs 6.56 ms)
#endif
#if DFL_DEVICE && DFL_SERIAL_WAVE
#define DFL_U(x) __builtin_amdgcn_readfirstlane((uint32_t)(x))
#else
#define DFL_U(x) ((uint32_t)(x))
#endif
// the wave that runs a serial step: the device's whole wave of `lane0`, the host's lane0 itself
DFL_HD inline bool serial_lane(int lane, int lane0) {
#if DFL_DEVICE && DFL_SERIAL_WAVE
    return (lane >> 6) == (lane0 >> 6);
#else
    return lane == lane0;
#endif
}
// In-place minimum-redundancy code lengths (Moffat & Katajainen 1995) over
// a[0..m) = frequencies sorted ascending; on return a[i] is the code length
// of the i-th symbol (non-increasing in i).
DFL_HD inline void mr_lengths(uint32_t *a, int m) {
    if (m == 1) { a[0] = 1; return; }
    // phase 1: internal-node weights and parent pointers
    a[0] = DFL_U(a[0]) + DFL_U(a[1]);
    int root = 0, leaf = 2;
    for (int next = 1; next < m - 1; ++next) {
        const uint32_t ar = DFL_U(a[root]), al = leaf < m ? DFL_U(a[leaf]) : 0u;
        uint32_t w;
        if (leaf >= m || ar < al) { w = ar; a[root++] = (uint32_t)next; }
        else { w = al; ++leaf; }
        const uint32_t ar2 = root < next ? DFL_U(a[root]) : 0u, al2 = leaf < m ? DFL_U(a[leaf]) : 0u;
        if (leaf >= m || (root < next && ar2 < al2)) { w += ar2; a[root++] = (uint32_t)next; }
        else { w += al2; ++leaf; }
        a[next] = w;
    }
    // phase 2: internal-node depths
    a[m - 2] = 0;
    for (int next = m - 3; next >= 0; --next) a[next] = DFL_U(a[DFL_U(a[next])]) + 1;
    // phase 3: leaf depths
    int avail = 1, used = 0, depth = 0;
    root = m - 2;
    int next = m - 1;
    while (avail > 0) {
        while (root >= 0 && (int)DFL_U(a[root]) == depth) { ++used; --root; }
        while (avail > used) { a[next--] = (uint32_t)depth; --avail; }
        avail = 2 * used;
        ++depth;
        used = 0;
    }
}

// The same code as mr_lengths, as counts of codes per length (num[0..32],
// lengths above 32 counted at 32) and with the serial chains of LDS loads
// batched: in phase 1 the leaves and the internal nodes are consumed in
// order, so the next two of each are loaded together up front (an internal
// node at root + 1 is only used once it exists, root + 1 < next); phase 2
// takes the parent pointers of eight nodes in one go, then their parents'
// depths (a parent inside the batch from the batch's own registers);
// phase 3 counts equal depths eight at a time.  a[] is scratch afterwards.
DFL_HD inline void mr_counts(uint32_t *a, int m, uint32_t *num) {
    for (int i = 0; i <= 32; ++i) num[i] = 0;
    if (m == 1) { num[1] = 1; return; }
    // phase 1
    a[0] = a[0] + a[1];
    int root = 0, leaf = 2;
    for (int next = 1; next < m - 1; ++next) {
        const uint32_t r0 = a[root], r1 = a[root + 1];
        const uint32_t l0 = leaf < m ? a[leaf] : 0u, l1 = leaf + 1 < m ? a[leaf + 1] : 0u;
        uint32_t w;
        bool took_root;
        if (leaf >= m || r0 < l0) { w = r0; a[root] = (uint32_t)next; took_root = true; }
        else { w = l0; took_root = false; }
        const int root2 = took_root ? root + 1 : root, leaf2 = took_root ? leaf : leaf + 1;
        const uint32_t rv = took_root ? r1 : r0, lv = took_root ? l0 : l1;
        if (leaf2 >= m || (root2 < next && rv < lv)) { w += rv; a[root2] = (uint32_t)next; root = root2 + 1; leaf = leaf2; }
        else { w += lv; root = root2; leaf = leaf2 + 1; }
        a[next] = w;
    }
    // phase 2: internal-node depths (node m - 2 is the root)
    a[m - 2] = 0;
    constexpr int B = 8;
    for (int next = m - 3; next >= 0; next -= B) {
        uint32_t ptr[B], dep[B], got[B];
DFL_UNROLL
        for (int k = 0; k < B; ++k) ptr[k] = next - k >= 0 ? a[next - k] : (uint32_t)(m - 2);
DFL_UNROLL
        for (int k = 0; k < B; ++k) got[k] = a[ptr[k]];
DFL_UNROLL
        for (int k = 0; k < B; ++k) {
            // parent inside this batch: node ptr[k] = next - j, j < k
            uint32_t d = got[k];
DFL_UNROLL
            for (int j = 0; j < k; ++j)
                if (ptr[k] == (uint32_t)(next - j)) d = dep[j];
            dep[k] = d + 1;
            if (next - k >= 0) a[next - k] = dep[k];
        }
    }
    // phase 3: leaves per depth; internal depths are non-decreasing as the
    // index falls
    int avail = 1, depth = 0;
    int r = m - 2;
    while (avail > 0) {
        int used = 0;
        for (;;) {
            uint32_t v[B];
DFL_UNROLL
            for (int k = 0; k < B; ++k) v[k] = r - k >= 0 ? a[r - k] : 0xffffffffu;
            int eq = 0;
DFL_UNROLL
            for (int k = 0; k < B; ++k) eq += (v[k] == (uint32_t)depth) ? 1 : 0;
            used += eq;
            r -= eq;
            if (eq < B) break;
        }
        const int leaves = avail - used;
        num[depth > 32 ? 32 : depth] += (uint32_t)leaves;
        avail = 2 * used;
        ++depth;
    }
}

// Length-limit code lengths a[0..m) (non-increasing, from mr_lengths) to
// max_len and hand them to the symbols of keys[0..m) (ascending frequency):
// the rarest symbols take the longest codes.
DFL_HD inline void limit_assign(uint32_t *a, const uint32_t *keys, int m, int max_len, uint8_t *len, uint32_t *num) {
    for (int i = 0; i <= 32; ++i) num[i] = 0;
    for (int i = 0; i < m; ++i) {
        const uint32_t v = DFL_U(a[i]), k = v > 32 ? 32 : v;
        num[k] = DFL_U(num[k]) + 1;
    }
    for (int i = max_len + 1; i <= 32; ++i) { num[max_len] = DFL_U(num[max_len]) + DFL_U(num[i]); num[i] = 0; }
    uint32_t total = 0;
    for (int i = max_len; i > 0; --i) total += DFL_U(num[i]) << (max_len - i);
    while (total != (1u << max_len)) {
        num[max_len] = DFL_U(num[max_len]) - 1;
        for (int i = max_len - 1; i > 0; --i) {
            const uint32_t ni = DFL_U(num[i]);
            if (ni) { num[i] = ni - 1; num[i + 1] = DFL_U(num[i + 1]) + 2; break; }
        }
        total--;
    }
    int k = 0;
    for (int l = max_len; l >= 1; --l)
        for (uint32_t c = 0, nl = DFL_U(num[l]); c < nl; ++c) len[DFL_U(keys[k++]) & 511] = (uint8_t)l;
}

// Codes per length limited to max_len with the Kraft sum restored (num[0..32]
// from mr_counts)
DFL_HD inline void limit_num(int max_len, uint32_t *num) {
    for (int i = max_len + 1; i <= 32; ++i) { num[max_len] += num[i]; num[i] = 0; }
    uint32_t total = 0;
    for (int i = max_len; i > 0; --i) total += num[i] << (max_len - i);
    while (total != (1u << max_len)) {
        num[max_len]--;
        for (int i = max_len - 1; i > 0; --i)
            if (num[i]) { num[i]--; num[i + 1] += 2; break; }
        total--;
    }
}
// ... and the assigning half for one rank (0 = rarest symbol)
DFL_HD inline uint8_t len_of_rank(const uint32_t *num, int max_len, uint32_t r) {
    uint32_t k = 0;
    for (int l = max_len; l >= 1; --l) {
        k += num[l];
        if (r < k) return (uint8_t)l;
    }
    return 0;
}

// Code lengths <= max_len for freq[0..n) (n <= 32) into len[0..n) on one
// thread; scratch holds 2n words.  At least `min_used` symbols get a code.
DFL_HD inline void build_lengths_small(const uint32_t *freq, int n, int max_len, uint8_t *len, uint32_t *scratch,
                                       int min_used, uint32_t *num) {
    int m = 0;
    uint32_t *keys = scratch, *f = scratch + n;
    for (int i = 0; i < n; ++i) {
        len[i] = 0;
        const uint32_t fi = DFL_U(freq[i]);
        if (fi) keys[m++] = (fi << 9) | (uint32_t)i;
    }
    for (int i = 0; i < n && m < min_used; ++i)
        if (!DFL_U(freq[i])) keys[m++] = (uint32_t)i;
    if (m == 0) return;
    if (m == 1) { len[DFL_U(keys[0]) & 511] = 1; return; }
    for (int i = 1; i < m; ++i) {
        const uint32_t v = DFL_U(keys[i]);
        int j = i - 1;
        for (uint32_t kj; j >= 0 && (kj = DFL_U(keys[j])) > v; --j) keys[j + 1] = kj;
        keys[j + 1] = v;
    }
    for (int i = 0; i < m; ++i) {
        const uint32_t fk = DFL_U(keys[i]) >> 9;
        f[i] = fk ? fk : 1;
    }
    mr_lengths(f, m);
    limit_assign(f, keys, m, max_len, len, num);
}

DFL_HD inline uint32_t reverse_bits(uint32_t v, int nb) {
#if DFL_DEVICE
    return __brev(v) >> (32 - nb);
#else
    uint32_t r = 0;
    for (int i = 0; i < nb; ++i) { r = (r << 1) | (v & 1); v >>= 1; }
    return r;
#endif
}

DFL_HD inline void first_codes(const uint8_t *len, int n, uint32_t *next, uint32_t *cnt) {
    for (int l = 0; l < 16; ++l) cnt[l] = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t l = DFL_U(len[i]);
        cnt[l] = DFL_U(cnt[l]) + 1;
    }
    cnt[0] = 0;
    uint32_t c = 0;
    next[0] = 0;
    for (int l = 1; l < 16; ++l) { c = (c + DFL_U(cnt[l - 1])) << 1; next[l] = c; }
}

// canonical code of symbol i: the first code of its length + the symbols of
// that length before it (parallel over symbols)
DFL_HD inline uint16_t code_of(const uint8_t *len, int i, const uint32_t *next) {
    const int L = len[i];
    if (!L) return 0;
    uint32_t r = 0;
    for (int j = 0; j < i; ++j) r += len[j] == L;
    return (uint16_t)reverse_bits(next[L] + r, L);
}

// P3a (all lanes): symbol keys and their ranks (sorted ascending by (freq, symbol))
DFL_HD inline void p3a_keys(Shared &s, int lane) {
    if (lane == 0) { s.lit_freq[256] = 1; s.m_lit = 0; s.m_dist = 0; s.last_lit = 0; s.last_dist = 0; }   // end of block
    for (int i = lane; i < 288; i += kT) {
        const uint32_t f = (i < 286) ? (i == 256 ? 1u : s.lit_freq[i]) : 0u;
        s.key_lit[i] = f ? ((f << 9) | (uint32_t)i) : 0u;
        s.lit_len[i] = 0;
    }
    if (lane < 32) {
        const uint32_t f = lane < 30 ? s.dist_freq[lane] : 0u;
        s.key_dist[lane] = f ? ((f << 9) | (uint32_t)lane) : 0u;
        s.dist_len[lane] = 0;
    }
}
DFL_HD inline void p3b_rank(Shared &s, int lane) {
    for (int i = lane; i < 288; i += kT) {
        const uint32_t k = s.key_lit[i];
        if (!k) continue;
        uint32_t r = 0;
        for (int j = 0; j < 288; ++j) { const uint32_t o = s.key_lit[j]; r += (o != 0) & (o < k); }
        s.srt_lit[r] = k;
        s.sort_a[r] = k >> 9;
        aadd(&s.m_lit, 1);
    }
    if (lane < 32) {
        const uint32_t k = s.key_dist[lane];
        if (k) {
            uint32_t r = 0;
            for (int j = 0; j < 32; ++j) { const uint32_t o = s.key_dist[j]; r += (o != 0) & (o < k); }
            s.srt_dist[r] = k;
            s.sort_d[r] = k >> 9;
            aadd(&s.m_dist, 1);
        }
    }
}

// P3c1: the two trees at once, literal/length on lane 0 and distance on the
// first lane of the second wave: code lengths by rank, codes per length
constexpr int kDistLane = kT > 64 ? 64 : 0;
DFL_HD inline void p3c_trees(Shared &s, int lane) {
    if (serial_lane(lane, 0)) {
        const int ml = (int)DFL_U(s.m_lit);              // >= 2: a literal and end of block
        mr_counts(s.sort_a, ml, s.num_lit);
        limit_num(15, s.num_lit);
    }
    if (serial_lane(lane, kDistLane)) {
        const int md = (int)DFL_U(s.m_dist);
        if (md <= 1) {                               // one code of length 1 (unused when md == 0)
            for (int i = 0; i <= 32; ++i) s.num_dist[i] = 0;
            s.num_dist[1] = 1;
        } else {
            mr_counts(s.sort_d, md, s.num_dist);
            limit_num(15, s.num_dist);
        }
    }
}
// P3c2 (all lanes): every symbol's length from its rank (the rarest take the
// longest codes), the highest coded symbols
DFL_HD inline void p3c_assign(Shared &s, int lane) {
    const uint32_t ml = s.m_lit, md = s.m_dist;
    for (uint32_t r = (uint32_t)lane; r < ml; r += kT) {
        const uint32_t sym = s.srt_lit[r] & 511;
        s.lit_len[sym] = len_of_rank(s.num_lit, 15, r);
        amax(&s.last_lit, sym);
    }
    if (lane == 0 && md == 0) s.dist_len[0] = 1;
    if ((uint32_t)lane < md) {
        const uint32_t sym = s.srt_dist[lane] & 511;
        s.dist_len[sym] = len_of_rank(s.num_dist, 15, (uint32_t)lane);
        amax(&s.last_dist, sym);
    }
}

DFL_HD inline void first_codes_from_counts(const uint32_t *num, uint32_t *next) {
    uint32_t c = 0;
    next[0] = 0;
    for (int l = 1; l < 16; ++l) { c = (c + (l > 1 ? DFL_U(num[l - 1]) : 0)) << 1; next[l] = c; }
}

// P3c3 (one wave, serial): first codes, the run-length-coded header and its code
// the header's code-length code and its bit count, from the run-length
// symbols' counts (t0_clf) (one lane)
DFL_HD inline void p3c_header_post(Shared &s) {
    uint32_t *clf = s.t0_clf;
    build_lengths_small(clf, 19, 7, s.cl_len, s.sort_a, 2, s.t0_num);
    first_codes(s.cl_len, 19, s.next_code[2], s.t0_cnt);
    int ncl = 19;
    while (ncl > 4 && !DFL_U(s.cl_len[kClOrder[ncl - 1]])) --ncl;
    s.hclen = (uint32_t)(ncl - 4);
    uint32_t bits = 3 + 5 + 5 + 4 + 3 * (uint32_t)ncl;
    for (int k = 0; k < 19; ++k)
        bits += DFL_U(clf[k]) * (DFL_U(s.cl_len[k]) + (k == 16 ? 2u : k == 17 ? 3u : k == 18 ? 7u : 0u));
    s.hdr_bits = bits;
}

DFL_HD inline void p3c_header(Shared &s) {
    first_codes_from_counts(s.num_lit, s.next_code[0]);
    first_codes_from_counts(s.num_dist, s.next_code[1]);
    const uint32_t last_lit = DFL_U(s.last_lit);
    const int nlit = last_lit + 1 > 257 ? (int)last_lit + 1 : 257;
    const int ndist = (int)DFL_U(s.last_dist) + 1;
    s.hlit = (uint32_t)(nlit - 257);
    s.hdist = (uint32_t)(ndist - 1);
    // run-length code the lengths (symbols 16 / 17 / 18)
    const int N = nlit + ndist;
    auto L = [&](int i) -> uint32_t { return i < nlit ? DFL_U(s.lit_len[i]) : DFL_U(s.dist_len[i - nlit]); };
    uint32_t *clf = s.t0_clf;
    for (int i = 0; i < 19; ++i) clf[i] = 0;
    uint32_t nr = 0;
    uint32_t v_next = N > 0 ? L(0) : 0u;
    for (int i = 0; i < N;) {
        const uint32_t v = v_next;
        int run = 1;
        while (i + run < N && (v_next = L(i + run)) == v) ++run;
        i += run;
        if (v == 0) {
            while (run >= 11) { const int r = run < 138 ? run : 138; s.rle[nr++] = (uint16_t)(18 | ((r - 11) << 8)); clf[18] = DFL_U(clf[18]) + 1; run -= r; }
            if (run >= 3) { s.rle[nr++] = (uint16_t)(17 | ((run - 3) << 8)); clf[17] = DFL_U(clf[17]) + 1; run = 0; }
            if (run > 0) clf[0] = DFL_U(clf[0]) + (uint32_t)run;
            while (run-- > 0) s.rle[nr++] = 0;
        } else {
            s.rle[nr++] = (uint16_t)v; --run;
            uint32_t nv = 1;
            while (run >= 3) { const int r = run < 6 ? run : 6; s.rle[nr++] = (uint16_t)(16 | ((r - 3) << 8)); clf[16] = DFL_U(clf[16]) + 1; run -= r; }
            nv += run > 0 ? (uint32_t)run : 0u;
            while (run-- > 0) s.rle[nr++] = (uint16_t)v;
            clf[v] = DFL_U(clf[v]) + nv;
        }
    }
    s.n_rle = nr;
    p3c_header_post(s);
}

// P3d (all lanes): canonical codes
// the first code of length L from the counts per length (one entry of
// first_codes_from_counts)
DFL_HD inline uint32_t first_code_of(const uint32_t *num, uint32_t L) {
    uint32_t c = 0;
    for (uint32_t l = 1; l <= L; ++l) c = (c + (l > 1 ? num[l - 1] : 0)) << 1;
    return c;
}
// p3d_codes' literal/length and distance codes on lanes i0, i0 + step, ...
// (the device runs them on waves 1-3 while wave 0 builds the header)
DFL_HD inline void p3d_codes_litdist(Shared &s, int i0, int step) {
    for (int i = i0; i < 288; i += step) {
        const uint32_t L = s.lit_len[i];
        uint16_t c = 0;
        if (i < 286 && L) {
            uint32_t r = 0;
            for (int j = 0; j < i; ++j) r += s.lit_len[j] == L;
            c = (uint16_t)reverse_bits(first_code_of(s.num_lit, L) + r, (int)L);
        }
        s.lit_code[i] = c;
        s.lit_cl[i] = c | L << 16;
    }
    for (int i = i0; i < 32; i += step) {
        const uint32_t L = s.dist_len[i];
        uint16_t c = 0;
        if (i < 30 && L) {
            uint32_t r = 0;
            for (int j = 0; j < i; ++j) r += s.dist_len[j] == L;
            c = (uint16_t)reverse_bits(first_code_of(s.num_dist, L) + r, (int)L);
        }
        s.dist_code[i] = c;
        s.dist_cl[i] = c | L << 16;
    }
}
DFL_HD inline void p3d_codes(Shared &s, int lane) {
    for (int i = lane; i < 288; i += kT) {
        const uint16_t c = i < 286 ? code_of(s.lit_len, i, s.next_code[0]) : 0;
        s.lit_code[i] = c;
        s.lit_cl[i] = c | (uint32_t)s.lit_len[i] << 16;
    }
    if (lane < 32) {
        const uint16_t c = lane < 30 ? code_of(s.dist_len, lane, s.next_code[1]) : 0;
        s.dist_code[lane] = c;
        s.dist_cl[lane] = c | (uint32_t)s.dist_len[lane] << 16;
    }
    if (lane < 19) s.cl_code[lane] = code_of(s.cl_len, lane, s.next_code[2]);
}

template <class O>
DFL_HD inline void write_header(const Shared &s, O &o) {
    o.put(1, 1);          // BFINAL
    o.put(2, 2);          // BTYPE = 10 (dynamic Huffman)
    o.put(s.hlit, 5);
    o.put(s.hdist, 5);
    o.put(s.hclen, 4);
    for (uint32_t i = 0; i < s.hclen + 4; ++i) o.put(s.cl_len[kClOrder[i]], 3);
    for (uint32_t i = 0; i < s.n_rle; ++i) {
        const uint32_t sym = s.rle[i] & 31, ex = s.rle[i] >> 8;
        o.put(s.cl_code[sym], s.cl_len[sym]);
        if (sym == 16) o.put(ex, 2);
        else if (sym == 17) o.put(ex, 3);
        else if (sym == 18) o.put(ex, 7);
    }
}

// `nb` (<= 4) little-endian bytes of v at byte offset `at` (byte stores)
DFL_HD inline void put_bytes(uint32_t *w, uint32_t at, uint32_t v, int nb) {
    uint8_t *o = reinterpret_cast<uint8_t *>(w);
    for (int i = 0; i < nb; ++i) o[at + (uint32_t)i] = (uint8_t)(v >> (8 * i));
}

// gzip member header with the BGZF extra field: 1f 8b 08 04 | mtime 0 |
// xfl 0 | os ff | xlen 6 | 'B' 'C' 2 0 | BSIZE (member bytes - 1)
template <class O>
DFL_HD inline void put_gzip_header(O &o, uint32_t bsize) {
    o.put(0x04088b1fu, 32);
    o.put(0, 32);
    o.put(0xff00u, 16);
    o.put(6, 16);
    o.put(0x00024342u, 32);
    o.put(bsize, 16);
}

// ---- the phases (lane = thread index) -----------------------------------------
// stored-or-compressed decision once the bits are known (any one lane)
DFL_HD inline void decide(Shared &s, uint32_t n, uint32_t end_bits) {
    s.body_bits = end_bits - 144 + s.lit_len[256];
    const uint32_t dbytes = (s.body_bits + 7) / 8;
    s.stored = (dbytes > kMaxDeflate || dbytes > n + 5) ? 1u : 0u;
    s.use_stage = (!s.stored && dbytes + 26 <= sizeof(s.stage)) ? 1u : 0u;
}

DFL_HD inline void p0_clear(Shared &s, int lane) {
    for (int i = lane; i < kHN; i += kT) { s.a_min[i] = kNone; s.b_min[i] = kNone; s.a_max[i] = 0; }
    for (int i = lane; i < 288; i += kT) s.lit_freq[i] = 0;
    if (lane < 32) s.dist_freq[lane] = 0;
    if (lane == 0) s.extra_bits = 0;
}
DFL_HD inline void p1_hash(Shared &s, uint32_t n, int lane) {
    uint32_t lo, hi;
    lane_range(n, lane, lo, hi);
#if DFL_DEVICE && DFL_P1W
    // a dword at a time: each input dword loaded once (the next one ahead),
    // its four positions' bytes by funnel shifts
    {
        const uint32_t *wi = reinterpret_cast<const uint32_t *>(s.in);
        const uint32_t end = hi < (n >= 3 ? n - 3 : 0) ? hi : (n >= 3 ? n - 3 : 0);   // p + 4 <= n
        uint32_t d = lo >> 2;
        uint32_t A = wi[d], B = wi[d + 1];
        for (uint32_t p0 = lo & ~3u; p0 < end; p0 += 4) {
            const uint32_t C = wi[d + 2];
DFL_UNROLL
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t p = p0 + k;
                if (p < lo || p >= end) continue;
                const uint32_t h = hash4(k ? __builtin_amdgcn_alignbyte(B, A, k) : A);
                if (p < 32768) { amin(&s.a_min[h], p); amax(&s.a_max[h], p + 1); }
                else amin(&s.b_min[h], p);
            }
            A = B;
            B = C;
            ++d;
        }
        return;
    }
#endif
    for (uint32_t p = lo; p < hi && p + 4 <= n; ++p) {
        const uint32_t h = hash4(ld32(s, p));
        if (p < 32768) { amin(&s.a_min[h], p); amax(&s.a_max[h], p + 1); }
        else amin(&s.b_min[h], p);
    }
}
DFL_HD inline uint32_t sub_crc(const Shared &s, uint32_t n, int l);
DFL_HD inline void p2_count(Shared &s, uint32_t n, int lane, uint32_t *tok) {
    uint32_t lo, hi;
    lane_range(n, lane, lo, hi);
#ifdef DFL_ABL_NOCNT
    CountTokV v{CountV{s, 0, lane}, TokV{tok, lane}};
#else
    CountTokV v{CountV{s}, TokV{tok, lane}};
#endif
    parse(s, n, lane, lo, hi, v);
    v.t.finish();
    if (v.c.extra) aadd(&s.extra_bits, v.c.extra);
#if !(DFL_DEVICE && DFL_CRC_LATE)
    s.lane_crc[lane] = sub_crc(s, n, lane);
#endif
}

// CRC32 register of sub-block l (no init / final xor), shifted past the rest
// of the block.  On the device it runs during the code-length phase, on the
// two waves that phase leaves idle (k_deflate, DFL_CRC_LATE).
DFL_HD inline uint32_t sub_crc(const Shared &s, uint32_t n, int l) {
    uint32_t lo, hi;
    lane_range(n, l, lo, hi);
    uint32_t c = 0;
#if defined(DFL_ABL_NOCRC)
    (void)c;
#elif DFL_DEVICE && DFL_CRCS
    // slice-by-N: N independent table loads per N / 4 dwords
    uint32_t p = lo;
    for (; p < hi && (p & 3); ++p) c = s.crc_t[0][(c ^ s.in[p]) & 0xff] ^ (c >> 8);
    const uint32_t *wi = reinterpret_cast<const uint32_t *>(s.in);
    for (; p + DFL_CRCS <= hi; p += DFL_CRCS) {
        const uint32_t a = c ^ wi[p >> 2];
#if DFL_CRCS == 8
        const uint32_t b = wi[(p >> 2) + 1];
        c = s.crc_t[7][a & 255] ^ s.crc_t[6][(a >> 8) & 255] ^ s.crc_t[5][(a >> 16) & 255] ^ s.crc_t[4][a >> 24] ^
            s.crc_t[3][b & 255] ^ s.crc_t[2][(b >> 8) & 255] ^ s.crc_t[1][(b >> 16) & 255] ^ s.crc_t[0][b >> 24];
#else
        c = s.crc_t[3][a & 255] ^ s.crc_t[2][(a >> 8) & 255] ^ s.crc_t[1][(a >> 16) & 255] ^ s.crc_t[0][a >> 24];
#endif
    }
    for (; p < hi; ++p) c = s.crc_t[0][(c ^ s.in[p]) & 0xff] ^ (c >> 8);
#else
    for (uint32_t p = lo; p < hi; ++p) c = crc_byte((c ^ s.in[p]) & 0xff) ^ (c >> 8);
#endif
    return (hi > lo) ? multmodp(x8nmodp(n - hi), c) : 0;
}
DFL_HD inline void p4_bits(Shared &s, uint32_t n, int lane, const uint32_t *tok) {
    uint32_t lo, hi;
    lane_range(n, lane, lo, hi);
    BitsV v{s};
    replay(s, tok, lane, lo, v);
    s.lane_bits[lane] = v.bits;
}
// between P4 and P5, sequential form (the host emulation; the kernel runs
// the same scan across the workgroup): bit offsets (deflate data begins at
// byte 18 of the member), stored decision, CRC; zeroes the words two lanes
// share, in both possible destinations (stage[] and the global slot)
DFL_HD inline void p4_scan(Shared &s, uint32_t n, uint32_t *out) {
    uint32_t acc = 3 * 8 * 6 + s.hdr_bits;
    for (int l = 0; l < kT; ++l) {
        s.lane_off[l] = acc;
        if (l && (acc & 31)) {
            out[acc >> 5] = 0;
            if ((acc >> 5) < sizeof(s.stage) / 4) s.stage[acc >> 5] = 0;
        }
        acc += s.lane_bits[l];
    }
    decide(s, n, acc);
    uint32_t c = multmodp(x8nmodp(n), 0xffffffffu);
    for (int l = 0; l < kT; ++l) c ^= s.lane_crc[l];
    s.crc = ~c;
}
// P5: into stage[] when use_stage (copied out by p6_copy), else into out.
// Two inlined copies, so that the LDS one writes with LDS instructions (one
// pointer that may be either is a flat pointer).
#if DFL_DEVICE
#define DFL_INLINE __attribute__((always_inline)) inline
#else
#define DFL_INLINE inline
#endif
template <bool kStage>
DFL_HD inline typename std::conditional<kStage, BitOut2, BitOut>::type make_out(uint32_t *w, uint32_t bitpos, bool own_last,
                                                                              uint32_t *dummy);
template <>
DFL_HD inline BitOut2 make_out<true>(uint32_t *w, uint32_t bitpos, bool own_last, uint32_t *dummy) {
    return BitOut2(w, bitpos, own_last, dummy);
}
template <>
DFL_HD inline BitOut make_out<false>(uint32_t *w, uint32_t bitpos, bool own_last, uint32_t *) {
    return BitOut(w, bitpos, own_last);
}
template <bool kStage>
DFL_HD DFL_INLINE void p5_emit_to(Shared &s, uint32_t n, int lane, const uint32_t *tok, uint32_t *out);
DFL_HD inline void p5_emit(Shared &s, uint32_t n, int lane, const uint32_t *tok, uint32_t *out) {
    if (s.use_stage) p5_emit_to<true>(s, n, lane, tok, s.stage);
    else p5_emit_to<false>(s, n, lane, tok, out);
}
template <bool kStage>
DFL_HD DFL_INLINE void p5_emit_to(Shared &s, uint32_t n, int lane, const uint32_t *tok, uint32_t *out) {
    uint32_t lo, hi;
    lane_range(n, lane, lo, hi);
    if (s.stored) {
        // stored block: BFINAL=1 BTYPE=00, LEN, NLEN, raw bytes (byte-aligned after the 3 bits)
        uint8_t *o = reinterpret_cast<uint8_t *>(out) + 18 + 5;
        for (uint32_t p = lo; p < hi; ++p) o[p] = s.in[p];
        return;
    }
    // the member in stage[] (LDS, nearly always): BitOut2 (its throwaway
    // word the lane's lane_bits entry, read before P5); else BitOut
    using O = typename std::conditional<kStage, BitOut2, BitOut>::type;
    using V = typename std::conditional<kStage, EmitV2, EmitV>::type;
    O o = make_out<kStage>(out, lane == 0 ? 0 : s.lane_off[lane], lane == kT - 1, &s.lane_bits[lane]);
    if (lane == 0) {
        put_gzip_header(o, (s.body_bits + 7) / 8 + 25);
        write_header(s, o);
    }
    V v{s, o};
    replay(s, tok, lane, lo, v);
    if (lane == kT - 1) {
        o.put(s.lit_code[256], s.lit_len[256]);
        o.put(0, (8 - (o.pos() & 7)) & 7);
        o.put(s.crc, 32);
        o.put(n, 32);
    }
    o.flush();
}
// after P5 (all lanes): a member assembled in stage[] to the slot, one
// coalesced word per lane per step
DFL_HD inline void p6_copy(const Shared &s, int lane, uint32_t *out) {
    if (!s.use_stage) return;
    const uint32_t words = ((s.body_bits + 7) / 8 + 26 + 3) / 4;
    for (uint32_t i = (uint32_t)lane; i < words; i += kT) out[i] = s.stage[i];
}

// thread 0 after P5: the member size; a stored block's framing
DFL_HD inline uint32_t p6_frame(const Shared &s, uint32_t n, uint32_t *out) {
    if (!s.stored) return (s.body_bits + 7) / 8 + 26;
    const uint32_t dbytes = 5 + n;
    put_bytes(out, 0, 0x04088b1fu, 4);
    put_bytes(out, 4, 0, 4);
    put_bytes(out, 8, 0xff00u, 2);
    put_bytes(out, 10, 6, 2);
    put_bytes(out, 12, 0x00024342u, 4);
    put_bytes(out, 16, dbytes + 25, 2);
    put_bytes(out, 18, 1, 1);
    put_bytes(out, 19, n, 2);
    put_bytes(out, 21, ~n & 0xffff, 2);
    put_bytes(out, 18 + dbytes, s.crc, 4);
    put_bytes(out, 22 + dbytes, n, 4);
    return dbytes + 26;
}

}  // namespace dfl
