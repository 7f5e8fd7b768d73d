// dcr_ingest.cpp — native BAM ingest (include/dcr_io.h): BGZF inflate on a
// worker pool, record walk, the reference's read filters, MI grouping,
// family checks, the four-way split and check_number_reads' random.sample
// (CPython's MT19937, bit for bit), and packing of processed families into
// the dcr_batch layout the GPU consumes.
//
// Per batch the work splits into a serial walk (record boundaries, filters,
// grouping, RNG; a few loads per record) and parallel parts (inflate of the
// next window of BGZF blocks; per-read copies of sequence / qualities /
// CIGAR into the caller's pinned arrays, queued by the walk as jobs).
//
// Reference: /root/reference/DuplexUMIConsensusReads.py (":line" below).
#include <zlib.h>
#include <tmmintrin.h>
#include <sys/stat.h>

#include <cctype>
#include <cmath>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/dcr_io.h"
#include "../../include/dcr_inflate.h"
#include "dcr_host.h"

using namespace dcrh;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &m) {
    g_err = m;
    return code;
}

struct TLDecomp {
    libdeflate_decompressor *d = nullptr;
    ~TLDecomp() {
        if (d) libdeflate_free_decompressor(d);
    }
    libdeflate_decompressor *get() {
        if (!d) d = libdeflate_alloc_decompressor();
        return d;
    }
};
thread_local TLDecomp tl_dec;

// ---------------------------------------------------------------------------
// CPython's random.Random (Modules/_randommodule.c genrand_uint32, getrandbits
// for k <= 32; Lib/random.py 3.10 _randbelow_with_getrandbits and sample)
struct PyRandom {
    uint32_t mt[624];
    int index = 625;
    bool seeded = false;

    uint32_t genrand() {
        static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
        const int N = 624, M = 397;
        uint32_t y;
        if (index >= N) {
            int kk;
            for (kk = 0; kk < N - M; kk++) {
                y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + M] ^ (y >> 1) ^ mag01[y & 1u];
            }
            for (; kk < N - 1; kk++) {
                y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
                mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1u];
            }
            y = (mt[N - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
            mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ mag01[y & 1u];
            index = 0;
        }
        y = mt[index++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    static int bit_length(uint32_t n) {
        int k = 0;
        while (n) { ++k; n >>= 1; }
        return k;
    }
    uint32_t randbelow(uint32_t n) {
        if (!n) return 0;
        const int k = bit_length(n);   // n < 2^31 here, so k <= 31
        uint32_t r = genrand() >> (32 - k);
        while (r >= n) r = genrand() >> (32 - k);
        return r;
    }
    // random.sample(range(n), k) -> indices in selection order
    void sample(int n, int k, std::vector<int> &out) {
        out.assign((size_t)k, 0);
        long setsize = 21;
        if (k > 5) setsize += (long)std::pow(4.0, std::ceil(std::log((double)k * 3) / std::log(4.0)));
        if (n <= setsize) {
            std::vector<int> pool((size_t)n);
            for (int i = 0; i < n; ++i) pool[(size_t)i] = i;
            for (int i = 0; i < k; ++i) {
                const int j = (int)randbelow((uint32_t)(n - i));
                out[(size_t)i] = pool[(size_t)j];
                pool[(size_t)j] = pool[(size_t)(n - i - 1)];
            }
        } else {
            std::vector<char> sel((size_t)n, 0);
            for (int i = 0; i < k; ++i) {
                int j = (int)randbelow((uint32_t)n);
                while (sel[(size_t)j]) j = (int)randbelow((uint32_t)n);
                sel[(size_t)j] = 1;
                out[(size_t)i] = j;
            }
        }
    }
};

// 4-bit BAM sequence code pairs -> two ASCII bases ("=ACMGRSVTWYHKDBN")
struct SeqTable {
    uint16_t pair[256];
    SeqTable() {
        const char *a = "=ACMGRSVTWYHKDBN";
        for (int b = 0; b < 256; ++b) pair[b] = (uint16_t)((uint8_t)a[b >> 4] | ((uint8_t)a[b & 15] << 8));
    }
};
const SeqTable kSeq;

// 4-bit BAM sequence -> ASCII letters: 16 packed bytes (32 bases) per step
// with two byte shuffles of the 16-letter table (SSSE3, in x86-64-v2), the
// tail by the pair table.  Part of the pack copy, which runs on the pool for
// every read of a batch.
inline void decode_seq(const uint8_t *s, int32_t l_seq, uint8_t *d) {
    const int32_t half = l_seq >> 1;
    int32_t i = 0;
    const __m128i tab = _mm_loadu_si128((const __m128i *)"=ACMGRSVTWYHKDBN");
    const __m128i m = _mm_set1_epi8(15);
    for (; i + 16 <= half; i += 16) {
        const __m128i v = _mm_loadu_si128((const __m128i *)(s + i));
        const __m128i hi = _mm_shuffle_epi8(tab, _mm_and_si128(_mm_srli_epi16(v, 4), m));
        const __m128i lo = _mm_shuffle_epi8(tab, _mm_and_si128(v, m));
        _mm_storeu_si128((__m128i *)(d + 2 * i), _mm_unpacklo_epi8(hi, lo));
        _mm_storeu_si128((__m128i *)(d + 2 * i + 16), _mm_unpackhi_epi8(hi, lo));
    }
    for (; i < half; ++i) std::memcpy(d + 2 * i, &kSeq.pair[s[i]], 2);
    if (l_seq & 1) d[l_seq - 1] = (uint8_t)(kSeq.pair[s[half]] & 0xff);
}

// One parsed record (offsets relative to the window start)
struct Rec {
    size_t off;         // offset of block_size
    uint32_t len;       // 4 + block_size
    int32_t tid, pos;
    uint16_t flag, n_cig;
    uint8_t mapq;
    int32_t l_seq;
    uint32_t o_cig, o_seq, o_qual;   // offsets of the fields from off
    uint32_t o_mi, o_rx;             // offsets of the MI / RX string values (0: absent)
    uint16_t l_mi, l_rx;             // string lengths
    uint8_t mi_type, rx_type;        // tag type codes ('Z' expected)
    uint16_t l_code;                 // MI prefix before the first '/'
    int8_t pf;                       // pass_filters: 1 pass, 0 excluded, -1 the reference stops
    uint8_t fmsg;                    // which stop (kFilterMsg)
    uint8_t perr;                    // malformed record (kParseErr), 0 ok
    uint8_t eqx;                     // CIGAR still holds '=' / 'X' after the trim (:374-375)
    int8_t subk;                     // split_family subfamily (:132-154): A1 B1 A2 B2 = 0..3, -1 none
    int64_t end_kept;                // pos + length after clip removal (the T bound)
    char code[24];                   // the MI prefix, when l_code <= 24 (else read from the window)
};

const char *const kParseErr[] = {"", "malformed BAM record (l_seq < 0)",
                                 "malformed BAM record (fields past block_size)",
                                 "malformed BAM aux field (unterminated string)", "malformed BAM aux array",
                                 "malformed BAM aux field type", "malformed BAM aux field (past block_size)"};
struct FilterMsg { int kind; const char *msg; };
const FilterMsg kFilterMsg[] = {
    {0, ""},
    {DCR_ERR_EXIT, "ERROR: family code tag (MI) not found in file"},
    {DCR_ERR_EXIT, "ERROR: family code tag (RX) not found in file"},
    {DCR_ERR_TYPE, "argument of type 'NoneType' is not iterable"},
    {DCR_ERR_EXIT, "ERROR: unexpected symbols (P, N, B, *) were found in CIGAR strings."},
    {DCR_ERR_EXIT, "ERROR: softclips (S) found in the middle of the read."}};

struct Job {
    size_t rec;         // window offset of the record
    int64_t dst_base;
    int64_t dst_cig;
    int32_t read;       // batch read index: the per-read fields are written by the copy job
};

}  // namespace

// The per-record parse (fields, aux MI / RX, the reference's filters, clip
// bound, '=' / 'X' outcome, subfamily): runs on the scanner's pool ahead of
// the walk, or on the ingest pool for records the scanner did not index.
struct RecParser {
    int min_map_quality = 0, min_base_quality = 0;
    const uint8_t *at(const uint8_t *wb, const Rec &r, uint32_t o) const { return wb + r.off + o; }

    // -- record parse ------------------------------------------------------------
    // the fields of the whole record at window offset off (0 ok, else kParseErr)
    int parse_at(const uint8_t *wb, size_t off, Rec &rc) const {
        const uint8_t *base = wb + off;
        const uint8_t *r = base + 4;
        rc.off = off;
        rc.len = 4u + (uint32_t)rdi32(base);
        rc.tid = rdi32(r);
        rc.pos = rdi32(r + 4);
        const uint32_t l_rn = r[8];
        rc.mapq = r[9];
        rc.n_cig = rd16(r + 12);
        rc.flag = rd16(r + 14);
        rc.l_seq = rdi32(r + 16);
        rc.perr = 0;
        if (rc.l_seq < 0) return 1;
        rc.o_cig = 4 + 32 + l_rn;
        rc.o_seq = rc.o_cig + 4u * rc.n_cig;
        rc.o_qual = rc.o_seq + (uint32_t)((rc.l_seq + 1) >> 1);
        size_t p = rc.o_qual + (size_t)rc.l_seq;
        if (p > rc.len) return 2;
        rc.o_mi = rc.o_rx = 0;
        rc.l_mi = rc.l_rx = 0;
        rc.mi_type = rc.rx_type = 0;
        // aux fields
        while (p + 3 <= rc.len) {
            const uint8_t t0 = base[p], t1 = base[p + 1], ty = base[p + 2];
            size_t v = p + 3, e;
            switch (ty) {
                case 'A': case 'c': case 'C': e = v + 1; break;
                case 's': case 'S': e = v + 2; break;
                case 'i': case 'I': case 'f': e = v + 4; break;
                case 'd': e = v + 8; break;
                case 'Z': case 'H': {
                    const void *z = std::memchr(base + v, 0, rc.len - v);
                    if (!z) return 3;
                    e = (size_t)((const uint8_t *)z - base) + 1;
                    break;
                }
                case 'B': {
                    if (v + 5 > rc.len) return 4;
                    const uint8_t sub = base[v];
                    const uint32_t n = rd32(base + v + 1);
                    size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                    e = v + 5 + es * (size_t)n;
                    break;
                }
                default: return 5;
            }
            if (e > rc.len) return 6;
            // the first occurrence, as pysam's get_tag (bam_aux_get)
            if (t0 == 'M' && t1 == 'I' && !rc.mi_type) {
                rc.mi_type = ty;
                rc.o_mi = (uint32_t)v;
                rc.l_mi = (uint16_t)(ty == 'Z' ? e - v - 1 : 0);
            } else if (t0 == 'R' && t1 == 'X' && !rc.rx_type) {
                rc.rx_type = ty;
                rc.o_rx = (uint32_t)v;
                rc.l_rx = (uint16_t)(ty == 'Z' ? e - v - 1 : 0);
            }
            p = e;
        }
        rc.l_code = rc.l_mi;
        if (rc.mi_type == 'Z') {
            const void *sl = std::memchr(base + rc.o_mi, '/', rc.l_mi);
            if (sl) rc.l_code = (uint16_t)((const uint8_t *)sl - (base + rc.o_mi));
        }
        // inline copies, zero-padded: the walk compares them as whole words
        std::memset(rc.code, 0, sizeof rc.code);
        if (rc.mi_type == 'Z' && rc.l_code <= sizeof rc.code) std::memcpy(rc.code, base + rc.o_mi, rc.l_code);
        int msg = 0;
        rc.pf = (int8_t)filters(wb, rc, msg);
        rc.fmsg = (uint8_t)msg;
        rc.end_kept = (int64_t)rc.pos + rc.l_seq - clip_total(wb, rc);
        {
            const bool rev = rc.flag & 16, r1 = rc.flag & 64, r2 = rc.flag & 128;
            rc.subk = (int8_t)((!rev && r1) ? 0 : (!rev && r2) ? 1 : (rev && r1) ? 2 : (rev && r2) ? 3 : -1);
        }
        rc.eqx = rc.pf == 1 && eqx_after_trim(wb, rc);
        return 0;
    }

    // pass_filters (:1135-1181): 1 pass, 0 excluded, -1 the reference stops (err set)
    int filters(const uint8_t *wb, const Rec &r, int &msg) const {
        if (!r.mi_type) { msg = 1; return -1; }
        if (!r.rx_type) { msg = 2; return -1; }
        if (r.n_cig == 0) { msg = 3; return -1; }
        const uint8_t *c = at(wb, r, r.o_cig);
        for (uint32_t i = 0; i < r.n_cig; ++i) {
            const uint32_t op = rd32(c + 4 * i) & 15;
            if (op == 3 || op == 6 || op >= 9) { msg = 4; return -1; }
        }
        for (uint32_t i = 1; i + 1 < r.n_cig; ++i)
            if ((rd32(c + 4 * i) & 15) == 4) { msg = 5; return -1; }
        const uint16_t fl = r.flag;
        return (fl & 1) && (fl & 2) && !(fl & 4) && !(fl & 8) && !(fl & 2048) && !(fl & 512) &&
               (int)r.mapq >= min_map_quality;
    }

    // end soft clips of a read (batch.py _end_soft_clips; remove_clipping :214-226)
    int32_t clip_total(const uint8_t *wb, const Rec &r) const {
        const uint8_t *c = at(wb, r, r.o_cig);
        const int n = r.n_cig;
        if (n == 0) return 0;
        auto op = [&](int i) { return (int)(rd32(c + 4 * i) & 15); };
        auto ln = [&](int i) { return (int32_t)(rd32(c + 4 * i) >> 4); };
        const int first = 0, last = n - 1;
        int32_t c5 = 0;
        if (op(first) == 4) c5 = ln(first);
        else if (op(first) == 5 && n > 1 && op(first + 1) == 4) c5 = ln(first + 1);
        const int i5 = op(first) == 4 ? first : first + 1;
        int c3i = -1;
        if (op(last) == 4) c3i = last;
        else if (op(last) == 5 && n > 1) c3i = last - 1;
        int32_t c3 = 0;
        if (c3i >= first && op(c3i) == 4 && !(c5 > 0 && c3i == i5)) c3 = ln(c3i);
        return c5 + c3;
    }

    // does the read's CIGAR, after remove_clipping and trim_3prime_N, still
    // hold a '=' / 'X' op (change_match_mismatch_operations prints, :374-375)?
    bool eqx_after_trim(const uint8_t *wb, const Rec &r) const {
        const uint8_t *c = at(wb, r, r.o_cig);
        bool any = false;
        for (uint32_t i = 0; i < r.n_cig; ++i) {
            const uint32_t op = rd32(c + 4 * i) & 15;
            any |= (op == 7 || op == 8);
        }
        if (!any || r.l_seq == 0) return false;
        // remove_clipping: S bases leave the sequence (:214-251)
        int32_t s5 = 0, s3 = 0;
        bool inseq = false, modified = false;
        int64_t expanded = 0;
        for (uint32_t i = 0; i < r.n_cig; ++i) {
            const uint32_t w = rd32(c + 4 * i), op = w & 15, ln = w >> 4;
            if (op == 5) modified = true;
            else if (op == 4) {
                modified = true;
                if (!inseq) s5 = (int32_t)ln; else s3 = (int32_t)ln;
            } else {
                inseq = true;
                expanded += ln;
            }
        }
        (void)modified;
        int32_t b = s5, e = r.l_seq - s3;       // seq[s5 : -s3] (s3 > 0) or seq[s5:]
        if (s3 == 0) e = r.l_seq;
        if (e < b) e = b;
        // mask (:279-283) then count the trailing 'N' (:306-312)
        const uint8_t *sq = at(wb, r, r.o_seq), *ql = at(wb, r, r.o_qual);
        int32_t tn = 0;
        for (int32_t i = e - 1; i >= b; --i) {
            const int code = (sq[i >> 1] >> ((i & 1) ? 0 : 4)) & 15;
            if (code == 15 || (int)ql[i] < min_base_quality) ++tn;
            else break;
        }
        // original_cigar[:len - tn] with Python slice semantics (:320-322)
        int64_t keep = expanded - tn;
        if (keep < 0) keep = std::max<int64_t>(0, expanded + keep);
        int64_t pos = 0;
        for (uint32_t i = 0; i < r.n_cig && pos < keep; ++i) {
            const uint32_t w = rd32(c + 4 * i), op = w & 15, ln = w >> 4;
            if (op == 4 || op == 5) continue;
            if (op == 7 || op == 8) return true;
            pos += ln;
        }
        return false;
    }

};

// Background BGZF inflate and record index, two pipeline stages ahead of the
// record walk:
//   inflate thread  reads the file and inflates ~32 MiB runs of whole blocks
//                   (on its own worker pool) into a chunk;
//   scanner thread  follows the block_size chain through the chunk (the BAM
//                   header first) and parses every record that starts and
//                   ends inside it (on a second pool), so the walk gets
//                   parsed records and does no pointer chasing of its own.
// Each chunk keeps headroom in front of its data so the walk can put the
// bytes it still needs (the open family, a record straddling the chunk
// boundary) right before the new data without moving it: record offsets are
// then the same in the chunk buffer and in the walk's window.  On anything
// unexpected the scanner stops indexing and the walk's own serial scan (with
// its error messages) takes over.
struct Chunk {
    HugeBuf buf;                    // [kHead headroom][len inflated bytes]
    uint8_t *pin = nullptr;         // the same, page-locked (GPU inflate), instead of buf
    uint8_t *data() { return pin ? pin : buf.data(); }
    size_t len = 0;
    bool eof = false;               // nothing follows this chunk
    std::string err;
    bool indexed = false;           // recs holds every record starting after the first
    std::vector<Rec> recs;          // boundary in this chunk and ending in it (off from buf start)
    std::vector<size_t> offs;       // the chain's record starts (parse stage input)
    bool chained = false;           // the chain walked this chunk (its offs are valid)
};

// Record-index vectors of released chunks, kept for the next ingest of the
// process (as HugeCache keeps the chunk buffers): freeing four ~13 MB vectors
// per ingest unmapped their pages inside every CLI pass (~18 ms of a close)
class RecsCache {
  public:
    static RecsCache &get() {
        static RecsCache c;
        return c;
    }
    std::vector<Rec> take() {
        std::lock_guard<std::mutex> g(mu_);
        if (spare_.empty()) return {};
        std::vector<Rec> v = std::move(spare_.back());
        spare_.pop_back();
        return v;
    }
    void give(std::vector<Rec> &&v) {
        std::lock_guard<std::mutex> g(mu_);
        if (spare_.size() >= 16 || v.capacity() == 0) return;
        v.clear();                          // keeps the capacity
        spare_.push_back(std::move(v));
    }

  private:
    std::mutex mu_;
    std::vector<std::vector<Rec>> spare_;
};

// Thread pools of closed ingests, kept for the next ones of the process: a
// pool's threads are joined when it is destroyed, and on a loaded machine
// their wake-ups made an ingest's close take 6-14 ms per pool (measured; the
// CLI closes an ingest per pass).  A pool is handed to one ingest at a time.
class PoolCache {
  public:
    static PoolCache &get() {
        static PoolCache *c = new PoolCache;     // never destroyed: its threads end with the process
        return *c;
    }
    std::unique_ptr<Pool> take(int n) {
        {
            std::lock_guard<std::mutex> g(mu_);
            for (size_t i = 0; i < spare_.size(); ++i)
                if (spare_[i]->size() == std::max(1, n)) {
                    std::unique_ptr<Pool> p = std::move(spare_[i]);
                    spare_.erase(spare_.begin() + (long)i);
                    return p;
                }
        }
        return std::unique_ptr<Pool>(new Pool(n));
    }
    void give(std::unique_ptr<Pool> p) {
        if (!p) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (spare_.size() < 16) {
                spare_.push_back(std::move(p));
                return;
            }
        }
        p.reset();                                // more than enough kept: this one joins its threads
    }

  private:
    std::mutex mu_;
    std::vector<std::unique_ptr<Pool>> spare_;
};

// the GPU inflate hook (dcr_io_set_inflate_hook), copied by each Inflater
std::mutex g_hook_mu;
dcr_inflate_hook g_hook{};
bool g_hook_set = false;

// override of a pool's size (A/B runs): the variable's value if set and positive
inline int env_threads(const char *name, int dflt) {
    const char *v = std::getenv(name);
    const int n = v ? std::atoi(v) : 0;
    return n > 0 ? std::min(n, 64) : dflt;
}

class Inflater {
  public:
    static constexpr size_t kHead = (size_t)8 << 20;
    static constexpr size_t kWant = (size_t)32 << 20;
#ifndef DCR_WANT_GPU_MIB
#define DCR_WANT_GPU_MIB 64   // A/B builds only
#endif
    static constexpr size_t kWantGpu = (size_t)DCR_WANT_GPU_MIB << 20;

    // ranged: start at the BGZF block at file offset start_coff, start_uoff
    // bytes into its data, on a record boundary (no header); end_coff >= 0:
    // stop end_uoff bytes into the data of the block at end_coff
    Inflater(FILE *f, int n_threads, const RecParser &rp, bool ranged = false, uint64_t start_coff = 0,
             uint32_t start_uoff = 0, int64_t end_coff = -1, uint32_t end_uoff = 0, bool host_only = false)
        : f_(f), pool_(PoolCache::get().take(env_threads("DCR_INFLATE_THREADS", n_threads))),
          spool_(PoolCache::get().take(env_threads("DCR_SCAN_THREADS", std::max(1, n_threads / 2)))), rp_(rp),
          end_coff_(end_coff),
          end_uoff_(end_uoff) {
        for (auto &c : chunks_) c.recs = RecsCache::get().take();
        if (ranged) {
            st_ = kRec;
            skip_ = start_uoff;
        }
        // A regular file is mapped whole: the blocks inflate straight from the
        // page cache, with no serial fread copy on this thread in front of the
        // pool (48 MiB before the first chunk could start, ~0.1 s per 0.5 GB
        // file), and the workers fault their own pages in parallel.  Anything
        // else (a pipe) streams through cbuf_.
        struct stat sb;
        const int fd = fileno(f_);
        if (fd >= 0 && fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode) && sb.st_size > 0) {
            void *p = mmap(nullptr, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
            if (p != MAP_FAILED) {
                map_ = (const uint8_t *)p;
                map_len_ = (size_t)sb.st_size;
                cbeg_ = ranged ? (size_t)std::min<uint64_t>(start_coff, map_len_) : 0;
                cend_ = map_len_;
                file_eof_ = true;
            }
        }
        if (!map_) {
            if (ranged) {
                std::fseek(f_, (long)start_coff, SEEK_SET);
                cpos_ = start_coff;
            }
            cbuf_.resize((size_t)48 << 20);
        }
        {
            std::lock_guard<std::mutex> g(g_hook_mu);
            const char *e = std::getenv("DCR_GPU_INFLATE");
            if (g_hook_set && !host_only && !(e && std::strcmp(e, "0") == 0)) {
                hook_ = g_hook;
                gpu_ = true;
            }
        }
        // GPU inflate: larger chunks (a launch needs ~1,000 members to fill the device)
        want_max_ = gpu_ ? kWantGpu : kWant;
        for (auto &c : chunks_) {
            if (gpu_ && hook_.host_alloc) c.pin = (uint8_t *)hook_.host_alloc(hook_.user, kHead + want_max_ + 0x10000);
            if (!c.pin) c.buf.resize(kHead + want_max_ + 0x10000);
            empty_.push_back(&c);
        }
        if (const char *he = std::getenv("DCR_HOST_CHUNK_EVERY")) host_every_ = std::max(0, std::atoi(he));
        if (gpu_ && map_ && hook_.stream_open) open_stream();
        if (gpu_ && !stream_) {
            stage_cap_ = want_max_ + ((size_t)1 << 20);
            if (hook_.host_alloc) stage_pin_ = (uint8_t *)hook_.host_alloc(hook_.user, stage_cap_);
            if (!stage_pin_) stage_.resize(stage_cap_);
        }
        th_ = std::thread([this] { loop(); });
        sth_ = std::thread([this] { scan_loop(); });
        pth_ = std::thread([this] { parse_loop(); });
    }
    ~Inflater() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
        sth_.join();
        pth_.join();
        stop_members_ = true;
        if (mth_.joinable()) mth_.join();
        if (stream_) hook_.stream_close(stream_);          // before the mapping it reads goes away
        // unmapping a whole input (page-table teardown, ~25 ms per 0.5 GB)
        // need not hold up the caller: a detached thread does it, 16 MiB at
        // a time, so it never holds the address-space lock for long (frees
        // and the next open's mmap would otherwise wait for all of it)
        if (map_) {
            uint8_t *p = (uint8_t *)map_;
            const size_t len = map_len_;
            std::thread([p, len] {
                constexpr size_t kSlice = (size_t)16 << 20;
                for (size_t o = 0; o < len; o += kSlice) munmap(p + o, std::min(kSlice, len - o));
            }).detach();
        }
        if (hook_.host_free) {
            for (auto &c : chunks_)
                if (c.pin) hook_.host_free(hook_.user, c.pin);
            if (stage_pin_) hook_.host_free(hook_.user, stage_pin_);
        }
        for (auto &c : chunks_) RecsCache::get().give(std::move(c.recs));
        PoolCache::get().give(std::move(pool_));
        PoolCache::get().give(std::move(spool_));
    }
    bool gpu() const { return gpu_; }

    // A mapped input's members for the device inflater's stream
    // (dcr_inflate_hook.stream_*): a helper thread walks the BGZF headers
    // (the walk fill() makes chunk by chunk) and appends them in batches, the
    // first small so the first launch starts at once.  On anything
    // unexpected it stops appending; fill()'s own walk then reports it.
    // Called before th_ starts: the walk's start offset is read here, on the
    // constructing thread, never by mth_ (fill() on th_ advances cbeg_; a
    // late-scheduled mth_ would start the stream at a later member, shifting
    // every fetch while each member's CRC still passed).
    void open_stream() {
        stream_ = hook_.stream_open(hook_.user, map_);
        if (!stream_) return;
        stream_out_ = 0;
        const size_t p0 = cbeg_, p_end = cend_;
        mth_ = std::thread([this, p0, p_end] { scan_members(p0, p_end); });
    }
    // Chunks the host pool inflates beside the device stream (every
    // host_every_-th, DCR_HOST_CHUNK_EVERY; 0: none): the stream skips their
    // members, fill() inflates them with libdeflate.  Chunk k is the k-th
    // fill(); its blocks follow fill()'s rule (whole blocks while the
    // chunk's output + 64 KiB fits want_: 4 MiB for the first, then
    // want_max_), which scan_members() replays over the member headers.
    bool host_chunk(size_t k) const { return host_every_ > 1 && k % (size_t)host_every_ == (size_t)host_every_ - 1; }
    void scan_members(size_t p, const size_t cend) {
        std::vector<dcr_bgzf_member> ms;
        int64_t out = 0;
        size_t batch = 128;
        size_t ck = 0, ctotal = 0, cwant = want_;    // fill()'s chunking, replayed
        auto flush = [&](bool last) {
            hook_.stream_add(stream_, ms.data(), (int32_t)ms.size(), last ? 1 : 0);
            ms.clear();
        };
        while (p + 18 <= cend && !stop_members_.load(std::memory_order_relaxed)) {
            if (end_coff_ >= 0 && p >= (uint64_t)end_coff_) {
                if (p != (uint64_t)end_coff_ || end_uoff_ == 0) break;
            }
            const uint8_t *h = map_ + p;
            if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) break;
            const size_t xlen = rd16(h + 10);
            if (cend - p < 12 + xlen) break;
            long bsize = -1;
            for (size_t i = 0; i + 4 <= xlen;) {
                const uint8_t *sf = h + 12 + i;
                const size_t slen = rd16(sf + 2);
                if (sf[0] == 66 && sf[1] == 67 && slen == 2) bsize = rd16(sf + 4);
                i += 4 + slen;
            }
            if (bsize < 0) break;
            const size_t blen = (size_t)bsize + 1;
            if (blen < 12 + xlen + 8 || cend - p < blen) break;
            const uint32_t isize = rd32(h + blen - 4);
            if (isize > 0x10000) break;
            if (ctotal + 0x10000 > cwant) {
                ++ck;
                ctotal = 0;
                cwant = want_max_;
            }
            ctotal += isize;
            if (!host_chunk(ck)) {
                ms.push_back(dcr_bgzf_member{(int64_t)(p + 12 + xlen), out, (uint32_t)(blen - 12 - xlen - 8), isize,
                                             rd32(h + blen - 8), 0});
                out += isize;
            }
            const bool last_of_range = end_coff_ >= 0 && p == (uint64_t)end_coff_;
            p += blen;
            if (last_of_range) break;
            if (ms.size() >= batch) {
                flush(false);
                batch = 1024;
            }
        }
        flush(true);
    }

    Chunk *next() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !full_.empty(); });
        Chunk *c = full_.front();
        full_.pop_front();
        return c;
    }
    void give_back(Chunk *c) {
        {
            std::lock_guard<std::mutex> g(mu_);
            empty_.push_back(c);
        }
        cv_.notify_all();
    }
    double scan_s = 0, index_parse_s = 0;   // DCR_INGEST_PROF

  private:
    void loop() {
        for (;;) {
            Chunk *c;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !empty_.empty(); });
                if (stop_) return;
                c = empty_.front();
                empty_.pop_front();
            }
            fill(*c);
            const bool last = c->eof || !c->err.empty();
            {
                std::lock_guard<std::mutex> g(mu_);
                inflated_.push_back(c);
            }
            cv_.notify_all();
            if (last) return;
        }
    }
    void scan_loop() {
        for (;;) {
            Chunk *c;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !inflated_.empty(); });
                if (stop_) return;
                c = inflated_.front();
                inflated_.pop_front();
            }
            chain(*c);
            const bool last = c->eof || !c->err.empty();
            {
                std::lock_guard<std::mutex> g(mu_);
                chained_.push_back(c);
            }
            cv_.notify_all();
            if (last) return;
        }
    }
    // the records' fields, on the scanner pool, one chunk behind the chain
    // (the chain of chunk k + 1 runs while chunk k is parsed)
    void parse_loop() {
        for (;;) {
            Chunk *c;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !chained_.empty(); });
                if (stop_) return;
                c = chained_.front();
                chained_.pop_front();
            }
            parse(*c);
            const bool last = c->eof || !c->err.empty();
            {
                std::lock_guard<std::mutex> g(mu_);
                full_.push_back(c);
            }
            cv_.notify_all();
            if (last) return;
        }
    }

    // the block_size chain through c, continuing the stream state of the
    // previous chunk (a field or a skip may straddle the boundary)
    void chain(Chunk &c) {
        c.recs.clear();
        c.indexed = false;
        c.chained = false;
        std::vector<size_t> &offs_ = c.offs;
        offs_.clear();
        if (dead_ || !c.err.empty()) { dead_ = true; return; }
        const double t0 = prof_ ? now() : 0;
        const uint8_t *d = c.data() + kHead;
        const size_t n = c.len;
        size_t pos = 0;
        auto field = [&](uint32_t &v) -> bool {      // a 4-byte field, possibly across chunks
            while (nfld_ < 4 && pos < n) fld_[nfld_++] = d[pos++];
            if (nfld_ < 4) return false;
            v = rd32(fld_);
            nfld_ = 0;
            return true;
        };
        for (;;) {
            if (skip_) {
                const size_t a = (size_t)std::min<uint64_t>(skip_, n - pos);
                pos += a;
                skip_ -= a;
                if (skip_) break;
            }
            uint32_t v;
            if (st_ == kRec) {
                if (nfld_ == 0) {
                    while (pos + 4 <= n) {                  // whole records inside the chunk
                        // the chain is a pointer chase through data other cores just wrote
                        __builtin_prefetch(d + pos + 16384);
                        __builtin_prefetch(d + pos + 16384 + 64);
                        __builtin_prefetch(d + pos + 16384 + 128);
                        __builtin_prefetch(d + pos + 16384 + 192);
                        const int32_t bs = rdi32(d + pos);
                        if (bs < 32) { dead_ = true; return; }
                        if (pos + 4 + (size_t)bs > n) break;
                        offs_.push_back(pos);
                        pos += 4 + (size_t)bs;
                    }
                    if (pos + 4 <= n) {                     // one that runs into the next chunk
                        skip_ = pos + 4 + (uint64_t)(uint32_t)rdi32(d + pos) - n;
                        pos = n;
                        break;
                    }
                }
                if (!field(v)) break;                       // its block_size straddles the boundary
                if ((int32_t)v < 32) { dead_ = true; return; }
                skip_ = v;
                continue;
            }
            if (!field(v)) break;
            const int32_t iv = (int32_t)v;
            switch (st_) {
                case kMagic:
                    if (v != 0x014d4142u) { dead_ = true; return; }   // "BAM\1"
                    st_ = kLText;
                    break;
                case kLText:
                    if (iv < 0) { dead_ = true; return; }
                    skip_ = v;
                    st_ = kNRef;
                    break;
                case kNRef:
                    if (iv < 0) { dead_ = true; return; }
                    nref_left_ = iv;
                    st_ = nref_left_ ? kLName : kRec;
                    break;
                default:                                    // kLName: name and l_ref
                    if (iv < 0) { dead_ = true; return; }
                    skip_ = (uint64_t)v + 4;
                    st_ = --nref_left_ ? kLName : kRec;
                    break;
            }
        }
        c.chained = true;
        if (prof_) scan_s += now() - t0;
    }
    void parse(Chunk &c) {
        if (!c.chained) return;
        const double t1 = prof_ ? now() : 0;
        const std::vector<size_t> &offs_ = c.offs;
        c.recs.resize(offs_.size());
        const uint8_t *base = c.data();
        const size_t chunk = 512;
        spool_->run((offs_.size() + chunk - 1) / chunk, [&](size_t k) {
            const size_t e = std::min(offs_.size(), (k + 1) * chunk);
            for (size_t i = k * chunk; i < e; ++i)
                c.recs[i].perr = (uint8_t)rp_.parse_at(base, kHead + offs_[i], c.recs[i]);
            return true;
        });
        c.indexed = true;
        if (prof_) index_parse_s += now() - t1;
    }
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }

    void top_up() {
        cpos_ += cbeg_;
        std::memmove(cbuf_.data(), cbuf_.data() + cbeg_, cend_ - cbeg_);
        cend_ -= cbeg_;
        cbeg_ = 0;
        while (!file_eof_ && cend_ < cbuf_.size()) {
            const size_t got = std::fread(cbuf_.data() + cend_, 1, cbuf_.size() - cend_, f_);
            cend_ += got;
            if (got == 0) file_eof_ = true;
        }
    }
    // inflate the next run of whole blocks into c (after its headroom)
    void fill(Chunk &c) {
        c.len = 0;
        c.eof = false;
        c.err.clear();
        struct Blk { size_t coff, clen, doff; uint32_t isize, crc; };
        std::vector<Blk> blks;
        size_t total = 0, cut = SIZE_MAX;
        if (range_done_) { c.eof = true; return; }
        // compressed bytes are only moved while no parsed block points into them
        if (!file_eof_ && cend_ - cbeg_ < cbuf_.size() / 2) top_up();
        for (;;) {
            while (!range_done_ && cend_ - cbeg_ >= 18 && total + 0x10000 <= want_) {
                if (end_coff_ >= 0 && cpos_ + cbeg_ >= (uint64_t)end_coff_) {
                    // the range's last block: only its first end_uoff bytes
                    range_done_ = true;
                    if (cpos_ + cbeg_ != (uint64_t)end_coff_ || end_uoff_ == 0) break;
                    cut = total + end_uoff_;
                }
                const uint8_t *h = cdata() + cbeg_;
                if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) { c.err = "not a BGZF file"; return; }
                const size_t xlen = rd16(h + 10);
                if (cend_ - cbeg_ < 12 + xlen) break;
                long bsize = -1;
                for (size_t i = 0; i + 4 <= xlen;) {
                    const uint8_t *sf = h + 12 + i;
                    const size_t slen = rd16(sf + 2);
                    if (sf[0] == 66 && sf[1] == 67 && slen == 2) bsize = rd16(sf + 4);
                    i += 4 + slen;
                }
                if (bsize < 0) { c.err = "BGZF block without BC field"; return; }
                const size_t blen = (size_t)bsize + 1;
                if (blen < 12 + xlen + 8) { c.err = "BGZF block size too small"; return; }
                if (cend_ - cbeg_ < blen) break;
                Blk b;
                b.coff = cbeg_ + 12 + xlen;
                b.clen = blen - 12 - xlen - 8;
                b.crc = rd32(h + blen - 8);
                b.isize = rd32(h + blen - 4);
                if (b.isize > 0x10000) { c.err = "BGZF ISIZE above 64 KiB"; return; }
                b.doff = Inflater::kHead + total;
                total += b.isize;
                blks.push_back(b);
                cbeg_ += blen;
            }
            if (!blks.empty() || range_done_) break;
            if (file_eof_) {
                if (cend_ > cbeg_) { c.err = "truncated BGZF block at the end of the file"; return; }
                break;
            }
            top_up();
        }
        uint8_t *dst = c.data();
        const uint8_t *src = cdata();
        auto host_inflate = [&](size_t i) {
            const Blk &b = blks[i];
            if (b.isize == 0) return b.clen <= 2;      // empty block (the EOF marker)
            size_t got = 0;
            if (libdeflate_deflate_decompress(tl_dec.get(), src + b.coff, b.clen, dst + b.doff, b.isize, &got) != 0 ||
                got != b.isize)
                return false;
            return libdeflate_crc32(0, dst + b.doff, b.isize) == b.crc;
        };
        bool ok = true;
        const bool host_k = stream_ && !blks.empty() && host_chunk(fill_k_);
        if (!blks.empty()) ++fill_k_;
        if (host_k) {
            ok = pool_->run(blks.size(), host_inflate);        // a chunk the stream skipped
        } else if (stream_ && !blks.empty()) {
            // inflated ahead by the device: copy this chunk's bytes out
            const size_t out_blocks = blks.back().doff + blks.back().isize - kHead;
            const int rc = hook_.stream_fetch(stream_, stream_out_, (int64_t)out_blocks, dst + kHead);
            if (rc != 0) {
                c.err = rc > 0 ? "BGZF block failed to inflate or CRC mismatch" : "GPU inflate failed";
                return;
            }
            stream_out_ += (int64_t)out_blocks;
            // the chunk's first member against its CRC32: a stream out of step
            // with this walk (host chunks skipped differently) would hand over
            // another member's bytes
            if (host_every_ > 1 && libdeflate_crc32(0, dst + blks[0].doff, blks[0].isize) != blks[0].crc) {
                c.err = "GPU inflate stream out of step with the reader";
                return;
            }
        } else if (gpu_ && !blks.empty()) {
            // the chunk's first k members inflate on the GPU (their compressed
            // bytes copied to page-locked staging by the pool first; CRC32 and
            // ISIZE checked on the device; output straight into the chunk
            // buffer) while the host pool inflates the rest; k follows the
            // measured times of both sides (their finish times meet)
            const size_t n = blks.size();
            const size_t k = std::min(n, std::max<size_t>(1, (size_t)(frac_ * (double)n + 0.5)));
            const size_t g0 = blks[0].coff, g1 = blks[k - 1].coff + blks[k - 1].clen;
            const size_t nb = g1 - g0;
            uint8_t *stage = stage_pin_ ? stage_pin_ : stage_.data();
            if (nb > stage_cap_) { c.err = "BGZF chunk larger than its staging buffer"; return; }
            const size_t piece = (size_t)1 << 20;
            pool_->run((nb + piece - 1) / piece, [&](size_t q) {
                const size_t a = q * piece, m = std::min(piece, nb - a);
                std::memcpy(stage + a, src + g0 + a, m);
                return true;
            });
            mem_.resize(k);
            for (size_t i = 0; i < k; ++i) {
                const Blk &b = blks[i];
                mem_[i] = dcr_bgzf_member{(int64_t)(b.coff - g0), (int64_t)(b.doff - kHead), (uint32_t)b.clen,
                                          b.isize, b.crc, 0};
            }
            const size_t out_k = blks[k - 1].doff + blks[k - 1].isize - kHead;
            int rc = 0;
            double t_gpu = 0, t_host = 0;
            std::thread gt([&] {
                const double t0 = now();
                rc = hook_.run(hook_.user, stage, (int64_t)nb, mem_.data(), (int32_t)k, dst + kHead, (int64_t)out_k);
                t_gpu = now() - t0;
            });
            const double th = now();
            if (k < n) ok = pool_->run(n - k, [&](size_t i) { return host_inflate(k + i); });
            t_host = now() - th;
            gt.join();
            if (rc != 0) {
                c.err = rc > 0 ? "BGZF block failed to inflate or CRC mismatch" : "GPU inflate failed";
                return;
            }
            if (k < n && t_gpu > 0 && t_host > 0) {
                frac_ *= std::sqrt(t_host / t_gpu);
                frac_ = std::min(0.95, std::max(0.05, frac_));
            } else if (k == n && t_gpu > 0) {
                frac_ = 0.95;
            }
        } else {
            ok = pool_->run(blks.size(), host_inflate);
        }
        if (!ok) { c.err = "BGZF block failed to inflate or CRC mismatch"; return; }
        c.len = total;
        if (blks.empty() && file_eof_ && cend_ == cbeg_) c.eof = true;
        want_ = want_max_;
        if (range_done_) {
            if (cut != SIZE_MAX) {
                if (cut > total) { c.err = "range end past the end of its BGZF block"; return; }
                c.len = cut;
            }
            c.eof = true;
        }
    }

    FILE *f_;
    std::unique_ptr<Pool> pool_, spool_;   // from PoolCache, given back in the destructor
    RecParser rp_;
    int64_t end_coff_;
    uint32_t end_uoff_;
    uint64_t cpos_ = 0;             // file offset of cdata()[0]
    const uint8_t *map_ = nullptr;  // the whole file, when it maps (then cpos_ = 0 and no top_up)
    size_t map_len_ = 0;
    const uint8_t *cdata() const { return map_ ? map_ : cbuf_.data(); }
    bool range_done_ = false;
    size_t want_ = (size_t)4 << 20;   // the first chunk is small: the walk starts sooner
    size_t want_max_ = kWant;
    bool gpu_ = false;                 // members inflated by hook_.run
    dcr_inflate_hook hook_{};
    uint8_t *stage_pin_ = nullptr;     // page-locked compressed staging (GPU inflate)
    HugeBuf stage_;
    size_t stage_cap_ = 0;
    std::vector<dcr_bgzf_member> mem_;
    void *stream_ = nullptr;           // the device inflater's stream over the whole mapped input
    std::thread mth_;                  // appends the input's members to stream_
    std::atomic<bool> stop_members_{false};
    int64_t stream_out_ = 0;           // output bytes fetched from it so far
    double frac_ = 0.5;                // share of a chunk's members inflated on the GPU
    int host_every_ = 0;               // every host_every_-th chunk inflated by the host pool (stream mode)
    size_t fill_k_ = 0;                // chunks filled so far
    HugeBuf cbuf_;
    size_t cbeg_ = 0, cend_ = 0;
    bool file_eof_ = false;
    Chunk chunks_[5];                  // filling, chaining, parsing, walked, one spare
    std::deque<Chunk *> empty_, inflated_, chained_, full_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    std::thread th_, sth_, pth_;
    // scanner stream state
    enum { kMagic, kLText, kNRef, kLName, kRec } st_ = kMagic;
    uint8_t fld_[4] = {0, 0, 0, 0};
    int nfld_ = 0;
    uint64_t skip_ = 0;
    int32_t nref_left_ = 0;
    bool dead_ = false;
    const bool prof_ = std::getenv("DCR_INGEST_PROF") != nullptr;
};

// DCR_INGEST_PROF=1: seconds per ingest stage, printed to stderr at close
struct IngestProf {
    bool on = std::getenv("DCR_INGEST_PROF") != nullptr;
    double wait_chunk = 0, scan = 0, parse = 0, flush = 0, walk_total = 0, complete = 0, tasks_wait = 0;
    int64_t indexed = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};

struct dcr_ingest {
    FILE *f = nullptr;
    IngestProf prof;
    dcr_ingest_cfg cfg{};
    std::unique_ptr<Pool> pool;          // pack jobs (on the packer thread, below)
    std::unique_ptr<Pool> ppool;         // record parse of serially scanned records (walk thread)
    std::unique_ptr<Inflater> infl;
    RecParser rp;
    // decompressed window: wb[wpos, wend) (a chunk's buffer, or big[] for huge leftovers)
    const uint8_t *wb = nullptr;
    size_t wpos = 0, wend = 0;
    Chunk *cur = nullptr;               // the chunk whose buffer is the window (null: big[])
    size_t ci = 0;                      // next unserved record of cur->recs
    HugeBuf big[2];
    int big_i = 0;
    bool data_eof = false;
    std::vector<uint8_t> header;
    // the open family (passing reads, input order): pointers into the served
    // records, or into fam_store once those are replaced (materialize_family)
    std::vector<const Rec *> fam;
    std::vector<Rec> fam_store;
    std::string umi2_;                   // check_family_UMIs scratch
    bool mid_end = false;     // the range stops before the end of the file
    std::vector<int32_t> sample_calls;   // (n, k) of every random.sample call
    // state gate (dcr_ingest_set_state_gate): called once, before the first
    // random.sample call, for the exact generator state to sample from
    dcr_state_gate_fn gate_fn = nullptr;
    void *gate_user = nullptr;
    bool gate_open = false;
    bool started = false;     // any passing read seen
    bool finished = false;    // EOF processed
    bool errored = false;
    // counters :1508
    int64_t passed = 0, excluded = 0, processed = 0, filtered = 0, records = 0;
    PyRandom rng;
    // pack jobs of the current batch
    std::vector<Job> jobs;
    std::vector<int> idx_tmp;

    ~dcr_ingest() {
        pk_stop_thread();
        if (prof.on)
            std::fprintf(stderr,
                         "[ingest] walk %.3f s: chunk wait %.3f, serial scan %.3f, parse %.3f, pack copy %.3f, "
                         "families %.3f, family tasks wait %.3f; scanner stage: chain %.3f, parse %.3f; indexed "
                         "records %lld of %lld\n",
                         prof.walk_total, prof.wait_chunk, prof.scan, prof.parse, prof.flush, prof.complete,
                         prof.tasks_wait,
                         infl ? infl->scan_s : 0.0,
                         infl ? infl->index_parse_s : 0.0, (long long)prof.indexed, (long long)records);
        infl.reset();             // stops the inflate thread before the file closes
        if (f) std::fclose(f);
        PoolCache::get().give(std::move(pool));
        PoolCache::get().give(std::move(ppool));
    }

    // make at least n bytes available at wpos (keeping the open family);
    // 1: ok, 0: clean end of data with fewer bytes, -1: error
    int need(size_t n) {
        while (wend - wpos < n) {
            if (data_eof) return 0;
            // queued families point into this window: a chunk window is
            // retired (given back once they have run, release_retired); a
            // window of the leftover buffers waits for them here
            {
                const size_t keep0 = fam.empty() ? wpos : std::min(wpos, fam.front()->off);
                if (!cur || wend - keep0 > Inflater::kHead) {
                    if (flush_tasks() < 0) return -1;
                } else {
                    kick_tasks(true);
                    release_retired();
                }
            }
            flush_jobs();                           // the pack jobs point into it too
            const double tw = prof.on ? IngestProf::now() : 0;
            Chunk *nx = infl->next();
            if (prof.on) prof.wait_chunk += IngestProf::now() - tw;
            if (!nx->err.empty()) {
                g_err = nx->err;
                data_eof = true;
                return -1;
            }
            const size_t keep = fam.empty() ? wpos : std::min(wpos, fam.front()->off);
            const size_t left = wend - keep;
            size_t base;
            const uint8_t *nbuf;
            if (left <= Inflater::kHead) {
                base = Inflater::kHead - left;
                if (left) std::memcpy(nx->data() + base, wb + keep, left);
                nbuf = nx->data();
            } else {                                 // a leftover larger than the headroom
                HugeBuf &bg = big[big_i];
                big_i ^= 1;
                bg.resize(left + nx->len + 16);
                std::memcpy(bg.data(), wb + keep, left);
                std::memcpy(bg.data() + left, nx->data() + Inflater::kHead, nx->len);
                base = 0;
                nbuf = bg.data();
            }
            for (auto &r : fam_store) r.off = r.off - keep + base;   // fam points into fam_store here
            wpos = wpos - keep + base;
            wend = base + left + nx->len;
            wb = nbuf;
            if (cur) {
                if (tasks.size() > tk_done_seen()) retired.push_back(Retired{cur, tasks.size()});
                else infl->give_back(cur);
            }
            ci = 0;
            if (nbuf == nx->data()) cur = nx;       // the chunk's record offsets hold in the window
            else { cur = nullptr; infl->give_back(nx); }
            if (nx->eof) data_eof = true;
        }
        return 1;
    }

    // -- pack jobs -------------------------------------------------------------
    // The walk appends a job per read it packs; every kPkStep jobs it hands
    // the new ones to the packer thread, which copies them on the pool while
    // the walk goes on (the copy had run between walk steps, the walk waiting
    // for it: ~40 % of an ingest).  Jobs point into the current window and
    // the batch, so the walk waits for the packer before the window moves
    // (need()) and before the batch is handed out (next()).  `jobs` is
    // reserved for the batch's reads, so it never reallocates under the packer.
    dcr_host_batch *hb = nullptr;
    static constexpr size_t kPkStep = 4096;
    std::thread pk_th;
    std::mutex pk_mu;
    std::condition_variable pk_cv;
    size_t pk_sub = 0, pk_done = 0;      // jobs [0, pk_sub) handed over, [0, pk_done) copied
    bool pk_quit = false;
    const uint8_t *pk_w = nullptr;       // the window and batch of the handed-over jobs
    dcr_host_batch *pk_b = nullptr;

    void pk_start_thread() {
        pk_th = std::thread([this] {
            for (;;) {
                size_t j0, j1, t0, t1;
                const uint8_t *w;
                dcr_host_batch *b;
                {
                    std::unique_lock<std::mutex> lk(pk_mu);
                    pk_cv.wait(lk, [&] { return pk_quit || pk_sub > pk_done || tk_sub > tk_done; });
                    if (pk_quit) return;
                    j0 = pk_done;
                    j1 = pk_sub;
                    t0 = tk_done;
                    t1 = tk_sub;
                    w = pk_w;
                    b = pk_b;
                }
                if (t1 > t0) run_tasks(b, t0, t1);
                if (j1 > j0) pack_range(w, b, jobs.data(), j0, j1);
                {
                    std::lock_guard<std::mutex> g(pk_mu);
                    pk_done = j1;
                    tk_done = t1;
                }
                pk_cv.notify_all();
            }
        });
    }
    void pk_stop_thread() {
        if (!pk_th.joinable()) return;
        {
            std::lock_guard<std::mutex> g(pk_mu);
            pk_quit = true;
        }
        pk_cv.notify_all();
        pk_th.join();
    }
    // hand the jobs appended since the last hand-over to the packer
    void kick_jobs(bool force) {
        if (jobs.size() == pk_sub || (!force && jobs.size() - pk_sub < kPkStep)) return;
        {
            std::lock_guard<std::mutex> g(pk_mu);
            pk_sub = jobs.size();
            pk_w = wb;
            pk_b = hb;
        }
        pk_cv.notify_all();
    }
    // -- deferred family completion --------------------------------------------
    // A family with nothing to sample (the common case) is reserved by the
    // walk -- its table entry, names, read / base / CIGAR / side-byte ranges
    // and column offsets, all sizes known from one pass over its records --
    // and the rest of complete_family (the UMI and rname checks, the split
    // and the per-read fields and copies) runs as a task on the packer thread
    // and its pool while the walk goes on.  Tasks point into the window and
    // the records, so they are drained (flush_tasks) before either changes,
    // before a family that samples (the checks of earlier families come
    // first, :1548-1551) and at the end of a batch; the first task (in input
    // order) that fails truncates the batch to its reservation and stops
    // there, exactly where complete_family would have stopped.
    // a family's records: a pointer list, or (p null) consecutive records
    struct RecList {
        const Rec *const *p;
        const Rec *base;
        const Rec *operator[](size_t i) const { return p ? p[i] : base + i; }
    };
    struct FamTask {
        const uint8_t *w;               // the window its records' offsets refer to
        uint32_t rb, n;                 // the family's records: pend_recs[rb, rb + n), or cbase[0, n)
        const Rec *cbase = nullptr;     // set when they are consecutive in the record index (no copy)
        int32_t t, f;                   // table entry; processed family (-1: filtered)
        int64_t read_base, base_off[4], cig_off[4];   // per subfamily (split order)
        int64_t filt_off;               // filtered: its bytes in side_filt
        // the batch and counters as they were before this family
        int32_t fam_before;
        int64_t names_before, exc_before, filt_before, ss_before, ds_before;
        int64_t c_passed, c_records, c_excluded, c_processed, c_filtered;
        int err_kind = DCR_ERR_NONE;
        std::string err;
    };
    std::vector<FamTask> tasks;
    std::vector<const Rec *> pend_recs;
    std::deque<Rec> task_recs;           // copies of queued records that lived in fam_store
    // chunks whose window queued tasks still read: given back once tasks
    // [0, upto) have run
    struct Retired { Chunk *c; size_t upto; };
    std::deque<Retired> retired;
    size_t tk_done_seen() {
        std::lock_guard<std::mutex> g(pk_mu);
        return tk_done;
    }
    void release_retired() {
        if (retired.empty()) return;
        const size_t done = tk_done_seen();
        while (!retired.empty() && retired.front().upto <= done) {
            infl->give_back(retired.front().c);
            retired.pop_front();
        }
    }
    size_t tk_sub = 0, tk_done = 0;      // tasks [0, tk_sub) handed over, [0, tk_done) run
    static constexpr size_t kTkStep = 256;

    void run_task(FamTask &T, const uint8_t *w, dcr_host_batch *b) const {
        const RecList fr{T.cbase ? nullptr : pend_recs.data() + T.rb, T.cbase};
        std::string umi2;
        T.err_kind = check_family(fr, T.n, w, umi2, T.err);
        if (T.err_kind != DCR_ERR_NONE) return;
        if (T.f < 0) {                  // filtered: its reads to _filteredfamilies.bam in input order
            int64_t o = T.filt_off;
            for (uint32_t i = 0; i < T.n; ++i) {
                std::memcpy(b->side_filt + o, w + fr[i]->off, fr[i]->len);
                o += fr[i]->len;
            }
            return;
        }
        // split_family order: subfamily k's reads in input order after those of k - 1
        int64_t ri[4], bo[4], co[4];
        int64_t acc = T.read_base;
        for (int k = 0; k < 4; ++k) {
            ri[k] = acc;
            acc = b->sub_off[4 * T.f + k + 1];
            bo[k] = T.base_off[k];
            co[k] = T.cig_off[k];
        }
        for (uint32_t j = 0; j < T.n; ++j) {
            const Rec &rc = *fr[j];
            const int k = rc.subk;
            if (k < 0) continue;
            const uint8_t *r = w + rc.off + 4;
            const uint32_t l_rn = r[8];
            const uint32_t n_cig = rd16(r + 12);
            const int32_t l_seq = rdi32(r + 16);
            const int64_t i = ri[k]++;
            b->read_pos[i] = rdi32(r + 4);
            b->read_mapq[i] = r[9];
            b->seq_len[i] = l_seq;
            b->seq_off[i] = bo[k];
            b->cig_off[i] = (int32_t)co[k];
            b->cig_n[i] = (int32_t)n_cig;
            const uint8_t *cig = r + 32 + l_rn;
            std::memcpy(b->cigar + co[k], cig, 4u * n_cig);
            const uint8_t *sq = cig + 4u * n_cig;
            decode_seq(sq, l_seq, b->bases + bo[k]);
            std::memcpy(b->quals + bo[k], sq + ((l_seq + 1) >> 1), (size_t)l_seq);
            bo[k] += l_seq;
            co[k] += n_cig;
        }
    }
    void run_tasks(dcr_host_batch *b, size_t t0, size_t t1) {
        const size_t chunk = 32;
        pool->run((t1 - t0 + chunk - 1) / chunk, [&](size_t c) {
            const size_t te = std::min(t1, t0 + (c + 1) * chunk);
            for (size_t t = t0 + c * chunk; t < te; ++t) run_task(tasks[t], tasks[t].w, b);
            return true;
        });
    }
    void kick_tasks(bool force) {
        if (tasks.size() == tk_sub || (!force && tasks.size() - tk_sub < kTkStep)) return;
        {
            std::lock_guard<std::mutex> g(pk_mu);
            tk_sub = tasks.size();
            pk_w = wb;
            pk_b = hb;
        }
        pk_cv.notify_all();
    }
    // run every queued task; the first failure (input order) cuts the batch
    // to that family's reservation and stops there.  1 ok, -1 stopped.
    int flush_tasks() {
        if (tasks.empty()) return 1;
        kick_tasks(true);
        {
            const double tw = prof.on ? IngestProf::now() : 0;
            std::unique_lock<std::mutex> lk(pk_mu);
            pk_cv.wait(lk, [&] { return tk_done == tk_sub; });
            tk_sub = tk_done = 0;
            if (prof.on) prof.tasks_wait += IngestProf::now() - tw;
        }
        for (const Retired &r : retired) infl->give_back(r.c);
        retired.clear();
        int rc = 1;
        for (FamTask &T : tasks) {
            if (T.err_kind == DCR_ERR_NONE) continue;
            dcr_host_batch *b = hb;
            b->n_tab = T.t;
            b->n_fam = T.fam_before;
            b->n_reads = T.read_base;
            b->n_bases = T.base_off[0];
            b->n_cigar = T.cig_off[0];
            b->n_names = T.names_before;
            b->n_side_exc = T.exc_before;
            b->n_side_filt = T.filt_before;
            b->ss_cols = T.ss_before;
            b->ds_cols = T.ds_before;
            passed = T.c_passed;
            records = T.c_records;
            excluded = T.c_excluded;
            processed = T.c_processed;
            filtered = T.c_filtered;
            rc = stop(T.err_kind, T.err);
            break;
        }
        tasks.clear();
        pend_recs.clear();
        task_recs.clear();
        return rc;
    }

    // preprocess_family for a family that samples nothing, deferred (above);
    // a family that samples, or that the reservation cannot describe, takes
    // complete_family after the queued tasks.  Returns as complete_family.
    int queue_family() {
        dcr_host_batch *b = hb;
        const Rec &r0 = *fam.front();
        int64_t nb = 0, nc = 0, filt_bytes = 0;
        int64_t cnt[4] = {0, 0, 0, 0}, nbk[4] = {0, 0, 0, 0}, nck[4] = {0, 0, 0, 0};
        int64_t mn[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0};
        int16_t eqx[4] = {0, 0, 0, 0};
        const Rec *first[4] = {nullptr, nullptr, nullptr, nullptr};
        for (const Rec *r : fam) {
            nb += r->l_seq;
            nc += r->n_cig;
            filt_bytes += r->len;
            const int k = r->subk;
            if (k < 0) continue;
            if (!first[k]) {
                first[k] = r;
                mn[k] = r->pos;
                mx[k] = r->end_kept;
            } else {
                if (r->pos < mn[k]) mn[k] = r->pos;
                if (r->end_kept > mx[k]) mx[k] = r->end_kept;
            }
            ++cnt[k];
            nbk[k] += r->l_seq;
            nck[k] += r->n_cig;
            if (eqx[k] < 0x7fff && r->eqx) ++eqx[k];
        }
        bool samples = false, enough = true;
        for (int k = 0; k < 4; ++k) {                      // check_number_reads (:157-188)
            if (cnt[k] < cfg.min_reads) { enough = false; break; }
            if (cnt[k] > cfg.max_reads) { samples = true; break; }
        }
        const size_t l_code = r0.l_code;
        // the RX written below is that of the first A1 and B1 read, whose
        // length the deferred UMI check (run_task) has not yet tied to r0's
        const int64_t l_rx0 = first[0] ? first[0]->l_rx : 0, l_rx2 = first[2] ? first[2]->l_rx : 0;
        const int64_t names_need = (int64_t)l_code + 1 + (l_rx0 + 1) + (l_rx2 + 1) + 64 * 2;
        // the family's records consecutive in the record index (not copies in fam_store)?
        bool contig = fam.front() < fam_store.data() || fam.front() >= fam_store.data() + fam_store.size();
        for (size_t j = 1; j < fam.size() && contig; ++j) contig = fam[j] == fam.front() + j;
        if (samples || (!contig && pend_recs.size() + fam.size() > pend_recs.capacity()) ||
            tasks.size() == tasks.capacity()) {
            if (flush_tasks() < 0) return -1;
            return complete_family();
        }
        const bool fits = b->n_tab < b->cap_tab && b->n_fam < b->cap_fam &&
                          b->n_reads + (int64_t)fam.size() <= b->cap_reads && b->n_bases + nb <= b->cap_bases &&
                          b->n_cigar + nc <= b->cap_cigar && b->n_names + names_need <= b->cap_names &&
                          b->n_side_filt + filt_bytes <= b->cap_side;
        if (!fits) {
            if (b->n_tab == 0 && b->n_side_exc == 0) {
                if (flush_tasks() < 0) return -1;
                return fail_capacity("one family exceeds the batch capacities");
            }
            return 0;
        }
        FamTask T;
        T.rb = (uint32_t)pend_recs.size();
        T.n = (uint32_t)fam.size();
        T.fam_before = b->n_fam;
        T.names_before = b->n_names;
        T.exc_before = b->n_side_exc;
        T.filt_before = b->n_side_filt;
        T.ss_before = b->ss_cols;
        T.ds_before = b->ds_cols;
        T.read_base = b->n_reads;
        T.c_passed = passed;
        T.c_records = records;
        T.c_excluded = excluded;
        T.c_processed = processed;
        T.c_filtered = filtered;
        const int32_t t = b->n_tab++;
        T.t = t;
        b->tab_sampled[t] = 0;
        b->tab_exc_cut[t] = b->n_side_exc;
        b->tab_filt_cut[t] = b->n_side_filt;
        b->tab_code[t] = put_name(code_of(r0), l_code);
        const int64_t code_off = b->tab_code[t];
        int64_t bo = b->n_bases, co = b->n_cigar;
        for (int k = 0; k < 4; ++k) {
            T.base_off[k] = bo;
            T.cig_off[k] = co;
            bo += nbk[k];
            co += nck[k];
        }
        if (!enough) {
            b->tab_kind[t] = DCR_FAM_FILTERED;
            b->tab_proc[t] = -1;
            T.f = -1;
            T.filt_off = b->n_side_filt;
            b->n_side_filt += filt_bytes;
            ++filtered;
        } else {
            const int32_t f = b->n_fam++;
            T.f = f;
            T.filt_off = 0;
            b->tab_kind[t] = DCR_FAM_PROCESSED;
            b->tab_proc[t] = f;
            b->fam_tid[f] = r0.tid;
            b->fam_code[f] = code_off;
            for (int k = 0; k < 4; ++k) {
                b->fam_eqx[4 * f + k] = (uint16_t)eqx[k];
                b->sub_off[4 * f + k + 1] = b->sub_off[4 * f + k] + cnt[k];
                const int64_t tt = (std::max<int64_t>(mx[k] - mn[k], 1) + 15) & ~(int64_t)15;
                b->ss_col_off[4 * f + k + 1] = b->ss_col_off[4 * f + k] + tt;
            }
            for (int j = 0; j < 2; ++j) {
                const int a = 2 * j, c = 2 * j + 1;
                int64_t tt = std::max(mx[a], mx[c]) - std::min(mn[a], mn[c]);
                tt = (std::max<int64_t>(tt, 1) + 15) & ~(int64_t)15;
                b->ds_col_off[2 * f + j + 1] = b->ds_col_off[2 * f + j] + tt;
            }
            b->n_reads = b->sub_off[4 * f + 4];
            b->n_bases = bo;
            b->n_cigar = co;
            b->ss_cols = b->ss_col_off[4 * f + 4];
            b->ds_cols = b->ds_col_off[2 * f + 2];
            // writer metadata: RX of the read0 of A1 and of B1 (:1367 via add_tags)
            for (int j = 0; j < 2; ++j) {
                const Rec *r = first[2 * j];
                if (!r) b->fam_rx[2 * f + j] = put_name("", 0);
                else b->fam_rx[2 * f + j] = put_name(rx_of(*r), r->l_rx);
            }
            ++processed;
        }
        T.w = wb;
        // consecutive records of the record index (the common case): the task
        // points at them, no per-record copy into pend_recs (whose 8-byte
        // writes each cost a write-allocate miss: 25 cycles per read).
        // Otherwise pointers; records materialized into fam_store move with
        // the next window (need() rewrites their offsets): the task keeps copies
        const Rec *fs0 = fam_store.data(), *fs1 = fs0 + fam_store.size();
        if (contig) {
            T.cbase = fam.front();
        } else {
            for (const Rec *r : fam) {
                if (r >= fs0 && r < fs1) {
                    task_recs.push_back(*r);
                    pend_recs.push_back(&task_recs.back());
                } else {
                    pend_recs.push_back(r);
                }
            }
        }
        tasks.push_back(std::move(T));
        if (tasks.size() - tk_sub >= kTkStep) release_retired();
        return 1;
    }

    void flush_jobs() {
        if (jobs.empty()) return;
        const double tf = prof.on ? IngestProf::now() : 0;
        struct Acc {
            double &d, t;
            bool on;
            ~Acc() { if (on) d += IngestProf::now() - t; }
        } acc{prof.flush, tf, prof.on};
        kick_jobs(true);
        {
            std::unique_lock<std::mutex> lk(pk_mu);
            pk_cv.wait(lk, [&] { return pk_done == pk_sub; });
            pk_sub = pk_done = 0;
        }
        jobs.clear();
    }
    void pack_range(const uint8_t *w, dcr_host_batch *b, const Job *jobv, size_t j0, size_t j1) {
        const size_t chunk = 2048;
        const size_t nchunks = (j1 - j0 + chunk - 1) / chunk;
        pool->run(nchunks, [&](size_t c) {
            const size_t je = std::min(j1, j0 + (c + 1) * chunk);
            for (size_t j = j0 + c * chunk; j < je; ++j) {
                const Job &jb = jobv[j];
                const uint8_t *r = w + jb.rec + 4;
                const uint32_t l_rn = r[8];
                const uint32_t n_cig = rd16(r + 12);
                const int32_t l_seq = rdi32(r + 16);
                const int32_t i = jb.read;
                b->read_pos[i] = rdi32(r + 4);
                b->read_mapq[i] = r[9];
                b->seq_len[i] = l_seq;
                b->seq_off[i] = jb.dst_base;
                b->cig_off[i] = (int32_t)jb.dst_cig;
                b->cig_n[i] = (int32_t)n_cig;
                const uint8_t *cig = r + 32 + l_rn;
                std::memcpy(b->cigar + jb.dst_cig, cig, 4u * n_cig);
                const uint8_t *s = cig + 4u * n_cig;
                decode_seq(s, l_seq, b->bases + jb.dst_base);
                std::memcpy(b->quals + jb.dst_base, s + ((l_seq + 1) >> 1), (size_t)l_seq);
            }
            return true;
        });
    }

    // parsed records ahead of the walk: rqp[rq_pos, rq_n) (the scanner's
    // index of the current chunk, or rq from the serial scan)
    const Rec *rqp = nullptr;
    std::vector<Rec> rq;
    std::vector<size_t> rq_off;
    size_t rq_pos = 0, rq_n = 0;

    // scan the next complete records of the window (block_size chain) and
    // parse them on the pool; 1 some, 0 end of data, -1 error (g_err)
    // the open family's records out of rq before rq is refilled
    void materialize_family() {
        if (fam.empty()) return;
        std::vector<Rec> tmp;
        tmp.reserve(fam.size());
        for (const Rec *r : fam) tmp.push_back(*r);
        fam_store.swap(tmp);
        for (size_t i = 0; i < fam.size(); ++i) fam[i] = &fam_store[i];
    }

    int prefetch_records() {
        constexpr size_t kRQ = 16384;
        // queued families may point into rq (the serial scan's records): drain
        // them before rq is refilled; the scanner's records of a chunk stay
        // put until need() gives the chunk back, which drains them itself
        if (rqp == rq.data() && flush_tasks() < 0) return -1;
        materialize_family();
        if (rq.size() < kRQ) { rq.resize(kRQ); rq_off.resize(kRQ); }
        rq_pos = rq_n = 0;
        size_t n = 0;
        double ts = prof.on ? IngestProf::now() : 0;
        size_t stop_at = SIZE_MAX;
        for (;;) {
            // the scanner's records of the current chunk, from wpos on
            if (cur && cur->indexed && ci < cur->recs.size()) {
                const std::vector<Rec> &R = cur->recs;
                while (ci < R.size() && R[ci].off < wpos) ++ci;
                if (ci < R.size() && R[ci].off == wpos) {
                    rqp = R.data() + ci;
                    rq_n = R.size() - ci;
                    ci = R.size();
                    prof.indexed += (int64_t)rq_n;
                    return 1;
                }
            }
            // serial scan: records straddling a chunk boundary, unindexed chunks
            stop_at = (cur && cur->indexed && ci < cur->recs.size()) ? cur->recs[ci].off : SIZE_MAX;
            size_t p = wpos;
            while (n < kRQ && wend - p >= 4 && p < stop_at) {
                __builtin_prefetch(wb + p + 16384);
                __builtin_prefetch(wb + p + 16384 + 64);
                __builtin_prefetch(wb + p + 16384 + 128);
                __builtin_prefetch(wb + p + 16384 + 192);
                const int32_t bs = rdi32(wb + p);
                if (bs < 32) {
                    if (n == 0) { g_err = "malformed BAM record (block_size < 32)"; return -1; }
                    break;
                }
                if (wend - p - 4 < (size_t)bs) break;
                rq_off[n++] = p;
                p += 4 + (size_t)bs;
            }
            if (n > 0) break;
            int st;
            if (wend - wpos >= 4) {
                const int32_t bs = rdi32(wb + wpos);
                if (bs < 32) { g_err = "malformed BAM record (block_size < 32)"; return -1; }
                st = need(4 + (size_t)bs);
            } else {
                st = need(4);
            }
            if (st < 0) return -1;
            if (st == 0) {
                if (wend > wpos) { g_err = "truncated BAM record at the end of the file"; return -1; }
                return 0;
            }
        }
        // a serial record running past the index's next record: the index is off
        if (stop_at != SIZE_MAX && rq_off[n - 1] + 4 + (size_t)rdi32(wb + rq_off[n - 1]) > stop_at) cur->indexed = false;
        const size_t chunk = 512;
        const double tp = prof.on ? IngestProf::now() : 0;
        if (prof.on) prof.scan += tp - ts;
        ppool->run((n + chunk - 1) / chunk, [&](size_t c) {
            const size_t e = std::min(n, (c + 1) * chunk);
            for (size_t i = c * chunk; i < e; ++i) rq[i].perr = (uint8_t)rp.parse_at(wb, rq_off[i], rq[i]);
            return true;
        });
        if (prof.on) prof.parse += IngestProf::now() - tp;
        rqp = rq.data();
        rq_n = n;
        return 1;
    }

    const uint8_t *at(const Rec &r, uint32_t o) const { return wb + r.off + o; }

    const char *code_of(const Rec &r) const {
        return r.l_code <= sizeof r.code ? r.code : (const char *)at(r, r.o_mi);
    }
    const char *rx_of(const Rec &r) const { return (const char *)at(r, r.o_rx); }
    bool same_code(const Rec &a, const Rec &b) const {
        if (a.l_code != b.l_code) return false;
        if (a.l_code <= sizeof a.code) {            // zero-padded inline copies: three words
            uint64_t x[3], y[3];
            std::memcpy(x, a.code, sizeof x);
            std::memcpy(y, b.code, sizeof y);
            return ((x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2])) == 0;
        }
        return std::memcmp(code_of(a), code_of(b), a.l_code) == 0;
    }

    // check_family_UMIs (:100-113), every RX is umi1 or its swapped halves,
    // then check_family_rnames (:116-128), over the family's records fr[0, n)
    // in window w.  Returns DCR_ERR_NONE or the error kind with its message.
    int check_family(RecList fr, size_t n, const uint8_t *w, std::string &umi2, std::string &msg) const {
        const Rec &r0 = *fr[0];
        auto rx_at = [&](const Rec &r) { return (const char *)(w + r.off + r.o_rx); };
        auto code_at = [&](const Rec &r) { return r.l_code <= sizeof r.code ? r.code : (const char *)(w + r.off + r.o_mi); };
        if (r0.rx_type != 'Z') { msg = "'int' object has no attribute 'split'"; return DCR_ERR_ATTRIBUTE; }
        const char *umi1 = rx_at(r0);
        const size_t l1 = r0.l_rx;
        const char *d1p = (const char *)std::memchr(umi1, '-', l1);
        if (!d1p) { msg = "list index out of range"; return DCR_ERR_INDEX; }
        const size_t d1 = (size_t)(d1p - umi1);
        const char *d2p = (const char *)std::memchr(umi1 + d1 + 1, '-', l1 - d1 - 1);
        const size_t e2 = d2p ? (size_t)(d2p - umi1) : l1;
        umi2.assign(umi1 + d1 + 1, e2 - d1 - 1);
        umi2 += '-';
        umi2.append(umi1, d1);
        for (size_t i = 0; i < n; ++i) {
            const Rec *r = fr[i];
            if (r->rx_type != 'Z') { msg = "RX tag is not a string"; return DCR_ERR_ATTRIBUTE; }
            const char *x = rx_at(*r);
            const bool eq1 = r->l_rx == l1 && std::memcmp(x, umi1, l1) == 0;
            const bool eq2 = !eq1 && r->l_rx == umi2.size() && std::memcmp(x, umi2.data(), r->l_rx) == 0;
            if (!eq1 && !eq2) {
                msg = "ERROR: family " + std::string(code_at(r0), r0.l_code) +
                      " has different UMI tags. \n Please check output file of previous step of the pipeline "
                      "(fgbio GroupReadsByUmi)";
                return DCR_ERR_EXIT;
            }
        }
        for (size_t i = 1; i < n; ++i)
            if (fr[i]->tid != r0.tid) {
                msg = "ERROR: family " + std::string(code_at(r0), r0.l_code) +
                      " has difference rnames (e.g. chromosome numbers). \n Please check output file of previous "
                      "step of the pipeline (fgbio GroupReadsByUmi)";
                return DCR_ERR_EXIT;
            }
        return DCR_ERR_NONE;
    }

    std::vector<const Rec *> sub[4];

    // preprocess_family up to the read loop (:1248-1264), then pack or file
    // the family.  Returns 1 done, 0 no room in this batch (nothing changed),
    // -1 the reference stops at this family (batch error set).
    int complete_family() {
        dcr_host_batch *b = hb;
        const Rec &r0 = *fam.front();
        const char *code = code_of(r0);
        const size_t l_code = r0.l_code;
        // capacity check first, with the unsampled family as the bound
        int64_t nb = 0, nc = 0, filt_bytes = 0;
        for (const Rec *r : fam) { nb += r->l_seq; nc += r->n_cig; filt_bytes += r->len; }
        const int64_t nfam_reads = (int64_t)fam.size();
        const int64_t names_need = (int64_t)l_code + 1 + 2 * (int64_t)(r0.l_rx + 1) + 64 * 2;
        const bool fits = b->n_tab < b->cap_tab && b->n_fam < b->cap_fam &&
                          b->n_reads + nfam_reads <= b->cap_reads && b->n_bases + nb <= b->cap_bases &&
                          b->n_cigar + nc <= b->cap_cigar && b->n_names + names_need <= b->cap_names &&
                          b->n_side_filt + filt_bytes <= b->cap_side;
        if (!fits) {
            if (b->n_tab == 0 && b->n_side_exc == 0)
                return fail_capacity("one family exceeds the batch capacities");
            return 0;
        }
        {
            std::string msg;
            const int kind = check_family(RecList{fam.data(), nullptr}, fam.size(), wb, umi2_, msg);
            if (kind != DCR_ERR_NONE) return stop(kind, msg);
        }
        // split_family (:132-154), the subfamily of each read from parse_at
        for (auto &sv : sub) sv.clear();
        for (const Rec *r : fam)
            if (r->subk >= 0) sub[r->subk].push_back(r);
        // check_number_reads (:157-188)
        int sampled = 0;
        bool enough = true;
        for (int k = 0; k < 4; ++k) {
            const int n = (int)sub[k].size();
            if (n < cfg.min_reads) { enough = false; break; }
            if (n > cfg.max_reads) {
                if (cfg.max_reads < 0) return stop(DCR_ERR_VALUE, "Sample larger than population or is negative");
                if (gate_fn && !gate_open) {
                    gate_open = true;
                    if (gate_fn(gate_user, rng.mt, &rng.index) != 0 || rng.index < 0 || rng.index > 624)
                    {
                        g_err = "the state gate gave no generator state";
                        return -1;
                    }
                }
                rng.sample(n, cfg.max_reads, idx_tmp);
                sample_calls.push_back(n);
                sample_calls.push_back(cfg.max_reads);
                std::vector<const Rec *> pick;
                pick.reserve(idx_tmp.size());
                for (int j : idx_tmp) pick.push_back(sub[k][(size_t)j]);
                sub[k].swap(pick);
                sampled |= 1 << k;
            }
        }
        const int32_t t = b->n_tab++;
        b->tab_sampled[t] = sampled;
        b->tab_exc_cut[t] = b->n_side_exc;
        b->tab_filt_cut[t] = b->n_side_filt;
        b->tab_code[t] = put_name(code, l_code);
        const int64_t code_off = b->tab_code[t];
        if (!enough) {
            // filtered family: its reads to _filteredfamilies.bam in input order (:1550-1551)
            b->tab_kind[t] = DCR_FAM_FILTERED;
            b->tab_proc[t] = -1;
            for (const Rec *r : fam) {
                std::memcpy(b->side_filt + b->n_side_filt, at(*r, 0), r->len);
                b->n_side_filt += r->len;
            }
            ++filtered;
            return 1;
        }
        // pack
        const int32_t f = b->n_fam++;
        b->tab_kind[t] = DCR_FAM_PROCESSED;
        b->tab_proc[t] = f;
        b->fam_tid[f] = r0.tid;
        b->fam_code[f] = code_off;
        int64_t mn[4], mx[4];
        for (int k = 0; k < 4; ++k) {
            int16_t eqx = 0;
            mn[k] = mx[k] = 0;
            bool first = true;
            for (const Rec *rp : sub[k]) {
                const Rec &r = *rp;
                const int32_t i = b->n_reads++;
                jobs.push_back(Job{r.off, b->n_bases, b->n_cigar, i});
                b->n_bases += r.l_seq;
                b->n_cigar += r.n_cig;
                const int64_t end = r.end_kept;
                if (first || r.pos < mn[k]) mn[k] = r.pos;
                if (first || end > mx[k]) mx[k] = end;
                first = false;
                if (eqx < 0x7fff && r.eqx) ++eqx;
            }
            b->fam_eqx[4 * f + k] = (uint16_t)eqx;
            b->sub_off[4 * f + k + 1] = b->n_reads;
            const int64_t tt = (std::max<int64_t>(mx[k] - mn[k], 1) + 15) & ~(int64_t)15;
            b->ss_col_off[4 * f + k + 1] = b->ss_col_off[4 * f + k] + tt;
        }
        for (int j = 0; j < 2; ++j) {
            const int a = 2 * j, c = 2 * j + 1;
            int64_t tt = std::max(mx[a], mx[c]) - std::min(mn[a], mn[c]);
            tt = (std::max<int64_t>(tt, 1) + 15) & ~(int64_t)15;
            b->ds_col_off[2 * f + j + 1] = b->ds_col_off[2 * f + j] + tt;
        }
        b->ss_cols = b->ss_col_off[4 * f + 4];
        b->ds_cols = b->ds_col_off[2 * f + 2];
        // writer metadata: RX of the read0 of A1 and of B1 (:1367 via add_tags)
        for (int j = 0; j < 2; ++j) {
            const std::vector<const Rec *> &sv = sub[2 * j];
            if (sv.empty()) b->fam_rx[2 * f + j] = put_name("", 0);
            else b->fam_rx[2 * f + j] = put_name((const char *)at(*sv[0], sv[0]->o_rx), sv[0]->l_rx);
        }
        ++processed;
        return 1;
    }

    int64_t put_name(const char *s, size_t n) {
        const int64_t o = hb->n_names;
        std::memcpy(hb->names + o, s, n);
        hb->names[o + (int64_t)n] = 0;
        hb->n_names += (int64_t)n + 1;
        return o;
    }

    int stop(int kind, const std::string &msg) {
        hb->end_kind = DCR_END_ERROR;
        hb->err_kind = kind;
        std::snprintf(hb->err_msg, sizeof hb->err_msg, "%s", msg.c_str());
        errored = true;
        return -1;
    }
    int cap_err = 0;
    int fail_capacity(const std::string &m) {
        g_err = m;
        cap_err = 1;
        return -1;
    }

    // -- one batch ----------------------------------------------------------------
    int next(dcr_host_batch *b) {
        hb = b;
        b->n_fam = b->n_reads = 0;
        b->n_cigar = b->n_bases = b->ss_cols = b->ds_cols = 0;
        b->n_tab = 0;
        b->end_kind = DCR_END_FULL;
        b->n_names = b->n_side_exc = b->n_side_filt = 0;
        b->err_kind = DCR_ERR_NONE;
        b->err_msg[0] = 0;
        b->sub_off[0] = 0;
        b->ss_col_off[0] = 0;
        b->ds_col_off[0] = 0;
        cap_err = 0;
        if (jobs.capacity() < (size_t)b->cap_reads) jobs.reserve((size_t)b->cap_reads);
        // the queued families never reallocate under the packer (queue_family
        // drains them first when they would)
        if (tasks.capacity() < (size_t)b->cap_tab) tasks.reserve((size_t)b->cap_tab);
        if (pend_recs.capacity() < (size_t)b->cap_reads) pend_recs.reserve((size_t)b->cap_reads);
        if (errored || finished) {
            b->end_kind = errored ? DCR_END_ERROR : DCR_END_EOF;
            return fail(DCR_IO_EARG, "the input has already ended");
        }
        const double tw = prof.on ? IngestProf::now() : 0;
        int rc = walk();
        if (flush_tasks() < 0 && rc >= 0) rc = -1;
        flush_jobs();
        if (prof.on) prof.walk_total += IngestProf::now() - tw;
        hb = nullptr;
        if (rc < 0) {
            if (cap_err) return DCR_IO_ECAPACITY;
            if (!errored) return DCR_IO_EFORMAT;
        }
        return DCR_IO_OK;
    }

    int walk() {
        dcr_host_batch *b = hb;
        for (;;) {
            if (rq_pos == rq_n) {
                const int st = prefetch_records();
                if (st < 0) return -1;
                if (st == 0) {
                    // end of input: the last family (:1610-1631)
                    if (!started && !mid_end) return stop(DCR_ERR_TYPE, "'NoneType' object is not subscriptable");
                    if (!fam.empty()) {
                        const int c = queue_family();
                        if (c <= 0) return c;
                        fam.clear();
                    }
                    finished = true;
                    b->end_kind = DCR_END_EOF;
                    return 1;
                }
            }
            const Rec &r = rqp[rq_pos];
            // a record that stops the reference comes after every queued
            // family: their checks first
            if ((r.perr || r.pf < 0 || (r.pf > 0 && r.mi_type != 'Z')) && flush_tasks() < 0) return -1;
            if (r.perr) { g_err = kParseErr[r.perr]; return -1; }
            if (r.pf < 0) return stop(kFilterMsg[r.fmsg].kind, kFilterMsg[r.fmsg].msg);
            if (r.pf == 0) {
                // excluded read -> _filteredreads.bam (:1523-1528)
                if (b->n_side_exc + r.len > b->cap_side) {
                    if (b->n_tab == 0 && b->n_side_exc == 0) return fail_capacity("a record exceeds cap_side");
                    return 1;
                }
                std::memcpy(b->side_exc + b->n_side_exc, at(r, 0), r.len);
                b->n_side_exc += r.len;
                ++excluded;
                ++records;
                wpos = r.off + r.len;
                ++rq_pos;
                continue;
            }
            if (r.mi_type != 'Z') return stop(DCR_ERR_ATTRIBUTE, "'int' object has no attribute 'split'");
            if (!fam.empty() && !same_code(r, *fam.front())) {
                const double tc = prof.on ? IngestProf::now() : 0;
                const int c = queue_family();
                if (prof.on) prof.complete += IngestProf::now() - tc;
                if (c <= 0) return c;      // 0: batch full, the read stays unconsumed
                fam.clear();
                kick_tasks(false);
                kick_jobs(false);
            }
            ++passed;
            ++records;
            started = true;
            fam.push_back(&r);
            wpos = r.off + r.len;
            ++rq_pos;
        }
    }
};

// ---------------------------------------------------------------------------
// Split points for family-range sharding (dcr_split_points).
namespace {

// a BGZF block header at h (avail bytes): 1f 8b 08 04, XLEN 6, "BC" 2 BSIZE
bool bgzf_header(const uint8_t *h, size_t avail, size_t &blen) {
    if (avail < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4) return false;
    if (rd16(h + 10) != 6 || h[12] != 'B' || h[13] != 'C' || rd16(h + 14) != 2) return false;
    blen = (size_t)rd16(h + 16) + 1;
    return blen >= 26;
}

struct SplitReader {
    FILE *f = nullptr;
    uint64_t fsize = 0;
    libdeflate_decompressor *dec = libdeflate_alloc_decompressor();
    std::vector<uint8_t> data;                         // inflated bytes of consecutive blocks
    std::vector<std::pair<uint64_t, size_t>> blocks;   // (file offset, start in data)
    uint64_t next = 0;                                 // file offset of the next block to read
    ~SplitReader() { libdeflate_free_decompressor(dec); }

    bool read_at(uint64_t off, uint8_t *dst, size_t n) {
        if (std::fseek(f, (long)off, SEEK_SET) != 0) return false;
        return std::fread(dst, 1, n, f) == n;
    }
    // first block start at or after target: a header followed by another one
    // (or the end of the file) at its BSIZE
    bool find_block(uint64_t target, uint64_t &out) {
        std::vector<uint8_t> w(1 << 18);
        for (uint64_t base = target; base < fsize; base += w.size() - 32) {
            const size_t n = (size_t)std::min<uint64_t>(w.size(), fsize - base);
            if (!read_at(base, w.data(), n)) return false;
            for (size_t j = 0; j + 18 <= n; ++j) {
                size_t blen;
                if (!bgzf_header(w.data() + j, n - j, blen)) continue;
                const uint64_t nx = base + j + blen;
                if (nx == fsize) { out = base + j; return true; }
                uint8_t h2[18];
                size_t b2;
                if (nx + 18 <= fsize && read_at(nx, h2, 18) && bgzf_header(h2, 18, b2)) { out = base + j; return true; }
            }
            if (n < w.size()) break;
        }
        return false;
    }
    // append the next block's data; false at the end of the file or on error
    bool more() {
        if (next >= fsize) return false;
        uint8_t h[18];
        size_t blen;
        if (!read_at(next, h, 18) || !bgzf_header(h, 18, blen) || next + blen > fsize) return false;
        std::vector<uint8_t> cb(blen);
        if (!read_at(next, cb.data(), blen)) return false;
        const uint32_t isize = rd32(cb.data() + blen - 4);
        if (isize > 0x10000) return false;
        const size_t at = data.size();
        data.resize(at + isize);
        size_t got = 0;
        if (isize && (libdeflate_deflate_decompress(dec, cb.data() + 18, blen - 26, data.data() + at, isize, &got) != 0 ||
                      got != isize))
            return false;
        blocks.emplace_back(next, at);
        next += blen;
        return true;
    }
    bool have(size_t n) {
        while (data.size() < n)
            if (!more()) return false;
        return true;
    }
    int64_t voff(size_t pos) const {
        for (size_t k = blocks.size(); k-- > 0;) {
            const size_t end = k + 1 < blocks.size() ? blocks[k + 1].second : data.size();
            if (blocks[k].second <= pos && pos < end) return (int64_t)((blocks[k].first << 16) | (pos - blocks[k].second));
        }
        return -1;
    }
};

// a plausible BAM record at o (every field, the read name and the aux
// fields up to exactly block_size); next = the following record
bool record_ok(SplitReader &rd, size_t o, int32_t n_ref, size_t &next) {
    if (!rd.have(o + 36)) return false;
    const int32_t bs = rdi32(rd.data.data() + o);
    if (bs < 32 || bs > (1 << 24) || !rd.have(o + 4 + (size_t)bs)) return false;
    const uint8_t *r = rd.data.data() + o + 4;
    const int32_t tid = rdi32(r), pos = rdi32(r + 4), l_seq = rdi32(r + 16), ntid = rdi32(r + 20), npos = rdi32(r + 24);
    const uint32_t l_rn = r[8], n_cig = rd16(r + 12);
    if (tid < -1 || tid >= n_ref || ntid < -1 || ntid >= n_ref || pos < -1 || npos < -1 || l_rn < 1 || l_seq < 0)
        return false;
    size_t p = 32 + l_rn + 4 * (size_t)n_cig + (size_t)((l_seq + 1) / 2) + (size_t)l_seq;
    if (p > (size_t)bs || r[32 + l_rn - 1] != 0) return false;
    for (uint32_t i = 0; i + 1 < l_rn; ++i)
        if (r[32 + i] < 33 || r[32 + i] > 126) return false;
    while (p < (size_t)bs) {
        if (p + 3 > (size_t)bs) return false;
        const uint8_t t0 = r[p], t1 = r[p + 1], ty = r[p + 2];
        if (!std::isalpha(t0) || !std::isalnum(t1)) return false;
        size_t v = p + 3, e;
        switch (ty) {
            case 'A': case 'c': case 'C': e = v + 1; break;
            case 's': case 'S': e = v + 2; break;
            case 'i': case 'I': case 'f': e = v + 4; break;
            case 'Z': case 'H': {
                const void *z = std::memchr(r + v, 0, (size_t)bs - v);
                if (!z) return false;
                e = (size_t)((const uint8_t *)z - r) + 1;
                break;
            }
            case 'B': {
                if (v + 5 > (size_t)bs) return false;
                const uint8_t sub = r[v];
                const size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 :
                                  (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
                if (!es) return false;
                e = v + 5 + es * (size_t)rd32(r + v + 1);
                break;
            }
            default: return false;
        }
        if (e > (size_t)bs) return false;
        p = e;
    }
    next = o + 4 + (size_t)bs;
    return true;
}

}  // namespace

extern "C" {

int dcr_io_abi_version(void) { return DCR_IO_ABI_VERSION; }

int dcr_io_set_inflate_hook(const dcr_inflate_hook *hook) {
    std::lock_guard<std::mutex> g(g_hook_mu);
    if (hook && hook->run) {
        g_hook = *hook;
        g_hook_set = true;
    } else {
        g_hook = dcr_inflate_hook{};
        g_hook_set = false;
    }
    return DCR_IO_OK;
}

int dcr_ingest_gpu_inflate(dcr_ingest *ing) { return ing && ing->infl && ing->infl->gpu() ? 1 : 0; }
const char *dcr_io_last_error(void) { return g_err.c_str(); }

static dcr_ingest *open_impl(const char *path, const dcr_ingest_cfg *cfg, bool ranged, int64_t start_voff,
                             int64_t end_voff) {
    if (!path || !cfg) { g_err = "NULL argument"; return nullptr; }
    FILE *f = std::fopen(path, "rb");
    if (!f) { g_err = std::string("cannot open ") + path; return nullptr; }
    std::unique_ptr<dcr_ingest> ing(new dcr_ingest);
    ing->f = f;
    ing->cfg = *cfg;
    // the scanner's and the pack copy's pools get half the threads: the three
    // pools run at once, and beyond the process's CPU share (16 on the GPU
    // box) their threads only preempt the serial stages (inflate thread,
    // walk) and draw quota throttling (profiles/r02pool: 192-194 -> 217-224 M
    // consensus bases/s with 8 + 8 instead of 16 + 16)
    ing->pool = PoolCache::get().take(env_threads("DCR_PACK_THREADS", std::max(1, pick_threads(cfg->n_threads) / 2)));
    ing->ppool = PoolCache::get().take(std::max(1, std::min(4, pick_threads(cfg->n_threads) / 4)));
    ing->pk_start_thread();
    ing->rp.min_map_quality = cfg->min_map_quality;
    ing->rp.min_base_quality = cfg->min_base_quality;
    const int64_t end_coff = end_voff >= 0 ? (end_voff >> 16) : -1;
    const uint32_t end_uoff = end_voff >= 0 ? (uint32_t)(end_voff & 0xffff) : 0;
    ing->mid_end = end_voff >= 0;
    ing->infl.reset(new Inflater(f, pick_threads(cfg->n_threads), ing->rp, ranged, (uint64_t)start_voff >> 16,
                                 (uint32_t)(start_voff & 0xffff), end_coff, end_uoff,
                                 (cfg->flags & DCR_INGEST_HOST_INFLATE) != 0));
    // seed like an unseeded random.Random is not reproducible; callers pass
    // their state with dcr_ingest_set_rng.  Default: random.seed(0).
    for (int i = 0; i < 624; ++i) ing->rng.mt[i] = 0;
    ing->rng.index = 624;
    if (ranged) {
        // the range starts on a record boundary start_uoff bytes into its first block
        const size_t skip = (size_t)(start_voff & 0xffff);
        const int st = ing->need(skip + 4);
        if (st < 0) return nullptr;
        if (st > 0) ing->wpos += skip;
        else ing->wpos = ing->wend;       // an empty range
        return ing.release();
    }
    // header: magic, l_text, text, n_ref, refs
    int st = ing->need(12);
    if (st <= 0) { if (st == 0) g_err = "empty BAM"; return nullptr; }
    const uint8_t *h = ing->wb + ing->wpos;
    if (std::memcmp(h, "BAM\1", 4) != 0) { g_err = "not a BAM file"; return nullptr; }
    const int32_t l_text = rdi32(h + 4);
    if (l_text < 0 || ing->need(12 + (size_t)l_text) <= 0) { g_err = "truncated BAM header"; return nullptr; }
    size_t p = 8 + (size_t)l_text;
    const int32_t n_ref = rdi32(ing->wb + ing->wpos + p);
    p += 4;
    for (int32_t i = 0; i < n_ref; ++i) {
        if (ing->need(p + 4) <= 0) { g_err = "truncated BAM header"; return nullptr; }
        const int32_t ln = rdi32(ing->wb + ing->wpos + p);
        if (ln < 0 || ing->need(p + 8 + (size_t)ln) <= 0) { g_err = "truncated BAM header"; return nullptr; }
        p += 8 + (size_t)ln;
    }
    ing->header.assign(ing->wb + ing->wpos, ing->wb + ing->wpos + p);
    ing->wpos += p;
    return ing.release();
}

dcr_ingest *dcr_ingest_open(const char *path, const dcr_ingest_cfg *cfg) { return open_impl(path, cfg, false, 0, -1); }

dcr_ingest *dcr_ingest_open_range(const char *path, const dcr_ingest_cfg *cfg, int64_t start_voff, int64_t end_voff) {
    return open_impl(path, cfg, start_voff != 0, start_voff, end_voff);
}

int dcr_split_points(const char *path, int32_t n_parts, const dcr_ingest_cfg *cfg, int64_t *voff) {
    if (!path || !cfg || n_parts < 1 || (n_parts > 1 && !voff)) return fail(DCR_IO_EARG, "bad arguments");
    for (int32_t i = 0; i + 1 < n_parts; ++i) voff[i] = -1;
    if (n_parts == 1) return DCR_IO_OK;
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(DCR_IO_EARG, std::string("cannot open ") + path);
    struct Closer { FILE *f; ~Closer() { std::fclose(f); } } closer{f};
    std::fseek(f, 0, SEEK_END);
    const uint64_t fsize = (uint64_t)std::ftell(f);
    // n_ref from the header
    int32_t n_ref = 0;
    {
        SplitReader rd;
        rd.f = f;
        rd.fsize = fsize;
        if (!rd.have(12) || std::memcmp(rd.data.data(), "BAM\1", 4) != 0) return fail(DCR_IO_EFORMAT, "not a BAM file");
        const size_t l_text = (size_t)rdi32(rd.data.data() + 4);
        if (!rd.have(12 + l_text)) return fail(DCR_IO_EFORMAT, "truncated BAM header");
        n_ref = rdi32(rd.data.data() + 8 + l_text);
    }
    RecParser rp;
    rp.min_map_quality = cfg->min_map_quality;
    rp.min_base_quality = cfg->min_base_quality;
    int64_t last = 0;
    for (int32_t part = 1; part < n_parts; ++part) {
        SplitReader rd;
        rd.f = f;
        rd.fsize = fsize;
        uint64_t b0;
        if (!rd.find_block(fsize * (uint64_t)part / (uint64_t)n_parts, b0) || b0 == 0) continue;
        rd.next = b0;
        // a record boundary: eight consecutive plausible records
        size_t c = SIZE_MAX;
        for (size_t o = 0; o < 0x20000 && rd.have(o + 36); ++o) {
            size_t q = o, nx;
            int k = 0;
            while (k < 8 && record_ok(rd, q, n_ref, nx)) { q = nx; ++k; }
            if (k == 8) { c = o; break; }
        }
        if (c == SIZE_MAX) continue;
        // then the first passing read whose code differs from the passing read before it
        std::string prev;
        bool have_prev = false;
        size_t found = SIZE_MAX;
        for (size_t o = c, nx; o < ((size_t)64 << 20); o = nx) {
            if (!record_ok(rd, o, n_ref, nx)) break;
            Rec r;
            if (rp.parse_at(rd.data.data(), o, r) != 0 || r.pf < 0) break;   // the reference stops here: no split
            if (r.pf == 0) continue;
            if (r.mi_type != 'Z') break;
            const char *cp = r.l_code <= sizeof r.code ? r.code : (const char *)rd.data.data() + o + r.o_mi;
            const std::string code(cp, r.l_code);
            if (have_prev && code != prev) { found = o; break; }
            prev = code;
            have_prev = true;
        }
        if (found == SIZE_MAX) continue;
        const int64_t v = rd.voff(found);
        if (v > last) {
            voff[part - 1] = v;
            last = v;
        }
    }
    return DCR_IO_OK;
}

int64_t dcr_bam_header(const char *path, uint8_t *out, int64_t cap) {
    if (!path) { g_err = "NULL argument"; return -1; }
    FILE *f = std::fopen(path, "rb");
    if (!f) { g_err = std::string("cannot open ") + path; return -1; }
    struct Closer { FILE *f; ~Closer() { std::fclose(f); } } closer{f};
    SplitReader rd;
    rd.f = f;
    std::fseek(f, 0, SEEK_END);
    rd.fsize = (uint64_t)std::ftell(f);
    if (!rd.have(12) || std::memcmp(rd.data.data(), "BAM\1", 4) != 0) { g_err = "not a BAM file"; return -1; }
    const int32_t l_text = rdi32(rd.data.data() + 4);
    if (l_text < 0 || !rd.have(12 + (size_t)l_text)) { g_err = "truncated BAM header"; return -1; }
    size_t p = 8 + (size_t)l_text;
    const int32_t n_ref = rdi32(rd.data.data() + p);
    p += 4;
    for (int32_t i = 0; i < n_ref; ++i) {
        if (!rd.have(p + 4)) { g_err = "truncated BAM header"; return -1; }
        const int32_t ln = rdi32(rd.data.data() + p);
        if (ln < 0 || !rd.have(p + 8 + (size_t)ln)) { g_err = "truncated BAM header"; return -1; }
        p += 8 + (size_t)ln;
    }
    if (out && (int64_t)p <= cap) std::memcpy(out, rd.data.data(), p);
    return (int64_t)p;
}

int64_t dcr_ingest_sample_calls(dcr_ingest *ing, int32_t *out, int64_t cap) {
    if (!ing) return -1;
    const int64_t n = (int64_t)ing->sample_calls.size() / 2;
    if (out)
        for (int64_t i = 0; i < std::min(n, cap); ++i) {
            out[2 * i] = ing->sample_calls[(size_t)(2 * i)];
            out[2 * i + 1] = ing->sample_calls[(size_t)(2 * i + 1)];
        }
    return n;
}

int dcr_py_replay(uint32_t *mt, int32_t *index, const int32_t *calls, int64_t n_calls) {
    if (!mt || !index || (n_calls > 0 && !calls) || *index < 0 || *index > 624) return fail(DCR_IO_EARG, "bad arguments");
    PyRandom r;
    std::memcpy(r.mt, mt, sizeof r.mt);
    r.index = *index;
    std::vector<int> v;
    for (int64_t i = 0; i < n_calls; ++i) {
        const int n = calls[2 * i], k = calls[2 * i + 1];
        if (n < 0 || k < 0 || k > n) return fail(DCR_IO_EARG, "bad sample call");
        r.sample(n, k, v);
    }
    std::memcpy(mt, r.mt, sizeof r.mt);
    *index = r.index;
    return DCR_IO_OK;
}

void dcr_ingest_close(dcr_ingest *ing) { delete ing; }

int64_t dcr_ingest_header(dcr_ingest *ing, const uint8_t **bytes) {
    if (!ing || !bytes) return -1;
    *bytes = ing->header.data();
    return (int64_t)ing->header.size();
}

int dcr_ingest_set_rng(dcr_ingest *ing, const uint32_t *mt, int32_t index) {
    if (!ing || !mt || index < 0 || index > 624) return fail(DCR_IO_EARG, "bad RNG state");
    std::memcpy(ing->rng.mt, mt, sizeof ing->rng.mt);
    ing->rng.index = index;
    return DCR_IO_OK;
}

int dcr_ingest_get_rng(dcr_ingest *ing, uint32_t *mt, int32_t *index) {
    if (!ing || !mt || !index) return fail(DCR_IO_EARG, "NULL argument");
    std::memcpy(mt, ing->rng.mt, sizeof ing->rng.mt);
    *index = ing->rng.index;
    return DCR_IO_OK;
}

int dcr_ingest_set_state_gate(dcr_ingest *ing, dcr_state_gate_fn fn, void *user) {
    if (!ing) return fail(DCR_IO_EARG, "NULL argument");
    ing->gate_fn = fn;
    ing->gate_user = user;
    ing->gate_open = false;
    return DCR_IO_OK;
}

int dcr_ingest_next(dcr_ingest *ing, dcr_host_batch *hb) {
    if (!ing || !hb) return fail(DCR_IO_EARG, "NULL argument");
    if (hb->cap_fam < 1 || hb->cap_tab < 1 || hb->cap_reads < 1 || !hb->sub_off || !hb->names)
        return fail(DCR_IO_EARG, "batch capacities not set");
    return ing->next(hb);
}

int dcr_ingest_counters(dcr_ingest *ing, int64_t *out) {
    if (!ing || !out) return fail(DCR_IO_EARG, "NULL argument");
    out[0] = ing->passed;
    out[1] = ing->excluded;
    out[2] = ing->processed;
    out[3] = ing->filtered;
    out[4] = ing->records;
    return DCR_IO_OK;
}

int dcr_py_sample(uint32_t *mt, int32_t *index, int32_t n, int32_t k, int32_t *out) {
    if (!mt || !index || !out || n < 0 || k < 0 || k > n) return fail(DCR_IO_EARG, "bad sample arguments");
    PyRandom r;
    std::memcpy(r.mt, mt, sizeof r.mt);
    r.index = *index;
    std::vector<int> v;
    r.sample(n, k, v);
    for (int i = 0; i < k; ++i) out[i] = v[(size_t)i];
    std::memcpy(mt, r.mt, sizeof r.mt);
    *index = r.index;
    return DCR_IO_OK;
}

}  // extern "C"
