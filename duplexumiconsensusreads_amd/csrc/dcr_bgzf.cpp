// Native BGZF codec (include/dcr_bgzf.h): the host-side byte stream under the
// drop-in's BAM reader and writer.  The reference gets this from htslib via
// pysam (DuplexUMIConsensusReads.py:1476, :1494-1502, :1519, :1594); here it is
// zlib raw inflate/deflate over BGZF blocks (SAM spec v1.6 §4.1), a batch of
// blocks at a time spread over host threads, consumed in file order.
#include "../../include/dcr_bgzf.h"

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

constexpr size_t kBlockData = 0xff00;      // uncompressed bytes per written block (htslib, bam.py)
constexpr size_t kMaxBlock = 0x10000;      // BSIZE + 1 never exceeds 64 KiB
const uint8_t kEof[28] = {0x1f, 0x8b, 0x08, 0x04, 0x00, 0x00, 0x00, 0x00, 0x00, 0xff, 0x06, 0x00, 0x42, 0x43,
                          0x02, 0x00, 0x1b, 0x00, 0x03, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00};

int pick_threads(int n) {
    if (n > 0) return std::min(n, 64);
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline void wr16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
inline void wr32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// Run fn(i) for i in [0, n) on up to nt threads (work taken from a shared counter).
template <class F>
bool parallel_for(int nt, size_t n, F fn) {
    std::atomic<size_t> next{0};
    std::atomic<bool> ok{true};
    auto worker = [&]() {
        for (size_t i; ok.load(std::memory_order_relaxed) && (i = next.fetch_add(1)) < n;)
            if (!fn(i)) ok = false;
    };
    int used = (int)std::min<size_t>((size_t)nt, n);
    std::vector<std::thread> pool;
    for (int t = 1; t < used; ++t) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    return ok;
}

struct Block {
    size_t coff, clen;   // compressed payload (after the header) in cbuf
    size_t doff;         // destination offset in dbuf
    uint32_t isize, crc;
};

}  // namespace

struct dcr_bgzf_reader {
    FILE* f = nullptr;
    int nt = 1;
    std::vector<uint8_t> cbuf;
    size_t cend = 0;
    bool file_eof = false;
    std::vector<uint8_t> dbuf;
    size_t dpos = 0, dend = 0;
    std::vector<Block> blocks;
    bool err = false;

    // Refill dbuf with the next batch of whole blocks; false at end of file or on error.
    bool refill() {
        if (!file_eof) {
            size_t got = fread(cbuf.data() + cend, 1, cbuf.size() - cend, f);
            cend += got;
            if (cend < cbuf.size()) file_eof = true;
        }
        blocks.clear();
        size_t p = 0, total = 0;
        while (cend - p >= 18) {
            const uint8_t* h = cbuf.data() + p;
            if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) {
                g_err = "not a BGZF file"; err = true; return false;
            }
            size_t xlen = rd16(h + 10);
            if (cend - p < 12 + xlen) break;
            long bsize = -1;
            for (size_t i = 0; i + 4 <= xlen;) {
                const uint8_t* s = h + 12 + i;
                size_t slen = rd16(s + 2);
                if (s[0] == 66 && s[1] == 67 && slen == 2) bsize = rd16(s + 4);
                i += 4 + slen;
            }
            if (bsize < 0) { g_err = "BGZF block without BC field"; err = true; return false; }
            size_t blen = (size_t)bsize + 1;
            if (blen < 12 + xlen + 8) { g_err = "BGZF block size too small"; err = true; return false; }
            if (cend - p < blen) break;
            Block b;
            b.coff = p + 12 + xlen;
            b.clen = blen - 12 - xlen - 8;
            b.crc = rd32(h + blen - 8);
            b.isize = rd32(h + blen - 4);
            b.doff = total;
            if (b.isize > kMaxBlock) { g_err = "BGZF ISIZE above 64 KiB"; err = true; return false; }
            total += b.isize;
            blocks.push_back(b);
            p += blen;
        }
        if (blocks.empty()) {
            if (cend == 0 && file_eof) return false;                   // clean end of file
            if (file_eof) { g_err = "truncated BGZF block"; err = true; return false; }
            // a single block larger than the buffer cannot happen (cbuf >= 64 KiB); read more
            return refill();
        }
        if (dbuf.size() < total) dbuf.resize(total);
        bool ok = parallel_for(nt, blocks.size(), [&](size_t i) {
            const Block& b = blocks[i];
            z_stream s{};
            if (inflateInit2(&s, -15) != Z_OK) return false;
            s.next_in = cbuf.data() + b.coff;
            s.avail_in = (uInt)b.clen;
            uint8_t dummy;
            s.next_out = b.isize ? dbuf.data() + b.doff : &dummy;   // zlib rejects a null next_out
            s.avail_out = b.isize;
            int rc = inflate(&s, Z_FINISH);
            bool good = (rc == Z_STREAM_END || (b.isize == 0 && rc == Z_BUF_ERROR)) && s.total_out == b.isize;
            inflateEnd(&s);
            if (!good) return false;
            return (b.isize ? crc32(0L, dbuf.data() + b.doff, b.isize) : 0u) == b.crc;
        });
        if (!ok) { g_err = "BGZF block failed to inflate or CRC mismatch"; err = true; return false; }
        std::memmove(cbuf.data(), cbuf.data() + p, cend - p);
        cend -= p;
        dpos = 0;
        dend = total;
        return true;
    }
};

struct dcr_bgzf_writer {
    FILE* f = nullptr;
    int nt = 1, level = 6;
    std::vector<uint8_t> in;        // pending uncompressed bytes (whole batch of blocks)
    size_t n_in = 0;
    std::vector<std::vector<uint8_t>> out;
    std::vector<size_t> out_len;

    // Compress in[0, n) as ceil(n / 0xff00) blocks in parallel, write them in order.
    bool flush(size_t n) {
        size_t nb = (n + kBlockData - 1) / kBlockData;
        if (out.size() < nb) { out.resize(nb); out_len.resize(nb); }
        bool ok = parallel_for(nt, nb, [&](size_t i) {
            size_t off = i * kBlockData, len = std::min(kBlockData, n - off);
            z_stream s{};
            if (deflateInit2(&s, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
            std::vector<uint8_t>& o = out[i];
            size_t cap = 18 + deflateBound(&s, len) + 8;
            if (o.size() < cap) o.resize(cap);
            s.next_in = in.data() + off;
            s.avail_in = (uInt)len;
            s.next_out = o.data() + 18;
            s.avail_out = (uInt)(cap - 26);
            // bam.BGZFWriter calls compressobj.compress() then flush(): the same two deflate calls
            int rc = deflate(&s, Z_NO_FLUSH);
            if (rc == Z_OK || rc == Z_BUF_ERROR) rc = deflate(&s, Z_FINISH);
            size_t clen = s.total_out;
            deflateEnd(&s);
            if (rc != Z_STREAM_END || clen + 26 > kMaxBlock) return false;
            uint8_t* h = o.data();
            h[0] = 0x1f; h[1] = 0x8b; h[2] = 8; h[3] = 4;
            wr32(h + 4, 0); h[8] = 0; h[9] = 0xff;
            wr16(h + 10, 6); h[12] = 66; h[13] = 67; wr16(h + 14, 2);
            wr16(h + 16, (uint32_t)(clen + 25));
            wr32(o.data() + 18 + clen, (uint32_t)crc32(0L, in.data() + off, (uInt)len));
            wr32(o.data() + 22 + clen, (uint32_t)len);
            out_len[i] = clen + 26;
            return true;
        });
        if (!ok) { g_err = "BGZF block failed to deflate"; return false; }
        for (size_t i = 0; i < nb; ++i)
            if (fwrite(out[i].data(), 1, out_len[i], f) != out_len[i]) { g_err = "write failed"; return false; }
        return true;
    }
};

extern "C" {

const char* dcr_bgzf_last_error(void) { return g_err.c_str(); }

dcr_bgzf_reader* dcr_bgzf_open_read(const char* path, int n_threads) {
    FILE* f = fopen(path, "rb");
    if (!f) { g_err = std::string("cannot open ") + path; return nullptr; }
    auto* r = new dcr_bgzf_reader;
    r->f = f;
    r->nt = pick_threads(n_threads);
    r->cbuf.resize(std::max<size_t>(4u << 20, (size_t)r->nt * (1u << 20)));
    return r;
}

int64_t dcr_bgzf_read(dcr_bgzf_reader* r, void* dst, int64_t n) {
    if (!r || n < 0) { g_err = "bad arguments"; return -1; }
    if (r->err) return -1;
    uint8_t* d = static_cast<uint8_t*>(dst);
    int64_t done = 0;
    while (done < n) {
        if (r->dpos == r->dend) {
            if (!r->refill()) {
                if (r->err) return -1;
                break;
            }
            continue;
        }
        size_t k = std::min<size_t>(r->dend - r->dpos, (size_t)(n - done));
        std::memcpy(d + done, r->dbuf.data() + r->dpos, k);
        r->dpos += k;
        done += (int64_t)k;
    }
    return done;
}

void dcr_bgzf_close_read(dcr_bgzf_reader* r) {
    if (!r) return;
    if (r->f) fclose(r->f);
    delete r;
}

dcr_bgzf_writer* dcr_bgzf_open_write(const char* path, int level, int n_threads) {
    if (level < 0 || level > 9) { g_err = "bad compression level"; return nullptr; }
    FILE* f = fopen(path, "wb");
    if (!f) { g_err = std::string("cannot open ") + path; return nullptr; }
    auto* w = new dcr_bgzf_writer;
    w->f = f;
    w->level = level;
    w->nt = pick_threads(n_threads);
    w->in.resize(kBlockData * (size_t)std::max(16, 8 * w->nt));
    return w;
}

int dcr_bgzf_write(dcr_bgzf_writer* w, const void* src, int64_t n) {
    if (!w || n < 0) { g_err = "bad arguments"; return -1; }
    const uint8_t* s = static_cast<const uint8_t*>(src);
    while (n > 0) {
        size_t k = std::min<size_t>(w->in.size() - w->n_in, (size_t)n);
        std::memcpy(w->in.data() + w->n_in, s, k);
        w->n_in += k; s += k; n -= (int64_t)k;
        if (w->n_in == w->in.size()) {
            if (!w->flush(w->n_in)) return -1;
            w->n_in = 0;
        }
    }
    return 0;
}

int dcr_bgzf_close_write(dcr_bgzf_writer* w) {
    if (!w) return -1;
    int rc = 0;
    if (w->n_in && !w->flush(w->n_in)) rc = -1;
    if (fwrite(kEof, 1, sizeof kEof, w->f) != sizeof kEof) rc = -1;
    if (fclose(w->f) != 0) rc = -1;
    delete w;
    return rc;
}

int64_t dcr_bam_index_records(const uint8_t* buf, int64_t n, int64_t* offs, int64_t max_recs,
                              int64_t* consumed) {
    int64_t p = 0, k = 0;
    while (k < max_recs && n - p >= 4) {
        int32_t bs = (int32_t)rd32(buf + p);
        if (bs < 0) { g_err = "negative BAM block_size"; return -1; }
        if (n - p - 4 < bs) break;
        offs[k++] = p;
        p += 4 + bs;
    }
    if (consumed) *consumed = p;
    return k;
}

}  // extern "C"
