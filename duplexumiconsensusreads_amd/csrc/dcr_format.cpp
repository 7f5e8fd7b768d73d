// dcr_format.cpp — native writer side (include/dcr_io.h): the duplex
// consensus records of a batch, built from kernel outputs with the
// reference's exact field and tag layout, and a BGZF writer that deflates
// blocks on a worker pool (libdeflate).
//
// Reference (/root/reference/DuplexUMIConsensusReads.py):
//   record fields        make_consensus_read :1352-1384
//   name / flag          get_consensus_id :892-933, get_consensus_flag :936-968
//   duplex tags          add_tags(method="double_strand") :1076-1120
//   mate fields          fix_paired_end_fields :1390-1419
//   pysam typing         smallest integer type, 'f' float32, 'Z' text, 'B' arrays;
//                        sd/se text is str() of a list of numpy-1.x ints: "[1, 2]"
#include <cctype>
#include <fcntl.h>
#include <unistd.h>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/dcr.h"
#include "../../include/dcr_io.h"
#include "dcr_host.h"

using namespace dcrh;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &m) {
    g_err = m;
    return code;
}

constexpr size_t kBlockData = 0xff00;
const uint8_t kEof[28] = {0x1f, 0x8b, 0x08, 0x04, 0x00, 0x00, 0x00, 0x00, 0x00, 0xff, 0x06, 0x00, 0x42, 0x43,
                          0x02, 0x00, 0x1b, 0x00, 0x03, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00};

struct TLComp {
    libdeflate_compressor *c[13] = {};
    ~TLComp() {
        for (auto *p : c)
            if (p) libdeflate_free_compressor(p);
    }
    libdeflate_compressor *get(int level) {
        if (!c[level]) c[level] = libdeflate_alloc_compressor(level);
        return c[level];
    }
};
thread_local TLComp tl_comp;

// ASCII -> 4-bit BAM code ("=ACMGRSVTWYHKDBN", either case; unknown 15)
struct NtTable {
    uint8_t code[256];
    NtTable() {
        std::memset(code, 15, sizeof code);
        const char *a = "=ACMGRSVTWYHKDBN";
        for (int i = 0; i < 16; ++i) {
            code[(uint8_t)a[i]] = (uint8_t)i;
            code[(uint8_t)std::tolower(a[i])] = (uint8_t)i;
        }
    }
};
const NtTable kNt;

// SAM spec §5.3 bin of [beg, end)
int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

// growable byte buffer with unchecked appends after reserve()
struct Buf {
    std::vector<uint8_t> v;
    size_t n = 0;
    void reserve(size_t more) {
        if (n + more > v.size()) v.resize(std::max(v.size() * 2, n + more + (1 << 20)));
    }
    uint8_t *p() { return v.data() + n; }
    void b(uint8_t x) { v[n++] = x; }
    void raw(const void *s, size_t k) { std::memcpy(v.data() + n, s, k); n += k; }
    void u16(uint32_t x) { wr16(p(), x); n += 2; }
    void u32(uint32_t x) { wr32(p(), x); n += 4; }
    void str(const char *s) { raw(s, std::strlen(s)); }
    void uint(uint32_t x) {
        char t[12];
        int k = 0;
        do { t[k++] = (char)('0' + x % 10); x /= 10; } while (x);
        while (k) v[n++] = (uint8_t)t[--k];
    }
    void sint(int64_t x) {
        if (x < 0) { v[n++] = '-'; x = -x; }
        char t[24];
        int k = 0;
        do { t[k++] = (char)('0' + x % 10); x /= 10; } while (x);
        while (k) v[n++] = (uint8_t)t[--k];
    }
};

// pysam's type code for an untyped int tag value (>= 0 here)
void int_tag(Buf &o, const char *tag, int64_t v) {
    o.raw(tag, 2);
    if (v < 0) {
        if (v >= -128) { o.b('c'); o.b((uint8_t)(int8_t)v); }
        else if (v >= -32768) { o.b('s'); o.u16((uint32_t)(uint16_t)(int16_t)v); }
        else { o.b('i'); o.u32((uint32_t)(int32_t)v); }
    } else if (v <= 255) { o.b('C'); o.b((uint8_t)v); }
    else if (v <= 65535) { o.b('S'); o.u16((uint32_t)v); }
    else { o.b('I'); o.u32((uint32_t)v); }
}

void float_tag(Buf &o, const char *tag, double v) {
    o.raw(tag, 2);
    o.b('f');
    const float f = (float)v;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    o.u32(u);
}

void z_begin(Buf &o, const char *tag) { o.raw(tag, 2); o.b('Z'); }

// ", <v>" for v < 1000 as 8 bytes (length in the last byte)
struct ListTab {
    uint8_t t[1000][8];
    ListTab() {
        for (int v = 0; v < 1000; ++v) {
            char s[8] = {',', ' '};
            int n = std::snprintf(s + 2, 6, "%d", v);
            std::memcpy(t[v], s, 7);
            t[v][7] = (uint8_t)(2 + n);
        }
    }
};
const ListTab kList;

// "[1, 2, 3]" (str() of a list of numpy-1.x ints); the caller reserved
// 7 bytes per value plus slack, so the 8-byte copies may run past the text
void list_text(Buf &o, const char *tag, const uint16_t *v, int32_t n) {
    z_begin(o, tag);
    o.b('[');
    uint8_t *p = o.p();
    for (int32_t i = 0; i < n; ++i) {
        const uint32_t x = v[i];
        if (x < 1000) {
            std::memcpy(p, kList.t[x], 8);
            p += kList.t[x][7];
        } else {
            p[0] = ','; p[1] = ' ';
            p += 2 + std::snprintf((char *)p + 2, 8, "%u", x);
        }
    }
    if (n) {                                   // drop the first ", "
        const size_t len = (size_t)(p - o.p());
        std::memmove(o.p(), o.p() + 2, len - 2);
        p -= 2;
    }
    o.n = (size_t)(p - o.v.data());
    o.b(']');
    o.b(0);
}

void phred_text(Buf &o, const char *tag, const uint8_t *q, int32_t n) {
    z_begin(o, tag);
    uint8_t *p = o.p();
    for (int32_t i = 0; i < n; ++i) p[i] = (uint8_t)(q[i] + 33);
    o.n += (size_t)n;
    o.b(0);
}

// B:C array of uint8 values (pysam infers 'C' for ints in 0..255)
void u8_array(Buf &o, const char *tag, const uint8_t *v, int32_t n) {
    o.raw(tag, 2);
    o.b('B');
    o.b('C');
    o.u32((uint32_t)n);
    o.raw(v, (size_t)n);
}


struct Ctx {
    const dcr_host_batch *hb;
    const dcr_fmt_out *ss, *ds;
};

// one BGZF block of in[0, len) (len <= 0xff00) at out (>= 64 KiB); returns its size
size_t bgzf_block(const uint8_t *in, size_t len, int level, uint8_t *out) {
    size_t clen = libdeflate_deflate_compress(tl_comp.get(level), in, len, out + 18, 0x10000 - 26);
    if (clen == 0) clen = libdeflate_deflate_compress(tl_comp.get(0), in, len, out + 18, 0x10000 - 26);
    if (clen == 0) return 0;
    out[0] = 0x1f; out[1] = 0x8b; out[2] = 8; out[3] = 4;
    wr32(out + 4, 0); out[8] = 0; out[9] = 0xff;
    wr16(out + 10, 6); out[12] = 66; out[13] = 67; wr16(out + 14, 2);
    wr16(out + 16, (uint32_t)(clen + 25));
    wr32(out + 18 + clen, libdeflate_crc32(0, in, len));
    wr32(out + 22 + clen, (uint32_t)len);
    return clen + 26;
}

}  // namespace

struct dcr_bgzw {
    FILE *f = nullptr;
    int level = 6;
    // the pool and the pending buffer are made on first use: the side-file
    // writers of most runs never write a record
    int n_threads = 0;
    std::unique_ptr<Pool> pool;
    std::unique_ptr<uint8_t[]> in;   // pending uncompressed bytes [in_cap]
    size_t in_cap = 0, n_in = 0;
    Pool &pl() {
        if (!pool) pool.reset(new Pool(pick_threads(n_threads)));
        return *pool;
    }
    std::vector<std::vector<uint8_t>> out;
    std::vector<size_t> out_len;
    int64_t bytes_in = 0, bytes_out = 0;
    bool bad = false;

    // deflate in[0, n) as blocks of 0xff00 bytes on the pool, write in order
    bool flush(size_t n) {
        const size_t nb = (n + kBlockData - 1) / kBlockData;
        if (out.size() < nb) { out.resize(nb); out_len.resize(nb); }
        const int lvl = level;
        auto one = [&](size_t i) {
            const size_t off = i * kBlockData, len = std::min(kBlockData, n - off);
            std::vector<uint8_t> &o = out[i];
            if (o.size() < 0x10000) o.resize(0x10000);
            out_len[i] = bgzf_block(in.get() + off, len, lvl, o.data());
            return out_len[i] != 0;
        };
        bool ok = true;
        if (nb == 1) ok = one(0);            // a header, a short tail: no pool needed
        else ok = pl().run(nb, one);
        if (!ok) { g_err = "BGZF block failed to deflate"; return false; }
        for (size_t i = 0; i < nb; ++i) {
            if (std::fwrite(out[i].data(), 1, out_len[i], f) != out_len[i]) { g_err = "write failed"; return false; }
            bytes_out += (int64_t)out_len[i];
        }
        bytes_in += (int64_t)n;
        return true;
    }
    bool put_compressed(const uint8_t *s, size_t n, size_t raw) {
        if (std::fwrite(s, 1, n, f) != n) { g_err = "write failed"; return false; }
        bytes_out += (int64_t)n;
        bytes_in += (int64_t)raw;
        return true;
    }
    bool write(const uint8_t *s, size_t n) {
        if (n && !in_cap) {
            in_cap = kBlockData * (size_t)std::max(64, 8 * pick_threads(n_threads));
            in.reset(new uint8_t[in_cap]);
        }
        while (n > 0) {
            const size_t k = std::min(in_cap - n_in, n);
            std::memcpy(in.get() + n_in, s, k);
            n_in += k; s += k; n -= k;
            if (n_in == in_cap) {
                if (!flush(n_in)) return false;
                n_in = 0;
            }
        }
        return true;
    }
};

namespace {

// one duplex record (pe j of processed family f)
void format_record(const Ctx &c, int32_t f, int j, const char *code, size_t l_code, Buf &o) {
    const dcr_host_batch *hb = c.hb;
    const dcr_fmt_out *ss = c.ss, *ds = c.ds;
    const int32_t k = 2 * f + j, a = 4 * f + 2 * j, b = a + 1;
    const int32_t pos = ds->pos[k], opos = ds->pos[2 * f + 1 - j];
    const int32_t len = ds->len[k];
    const int32_t tlen = ds->pos[2 * f + 1] + ds->len[2 * f + 1] - ds->pos[2 * f];
    const int32_t tid = hb->fam_tid[f];
    const int64_t ro = hb->ds_col_off[k], ao = hb->ss_col_off[a], bo = hb->ss_col_off[b];
    const size_t rec0 = o.n;
    o.u32(0);                                        // block_size
    o.u32((uint32_t)tid);                            // reference_id = read0's (:1363)
    o.u32((uint32_t)pos);                            // reference_start (:790)
    const char *pe = j == 0 ? "_paired-end1" : "_paired-end2";
    const size_t l_rn = 16 + l_code + 12 + 1;        // "consensus_family" code pe NUL
    o.b((uint8_t)l_rn);
    o.b((uint8_t)(ds->mapq[k] & 0xff));
    int64_t rl = 0;
    const uint32_t *cg = ds->cigar + ro;
    const int32_t nc = ds->n_cig[k];
    for (int32_t i = 0; i < nc; ++i) {
        const uint32_t op = cg[i] & 15;
        if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += cg[i] >> 4;
    }
    o.u16(pos >= 0 ? (uint32_t)reg2bin(pos, pos + (rl > 0 ? rl : 1)) : 4680u);
    o.u16((uint32_t)nc);
    o.u16(j == 0 ? 99u : 147u);                      // get_consensus_flag (:959-963)
    o.u32((uint32_t)len);
    o.u32((uint32_t)tid);                            // fix_paired_end_fields (:1406-1416)
    o.u32((uint32_t)opos);
    o.u32((uint32_t)(j == 0 ? tlen : -tlen));
    o.str("consensus_family");                       // get_consensus_id (:925-933)
    o.raw(code, l_code);
    o.str(pe);
    o.b(0);
    for (int32_t i = 0; i < nc; ++i) o.u32(cg[i]);
    const uint8_t *sq = ds->seq + ro;
    for (int32_t i = 0; i + 1 < len; i += 2) o.b((uint8_t)((kNt.code[sq[i]] << 4) | kNt.code[sq[i + 1]]));
    if (len & 1) o.b((uint8_t)(kNt.code[sq[len - 1]] << 4));
    o.raw(ds->qual + ro, (size_t)len);
    // tags, in add_tags' order (:1117-1120)
    z_begin(o, "MI");
    o.raw(code, l_code);
    o.b(0);
    z_begin(o, "RX");
    o.str(hb->names + hb->fam_rx[2 * f + j]);
    o.b(0);
    const int32_t a0 = hb->sub_off[a], a1 = hb->sub_off[a + 1], b0 = hb->sub_off[b], b1 = hb->sub_off[b + 1];
    u8_array(o, "aQ", hb->read_mapq + a0, a1 - a0);
    u8_array(o, "bQ", hb->read_mapq + b0, b1 - b0);
    // cQ: the two single-strand MAPQs (ints <= 255 -> 'C')
    o.raw("cQ", 2); o.b('B'); o.b('C'); o.u32(2);
    o.b((uint8_t)ss->mapq[a]); o.b((uint8_t)ss->mapq[b]);
    list_text(o, "ad", ss->d + ao, ss->n_de[a]);
    list_text(o, "bd", ss->d + bo, ss->n_de[b]);
    list_text(o, "cd", ds->d + ro, ds->n_de[k]);
    int_tag(o, "aD", ss->D[a]); int_tag(o, "bD", ss->D[b]); int_tag(o, "cD", ds->D[k]);
    int_tag(o, "aM", ss->M[a]); int_tag(o, "bM", ss->M[b]); int_tag(o, "cM", ds->M[k]);
    list_text(o, "ae", ss->e + ao, ss->n_de[a]);
    list_text(o, "be", ss->e + bo, ss->n_de[b]);
    list_text(o, "ce", ds->e + ro, ds->n_de[k]);
    float_tag(o, "aE", ss->E[a]); float_tag(o, "bE", ss->E[b]); float_tag(o, "cE", ds->E[k]);
    z_begin(o, "ac"); o.raw(ss->seq + ao, (size_t)ss->len[a]); o.b(0);
    z_begin(o, "bc"); o.raw(ss->seq + bo, (size_t)ss->len[b]); o.b(0);
    phred_text(o, "aq", ss->qual + ao, ss->len[a]);
    phred_text(o, "bq", ss->qual + bo, ss->len[b]);
    wr32(o.v.data() + rec0, (uint32_t)(o.n - rec0 - 4));
}

size_t record_bound(const Ctx &c, int32_t f, int j, size_t l_code) {
    const int32_t k = 2 * f + j, a = 4 * f + 2 * j, b = a + 1;
    size_t n = 36 + 16 + l_code + 13 + 4 * (size_t)c.ds->n_cig[k] + (size_t)c.ds->len[k] * 2;
    n += 8 + l_code + 4 + std::strlen(c.hb->names + c.hb->fam_rx[2 * f + j]);
    n += 24 + (size_t)(c.hb->sub_off[a + 1] - c.hb->sub_off[a]) + (size_t)(c.hb->sub_off[b + 1] - c.hb->sub_off[b]);
    n += 16 + 8 * (2 * (size_t)c.ss->n_de[a] + 2 * (size_t)c.ss->n_de[b] + 2 * (size_t)c.ds->n_de[k]) + 64;
    n += 9 * 8 + 3 * 8 + 2 * ((size_t)c.ss->len[a] + c.ss->len[b]) + 32;
    return n;
}

}  // namespace

extern "C" {

dcr_bgzw *dcr_bgzw_open(const char *path, int level, int n_threads) {
    if (!path || level < 0 || level > 12) { g_err = "bad arguments"; return nullptr; }
    // truncated at open, as fopen("wb"): works for any output (a FIFO,
    // /dev/null) and a run that never reaches close leaves a short file with
    // no BGZF EOF marker, never a new prefix over an old file's tail
    const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
    FILE *f = fd >= 0 ? ::fdopen(fd, "wb") : nullptr;
    if (!f) {
        if (fd >= 0) ::close(fd);
        g_err = std::string("cannot open ") + path;
        return nullptr;
    }
    auto *w = new dcr_bgzw;
    w->f = f;
    w->level = level;
    w->n_threads = n_threads;
    return w;
}

int dcr_bgzw_write(dcr_bgzw *w, const void *bytes, int64_t n) {
    if (!w || n < 0 || (n > 0 && !bytes)) return fail(DCR_IO_EARG, "bad arguments");
    if (w->bad) return fail(DCR_IO_EFILE, "writer failed earlier");
    if (!w->write((const uint8_t *)bytes, (size_t)n)) { w->bad = true; return DCR_IO_EFILE; }
    return DCR_IO_OK;
}

int dcr_bgzw_put_blocks(dcr_bgzw *w, const void *blocks, int64_t n, int64_t raw_bytes) {
    if (!w || n < 0 || (n > 0 && !blocks)) return fail(DCR_IO_EARG, "bad arguments");
    if (w->bad) return fail(DCR_IO_EFILE, "writer failed earlier");
    if (w->n_in) {                      // pending bytes first: blocks stay in order
        if (!w->flush(w->n_in)) { w->bad = true; return DCR_IO_EFILE; }
        w->n_in = 0;
    }
    if (n && !w->put_compressed((const uint8_t *)blocks, (size_t)n, (size_t)raw_bytes)) {
        w->bad = true;
        return DCR_IO_EFILE;
    }
    return DCR_IO_OK;
}

int dcr_bgzw_close(dcr_bgzw *w) {
    if (!w) return fail(DCR_IO_EARG, "NULL writer");
    int rc = DCR_IO_OK;
    if (!w->bad && w->n_in && !w->flush(w->n_in)) rc = DCR_IO_EFILE;
    if (std::fwrite(kEof, 1, sizeof kEof, w->f) != sizeof kEof) rc = fail(DCR_IO_EFILE, "write failed");
    if (std::fflush(w->f) != 0) rc = fail(DCR_IO_EFILE, "write failed");
    if (std::fclose(w->f) != 0) rc = fail(DCR_IO_EFILE, "close failed");
    delete w;
    return rc;
}

int dcr_bgzw_sizes(dcr_bgzw *w, int64_t *out2) {
    if (!w || !out2) return fail(DCR_IO_EARG, "NULL argument");
    out2[0] = w->bytes_out;
    out2[1] = w->bytes_in + (int64_t)w->n_in;
    return DCR_IO_OK;
}

int32_t dcr_fmt_scan(const dcr_host_batch *hb, const dcr_fmt_out *ss, const dcr_fmt_out *ds,
                     const int32_t *read_status, int32_t n_fam, int32_t *kind, int32_t *which) {
    *kind = DCR_FAIL_NONE;
    *which = -1;
    auto st_fail = [](int st) { return st != 0 && st != DCR_ST_UPSTREAM && !(st & DCR_ST_PREP); };
    auto unicode = [&](int32_t s) {
        const int64_t o = hb->ss_col_off[s];
        for (int32_t i = 0; i < ss->len[s]; ++i)
            if (ss->qual[o + i] >= 95) return true;   // chr(q + 33) outside ASCII
        return false;
    };
    for (int32_t f = 0; f < n_fam; ++f) {
        // preprocess_family's read loop (:1272-1283): the first subfamily
        // holding a failing read (DCR_ST_PREP | that read's status)
        (void)read_status;
        for (int k = 0; k < 4; ++k)
            if (ss->status[4 * f + k] & DCR_ST_PREP) {
                *kind = ss->status[4 * f + k] & 0x0f;
                *which = 8 + k;
                return f;
            }
        for (int k = 0; k < 4; ++k)                   // make_consensus_read x4 (:1564-1569)
            if (st_fail(ss->status[4 * f + k])) { *kind = ss->status[4 * f + k]; *which = k; return f; }
        for (int j = 0; j < 2; ++j) {                 // x2 duplex (:1581-1582), then its set_tags (:1384)
            if (st_fail(ds->status[2 * f + j])) { *kind = ds->status[2 * f + j]; *which = 4 + j; return f; }
            if (unicode(4 * f + 2 * j) || unicode(4 * f + 2 * j + 1)) { *kind = DCR_FAIL_UNICODE; *which = 4 + j; return f; }
        }
    }
    return n_fam;
}

int dcr_fmt_write(dcr_bgzw *w, const dcr_host_batch *hb, const dcr_fmt_out *ss, const dcr_fmt_out *ds,
                  int32_t n_fam) {
    if (!w || !hb || !ss || !ds || n_fam < 0 || n_fam > hb->n_fam) return fail(DCR_IO_EARG, "bad arguments");
    if (w->bad) return fail(DCR_IO_EFILE, "writer failed earlier");
    const int64_t *code_of = hb->fam_code;
    const Ctx c{hb, ss, ds};
    // pending bytes first (blocks stay in order)
    if (w->n_in) {
        if (!w->flush(w->n_in)) { w->bad = true; return DCR_IO_EFILE; }
        w->n_in = 0;
    }
    // chunks of families, each formatted and deflated by one task into its
    // own run of BGZF blocks (a record may span blocks), written in order
    const int32_t chunk = 128;
    const int32_t nch = (n_fam + chunk - 1) / chunk;
    const int32_t group = std::max(1, 4 * w->pl().size());
    struct Task { Buf raw; std::vector<uint8_t> comp; size_t n_comp = 0; };
    std::vector<Task> tasks((size_t)std::min(nch, group));
    const int lvl = w->level;
    for (int32_t g0 = 0; g0 < nch; g0 += group) {
        const int32_t g1 = std::min(nch, g0 + group);
        const bool ok = w->pl().run((size_t)(g1 - g0), [&](size_t gi) {
            Task &t = tasks[gi];
            Buf &o = t.raw;
            o.n = 0;
            const int32_t f0 = (g0 + (int32_t)gi) * chunk, f1 = std::min(n_fam, f0 + chunk);
            for (int32_t f = f0; f < f1; ++f) {
                const char *code = hb->names + code_of[f];
                const size_t lc = std::strlen(code);
                for (int j = 0; j < 2; ++j) {
                    o.reserve(record_bound(c, f, j, lc));
                    format_record(c, f, j, code, lc, o);
                }
            }
            const size_t nb = (o.n + kBlockData - 1) / kBlockData;
            if (t.comp.size() < nb * 0x10000) t.comp.resize(nb * 0x10000);
            t.n_comp = 0;
            for (size_t b = 0; b < nb; ++b) {
                const size_t off = b * kBlockData, len = std::min(kBlockData, o.n - off);
                const size_t cl = bgzf_block(o.v.data() + off, len, lvl, t.comp.data() + t.n_comp);
                if (!cl) return false;
                t.n_comp += cl;
            }
            return true;
        });
        if (!ok) { w->bad = true; return fail(DCR_IO_EFILE, "BGZF block failed to deflate"); }
        for (int32_t gi = 0; gi < g1 - g0; ++gi)
            if (!w->put_compressed(tasks[(size_t)gi].comp.data(), tasks[(size_t)gi].n_comp, tasks[(size_t)gi].raw.n)) {
                w->bad = true;
                return DCR_IO_EFILE;
            }
    }
    return DCR_IO_OK;
}

}  // extern "C"
