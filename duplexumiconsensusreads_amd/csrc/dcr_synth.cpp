// dcr_synth.cpp — synthetic duplex BAM records from a packed batch
// (include/dcr_io.h dcr_synth_write): the bench's input files at 10 M+
// reads, where building records one by one in Python is too slow.
//
// Layout follows the fgbio GroupReadsByUmi output the reference expects
// (DuplexUMIConsensusReads.py:132-154, :1185-1217) and synth.family_records:
// reads of a family contiguous, subfamilies A1 B2 B1 A2 with flags 99 163 83
// 147, MI "<fam>/A" on A1/A2 and "<fam>/B" on B1/B2, RX "U1-U2" on A and
// "U2-U1" on B, read names "mol<fam>_<k>_<j>".
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dcr_io.h"
#include "dcr_host.h"

using namespace dcrh;

namespace {

struct NtCode {
    uint8_t code[256];
    NtCode() {
        std::memset(code, 15, sizeof code);
        const char *a = "=ACMGRSVTWYHKDBN";
        for (int i = 0; i < 16; ++i) code[(uint8_t)a[i]] = (uint8_t)i;
    }
};
const NtCode kCode;

int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

void put32(std::vector<uint8_t> &o, uint32_t v) {
    const size_t n = o.size();
    o.resize(n + 4);
    wr32(o.data() + n, v);
}
void put16(std::vector<uint8_t> &o, uint32_t v) {
    const size_t n = o.size();
    o.resize(n + 2);
    wr16(o.data() + n, v);
}
void puts_(std::vector<uint8_t> &o, const std::string &s) { o.insert(o.end(), s.begin(), s.end()); }

}  // namespace

extern "C" int dcr_bgzw_write(dcr_bgzw *w, const void *bytes, int64_t n);

extern "C" int dcr_synth_write(dcr_bgzw *w, const dcr_synth_in *in, int n_threads) {
    if (!w || !in || in->n_fam < 0) return DCR_IO_EARG;
    static const uint16_t kFlag[4] = {99, 163, 83, 147};
    static const char kStrand[4] = {'A', 'B', 'B', 'A'};
    Pool pool(pick_threads(n_threads));
    const int32_t F = in->n_fam;
    const int32_t chunk = 256;
    const int32_t nch = (F + chunk - 1) / chunk;
    const int32_t group = 4 * pool.size();
    std::vector<std::vector<uint8_t>> bufs((size_t)std::min(nch, group));
    for (int32_t g0 = 0; g0 < nch; g0 += group) {
        const int32_t g1 = std::min(nch, g0 + group);
        pool.run((size_t)(g1 - g0), [&](size_t gi) {
            std::vector<uint8_t> &o = bufs[gi];
            o.clear();
            const int32_t f0 = (g0 + (int32_t)gi) * chunk, f1 = std::min(F, f0 + chunk);
            for (int32_t f = f0; f < f1; ++f) {
                const int64_t fid = in->fam_id0 + f;
                const std::string sf = std::to_string(fid);
                const char *u = in->umis + (size_t)f * 16;
                const std::string u1(u, 8), u2(u + 8, 8);
                // mate positions: first read of the opposite strand's subfamilies
                int32_t fwd_pos = -1, rev_pos = -1;
                for (int k = 0; k < 4; ++k) {
                    const int32_t a = in->sub_off[4 * f + k];
                    if (in->sub_off[4 * f + k + 1] > a) {
                        if (k < 2 && fwd_pos < 0) fwd_pos = in->read_pos[a];
                        if (k >= 2 && rev_pos < 0) rev_pos = in->read_pos[a];
                    }
                }
                for (int k = 0; k < 4; ++k) {
                    const std::string mi = sf + "/" + kStrand[k];
                    const std::string rx = kStrand[k] == 'A' ? u1 + "-" + u2 : u2 + "-" + u1;
                    for (int32_t r = in->sub_off[4 * f + k], j = 0; r < in->sub_off[4 * f + k + 1]; ++r, ++j) {
                        const std::string name = "mol" + sf + "_" + std::to_string(k) + "_" + std::to_string(j);
                        const int32_t L = in->seq_len[r], nc = in->cig_n[r];
                        const uint32_t *cg = in->cigar + in->cig_off[r];
                        int64_t rl = 0;
                        for (int32_t i = 0; i < nc; ++i) {
                            const uint32_t op = cg[i] & 15;
                            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) rl += cg[i] >> 4;
                        }
                        const int32_t pos = in->read_pos[r];
                        const int32_t mpos = k < 2 ? (rev_pos >= 0 ? rev_pos : pos) : (fwd_pos >= 0 ? fwd_pos : pos);
                        const int32_t tlen = k < 2 ? (mpos + L - pos) : -(pos + L - mpos);
                        const size_t rec0 = o.size();
                        put32(o, 0);
                        put32(o, (uint32_t)in->tid);
                        put32(o, (uint32_t)pos);
                        o.push_back((uint8_t)(name.size() + 1));
                        o.push_back(in->read_mapq[r]);
                        put16(o, (uint32_t)reg2bin(pos, pos + (rl > 0 ? rl : 1)));
                        put16(o, (uint32_t)nc);
                        put16(o, kFlag[k]);
                        put32(o, (uint32_t)L);
                        put32(o, (uint32_t)in->tid);
                        put32(o, (uint32_t)mpos);
                        put32(o, (uint32_t)tlen);
                        puts_(o, name);
                        o.push_back(0);
                        for (int32_t i = 0; i < nc; ++i) put32(o, cg[i]);
                        const uint8_t *b = in->bases + in->seq_off[r];
                        for (int32_t i = 0; i + 1 < L; i += 2) o.push_back((uint8_t)((kCode.code[b[i]] << 4) | kCode.code[b[i + 1]]));
                        if (L & 1) o.push_back((uint8_t)(kCode.code[b[L - 1]] << 4));
                        const uint8_t *q = in->quals + in->seq_off[r];
                        o.insert(o.end(), q, q + L);
                        puts_(o, "MIZ");
                        puts_(o, mi);
                        o.push_back(0);
                        puts_(o, "RXZ");
                        puts_(o, rx);
                        o.push_back(0);
                        wr32(o.data() + rec0, (uint32_t)(o.size() - rec0 - 4));
                    }
                }
            }
            return true;
        });
        for (int32_t gi = 0; gi < g1 - g0; ++gi)
            if (dcr_bgzw_write(w, bufs[(size_t)gi].data(), (int64_t)bufs[(size_t)gi].size()) != 0) return DCR_IO_EFILE;
    }
    return DCR_IO_OK;
}
