// dcr_deflate_host.cpp — the GPU BGZF block compressor (dcr_deflate.h) run
// as a sequential lane-by-lane emulation on the host: the same phase code
// the gfx950 kernel runs, for CPU tests against zlib / libdeflate inflate.
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/dcr_io.h"
#include "dcr_deflate.h"

extern "C" int64_t dcr_deflate_emulate(const uint8_t *in, int64_t n, uint8_t *out) {
    if (!in || !out || n <= 0 || n > (int64_t)dfl::kMaxIn) return -1;
    std::unique_ptr<dfl::Shared> sp(new dfl::Shared());
    dfl::Shared &s = *sp;
    const uint32_t N = (uint32_t)n;
    std::memcpy(s.in, in, (size_t)n);
    std::memset(s.in + n, 0, sizeof s.in - (size_t)n);
    // the slot starts as garbage, as on the device
    std::vector<uint32_t> w(dfl::kSlot / 4, 0xa5a5a5a5u), tok(dfl::kTokWords, 0);
    for (int l = 0; l < dfl::kT; ++l) dfl::p0_clear(s, l);
    for (int l = 0; l < dfl::kT; ++l) dfl::p1_hash(s, N, l);
    for (int l = 0; l < dfl::kT; ++l) dfl::p2_count(s, N, l, tok.data());
    for (int l = 0; l < dfl::kT; ++l) dfl::p3a_keys(s, l);
    for (int l = 0; l < dfl::kT; ++l) dfl::p3b_rank(s, l);
    for (int l = 0; l < dfl::kT; ++l) dfl::p3c_trees(s, l);
    for (int l = 0; l < dfl::kT; ++l) dfl::p3c_assign(s, l);
    dfl::p3c_header(s);
    for (int l = 0; l < dfl::kT; ++l) dfl::p3d_codes(s, l);
    for (int l = 0; l < dfl::kT; ++l) dfl::p4_bits(s, N, l, tok.data());
    dfl::p4_scan(s, N, w.data());
    for (int l = 0; l < dfl::kT; ++l) dfl::p5_emit(s, N, l, tok.data(), w.data());
    for (int l = 0; l < dfl::kT; ++l) dfl::p6_copy(s, l, w.data());
    const uint32_t total = dfl::p6_frame(s, N, w.data());
    std::memcpy(out, w.data(), total);
    return total;
}

// (test) the device's batched Huffman code-length counts (mr_counts) against
// the plain in-place algorithm (mr_lengths) on one alphabet: freq[0..m)
// ascending, m in 2..288; num_a / num_b (33 each) get the codes per length
// (limited to 15 bits) of the two
extern "C" int dcr_deflate_lengths_ab(const uint32_t *freq, int m, uint32_t *num_a, uint32_t *num_b) {
    if (!freq || !num_a || !num_b || m < 2 || m > 288) return -1;
    for (int i = 1; i < m; ++i)
        if (freq[i] < freq[i - 1] || !freq[i - 1]) return -1;
    std::vector<uint32_t> a(freq, freq + m), b(freq, freq + m);
    dfl::mr_lengths(a.data(), m);
    for (int i = 0; i <= 32; ++i) num_a[i] = 0;
    for (int i = 0; i < m; ++i) num_a[a[i] > 32 ? 32 : a[i]]++;
    dfl::limit_num(15, num_a);
    dfl::mr_counts(b.data(), m, num_b);
    dfl::limit_num(15, num_b);
    return 0;
}
