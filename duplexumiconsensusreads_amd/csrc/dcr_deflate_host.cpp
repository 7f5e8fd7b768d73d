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
