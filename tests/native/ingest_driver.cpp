// ingest_driver.cpp — TEST INFRASTRUCTURE: runs the native ingest
// (include/dcr_io.h) over a BAM to its end and prints its counters and a
// hash of every batch it packed, with the host pool (hook 0) or through the
// span-stream protocol of tests/native/stream_host.cpp (hook 1).  Built with
// the ingest's own sources under -fsanitize=thread or address
// (tests/native/Makefile) so races and lifetime errors of the stream path
// show up on the CPU; tests/test_stream_protocol.py compares the two hashes.
// DCR_TEST_PASSES=n runs n ingests one after another in the process (the
// bench's CLI passes share one inflater), printing a line per pass.
//   usage: ingest_driver BAM HOOK [READS_PER_BATCH]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/dcr_inflate.h"
#include "../../include/dcr_io.h"

extern "C" void dcr_test_stream_hook(dcr_inflate_hook *hook);
extern "C" void dcr_test_stream_stats(int64_t *out4);
extern "C" int64_t dcr_test_stream_late_allocs(void) __attribute__((weak));   // stream_host.cpp only

namespace {
uint64_t fnv(uint64_t h, const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}
template <class T>
std::vector<T> arr(size_t n) {
    return std::vector<T>(n > 0 ? n : 1);
}
}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s BAM HOOK [READS]\n", argv[0]);
        return 2;
    }
    const int use_hook = std::atoi(argv[2]);
    const int reads = argc > 3 ? std::atoi(argv[3]) : 1 << 18;
    dcr_inflate_hook hook{};
    if (use_hook) {
        dcr_test_stream_hook(&hook);
        if (dcr_io_set_inflate_hook(&hook) != 0) return 3;
    }
    const char *np = std::getenv("DCR_TEST_PASSES");
    const int passes = np && std::atoi(np) > 0 ? std::atoi(np) : 1;
    for (int pass = 0; pass < passes; ++pass) {
    dcr_ingest_cfg cfg{20, 1, 100, 20, 0, 0};
    dcr_ingest *ing = dcr_ingest_open(argv[1], &cfg);
    if (!ing) {
        std::fprintf(stderr, "open: %s\n", dcr_io_last_error());
        return 4;
    }
    const int f = reads / 4 + 16, t = 2 * f;
    const int64_t nb = 160LL * reads, nn = 96LL * t + (1 << 16), ns = 64LL << 20;
    auto sub_off = arr<int32_t>(4 * f + 1), read_pos = arr<int32_t>(reads), seq_len = arr<int32_t>(reads),
         cig_off = arr<int32_t>(reads), cig_n = arr<int32_t>(reads), fam_tid = arr<int32_t>(f),
         tab_kind = arr<int32_t>(t), tab_proc = arr<int32_t>(t), tab_sampled = arr<int32_t>(t);
    auto read_mapq = arr<uint8_t>(reads), bases = arr<uint8_t>(nb), quals = arr<uint8_t>(nb),
         side_exc = arr<uint8_t>(ns), side_filt = arr<uint8_t>(ns);
    auto seq_off = arr<int64_t>(reads), ss_col_off = arr<int64_t>(4 * f + 1), ds_col_off = arr<int64_t>(2 * f + 1),
         fam_code = arr<int64_t>(f), fam_rx = arr<int64_t>(2 * f), tab_code = arr<int64_t>(t),
         tab_exc_cut = arr<int64_t>(t), tab_filt_cut = arr<int64_t>(t);
    auto cigar = arr<uint32_t>(8 * reads);
    auto fam_eqx = arr<uint16_t>(4 * f);
    auto names = arr<char>(nn);
    dcr_host_batch hb{};
    hb.cap_fam = f;
    hb.cap_tab = t;
    hb.cap_reads = reads;
    hb.cap_cigar = 8LL * reads;
    hb.cap_bases = nb;
    hb.cap_names = nn;
    hb.cap_side = ns;
    hb.sub_off = sub_off.data();
    hb.read_pos = read_pos.data();
    hb.read_mapq = read_mapq.data();
    hb.seq_off = seq_off.data();
    hb.seq_len = seq_len.data();
    hb.cig_off = cig_off.data();
    hb.cig_n = cig_n.data();
    hb.cigar = cigar.data();
    hb.bases = bases.data();
    hb.quals = quals.data();
    hb.ss_col_off = ss_col_off.data();
    hb.ds_col_off = ds_col_off.data();
    hb.fam_tid = fam_tid.data();
    hb.fam_code = fam_code.data();
    hb.fam_rx = fam_rx.data();
    hb.fam_eqx = fam_eqx.data();
    hb.tab_kind = tab_kind.data();
    hb.tab_proc = tab_proc.data();
    hb.tab_sampled = tab_sampled.data();
    hb.tab_code = tab_code.data();
    hb.tab_exc_cut = tab_exc_cut.data();
    hb.tab_filt_cut = tab_filt_cut.data();
    hb.names = names.data();
    hb.side_exc = side_exc.data();
    hb.side_filt = side_filt.data();
    uint64_t h = 1469598103934665603ull;
    int batches = 0;
    for (;;) {
        if (dcr_ingest_next(ing, &hb) != 0) {
            std::printf("error %s\n", dcr_io_last_error());
            dcr_ingest_close(ing);
            return 5;
        }
        ++batches;
        const int F = hb.n_fam, n = hb.n_reads;
        h = fnv(h, sub_off.data(), 4 * (size_t)(4 * F + 1));
        h = fnv(h, read_pos.data(), 4 * (size_t)n);
        h = fnv(h, read_mapq.data(), (size_t)n);
        h = fnv(h, seq_len.data(), 4 * (size_t)n);
        h = fnv(h, cig_n.data(), 4 * (size_t)n);
        h = fnv(h, cigar.data(), 4 * (size_t)hb.n_cigar);
        h = fnv(h, bases.data(), (size_t)hb.n_bases);
        h = fnv(h, quals.data(), (size_t)hb.n_bases);
        h = fnv(h, tab_kind.data(), 4 * (size_t)hb.n_tab);
        h = fnv(h, side_exc.data(), (size_t)hb.n_side_exc);
        h = fnv(h, side_filt.data(), (size_t)hb.n_side_filt);
        h = fnv(h, &hb.end_kind, 4);
        if (hb.end_kind != DCR_END_FULL) break;
    }
    int64_t c[5] = {0, 0, 0, 0, 0};
    dcr_ingest_counters(ing, c);
    const int gpu = dcr_ingest_gpu_inflate(ing);
    dcr_ingest_close(ing);
    int64_t s[4] = {0, 0, 0, 0};
    dcr_test_stream_stats(s);
    std::printf("batches %d end %d records %lld passed %lld excluded %lld processed %lld filtered %lld hash %016llx "
                "hooked %d streams %lld spans %lld members %lld fetched %lld\n",
                batches, hb.end_kind, (long long)c[4], (long long)c[0], (long long)c[1], (long long)c[2],
                (long long)c[3], (unsigned long long)h, gpu, (long long)s[0], (long long)s[1], (long long)s[2],
                (long long)s[3]);
    if (dcr_test_stream_late_allocs) std::printf("late_allocs %lld\n", (long long)dcr_test_stream_late_allocs());
    std::fflush(stdout);
    }
    return 0;
}
