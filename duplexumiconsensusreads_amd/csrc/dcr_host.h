// dcr_host.h — internal helpers of the native host side (libdcr_io.so):
// a persistent worker pool, little-endian byte access, and the libdeflate
// entry points (the image ships libdeflate.so.0 without its header; these
// are its stable public prototypes, libdeflate.h v1.x).
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <new>
#include <sched.h>
#include <sys/mman.h>
#include <thread>
#include <vector>

extern "C" {
struct libdeflate_compressor;
struct libdeflate_decompressor;
struct libdeflate_compressor *libdeflate_alloc_compressor(int compression_level);
size_t libdeflate_deflate_compress(struct libdeflate_compressor *c, const void *in, size_t in_nbytes, void *out,
                                   size_t out_nbytes_avail);
size_t libdeflate_deflate_compress_bound(struct libdeflate_compressor *c, size_t in_nbytes);
void libdeflate_free_compressor(struct libdeflate_compressor *c);
struct libdeflate_decompressor *libdeflate_alloc_decompressor(void);
int libdeflate_deflate_decompress(struct libdeflate_decompressor *d, const void *in, size_t in_nbytes, void *out,
                                  size_t out_nbytes_avail, size_t *actual_out_nbytes_ret);
void libdeflate_free_decompressor(struct libdeflate_decompressor *d);
uint32_t libdeflate_crc32(uint32_t crc, const void *buffer, size_t len);
}

namespace dcrh {

inline uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline int32_t rdi32(const uint8_t *p) { return (int32_t)rd32(p); }
inline void wr16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
inline void wr32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// Mappings of released HugeBufs kept for the next ones (up to 1 GiB per
// process): an ingest maps ~210 MB of chunk buffers, and a fresh mapping pays
// its page faults again on every open (the CLI run after run in one process).
// Never unmapped at exit (the process's end reclaims them).
struct HugeCache {
    std::mutex mu;
    std::vector<std::pair<uint8_t *, size_t>> regions;
    size_t bytes = 0;
    static constexpr size_t kMax = (size_t)1 << 30;
    static HugeCache &get() {
        static HugeCache *c = new HugeCache;
        return *c;
    }
    // the smallest kept mapping of at least `cap` bytes (and at most twice that)
    uint8_t *take(size_t cap, size_t &got) {
        std::lock_guard<std::mutex> g(mu);
        size_t best = regions.size();
        for (size_t i = 0; i < regions.size(); ++i)
            if (regions[i].second >= cap && regions[i].second <= 2 * cap &&
                (best == regions.size() || regions[i].second < regions[best].second))
                best = i;
        if (best == regions.size()) return nullptr;
        uint8_t *p = regions[best].first;
        got = regions[best].second;
        regions.erase(regions.begin() + (long)best);
        bytes -= got;
        return p;
    }
    bool give(uint8_t *p, size_t cap) {
        std::lock_guard<std::mutex> g(mu);
        if (bytes + cap > kMax) return false;
        regions.emplace_back(p, cap);
        bytes += cap;
        return true;
    }
};

// Large host buffer on transparent huge pages (2 MiB) where the kernel
// allows it: the record walk reads inflated data at irregular strides, and
// with 4 KiB pages every few records cost a TLB miss.  resize() keeps the
// contents only when the capacity suffices; a new buffer's bytes are
// unspecified (a recycled mapping, HugeCache).
class HugeBuf {
  public:
    HugeBuf() = default;
    HugeBuf(const HugeBuf &) = delete;
    HugeBuf &operator=(const HugeBuf &) = delete;
    ~HugeBuf() { release(); }
    void resize(size_t n) {
        if (n <= cap_) { n_ = n; return; }
        release();
        constexpr size_t kHP = (size_t)2 << 20;
        const size_t cap = (n + kHP - 1) & ~(kHP - 1);
        size_t got = 0;
        uint8_t *q = HugeCache::get().take(cap, got);
        if (q) {
            p_ = q;
            cap_ = got;
            n_ = n;
            return;
        }
        void *p = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(p, cap, MADV_HUGEPAGE);
        p_ = (uint8_t *)p;
        cap_ = cap;
        n_ = n;
    }
    uint8_t *data() { return p_; }
    const uint8_t *data() const { return p_; }
    size_t size() const { return n_; }

  private:
    void release() {
        if (p_ && !HugeCache::get().give(p_, cap_)) munmap(p_, cap_);
        p_ = nullptr;
        cap_ = n_ = 0;
    }
    uint8_t *p_ = nullptr;
    size_t cap_ = 0, n_ = 0;
};

// CPUs this process may use: the affinity mask, capped by the cgroup's CPU
// quota (cgroup v2 cpu.max, or v1 cfs_quota / cfs_period), shared among the
// processes of this node's local ranks (LOCAL_WORLD_SIZE, set by
// torch.distributed.run).  hardware_concurrency() counts every CPU of the
// machine, which on a GPU node is many times the share of one process.
inline int available_cpus() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) {
        const unsigned hc = std::thread::hardware_concurrency();
        n = hc ? (int)hc : 1;
    }
    long quota = -1, period = 0;
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        if (std::fscanf(f, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0) quota = std::atol(q);
        std::fclose(f);
    } else if (FILE *fq = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
        if (std::fscanf(fq, "%ld", &quota) != 1) quota = -1;
        std::fclose(fq);
        if (FILE *fp = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (std::fscanf(fp, "%ld", &period) != 1) period = 0;
            std::fclose(fp);
        }
    }
    if (quota > 0 && period > 0) n = std::min<long>(n, std::max<long>(1, (quota + period - 1) / period));
    int ranks = 1;
    if (const char *e = std::getenv("LOCAL_WORLD_SIZE")) ranks = std::max(1, std::atoi(e));
    return std::max(1, n / ranks);
}

// threads of a host pool: n when the caller asks (n > 0), else this
// process's CPU share (available_cpus), at most 16
inline int pick_threads(int n) {
    if (n > 0) return std::min(n, 64);
    static const int avail = available_cpus();
    return std::max(1, std::min(avail, 16));
}

// Persistent workers; run(n, fn) calls fn(i) for i in [0, n) on the workers
// and the calling thread, returns false if any call returned false (the
// remaining calls are then skipped).  run() returns once every call has
// finished; it does not wait for workers that have not woken up yet (with
// more threads than cores, e.g. the inflater's pool beside this one, a late
// worker would otherwise hold every run for a scheduler time slice): a late
// worker finds the job's indices used up and goes back to sleep.
class Pool {
  public:
    explicit Pool(int n_threads) : nt_(std::max(1, n_threads)) {
        for (int t = 1; t < nt_; ++t) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return nt_; }
    bool run(size_t n, const std::function<bool(size_t)> &fn) {
        if (n == 0) return true;
        if (nt_ == 1 || n == 1) {
            for (size_t i = 0; i < n; ++i)
                if (!fn(i)) return false;
            return true;
        }
        auto job = std::make_shared<Job>();
        job->fn = &fn;
        job->n = n;
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = job;
            ++gen_;
        }
        cv_.notify_all();
        work(*job);
        {
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [&] { return job->done.load() == n; });
            if (job_ == job) job_.reset();
        }
        return job->ok.load();
    }

  private:
    struct Job {
        const std::function<bool(size_t)> *fn = nullptr;
        size_t n = 0;
        std::atomic<size_t> next{0}, done{0};
        std::atomic<bool> ok{true};
    };
    void work(Job &j) {
        for (;;) {
            const size_t i = j.next.fetch_add(1);
            if (i >= j.n) return;
            if (j.ok.load(std::memory_order_relaxed) && !(*j.fn)(i)) j.ok = false;
            if (j.done.fetch_add(1) + 1 == j.n) {
                std::lock_guard<std::mutex> g(mu_);
                done_cv_.notify_all();
            }
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                j = job_;
            }
            if (j) work(*j);
        }
    }
    int nt_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::shared_ptr<Job> job_;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace dcrh
