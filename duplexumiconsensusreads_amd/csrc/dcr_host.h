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
#include <functional>
#include <mutex>
#include <string>
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

inline int pick_threads(int n) {
    if (n > 0) return std::min(n, 64);
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc ? hc : 1u, 16u));
}

// Persistent workers; run(n, fn) calls fn(i) for i in [0, n) on the workers
// and the calling thread, returns false if any call returned false.
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
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            n_ = n;
            next_ = 0;
            ok_ = true;
            active_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return active_ == 0; });
        fn_ = nullptr;
        return ok_;
    }

  private:
    void work() {
        const std::function<bool(size_t)> *fn = fn_;
        for (size_t i; ok_.load(std::memory_order_relaxed) && (i = next_.fetch_add(1)) < n_;)
            if (!(*fn)(i)) ok_ = false;
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
            {
                std::lock_guard<std::mutex> g(mu_);
                if (--active_ == 0) done_cv_.notify_all();
            }
        }
    }
    int nt_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<bool(size_t)> *fn_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<bool> ok_{true};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace dcrh
