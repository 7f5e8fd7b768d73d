// r3_stream_host.cpp — TEST INFRASTRUCTURE: the ROUND-3 span-stream protocol
// (git 205281c, duplexumiconsensusreads_amd/csrc/dcr_inflate.hip:797-1057,
// the version the round-3 bench ran when its 16/16-pool process vanished,
// profiles/r03o/pool_ab_16_16_2_failed.log) restated on the host so the CPU
// suite can drive round 3's own ingest (extracted from git by
// tests/native/Makefile, target r3) through it.  Two worker threads take the
// roles of the device's two HIP streams: `k` (staging upload, k_inflate, the
// status download, the span's done event) and `out` (the fetch's
// device-to-host copies).  Each queue runs in order, as a HIP stream does,
// and page-locked / device buffers are heap blocks that are freed and
// re-allocated when a larger span needs them (hipHostFree / hipFree + malloc).
// What this version deliberately keeps from round 3:
//   * `fetched` rises only when a whole fetch returns (the small-block
//     deadlock), and a slot is reused once fetched >= the out1 of the span
//     four back;
//   * a fetch that fails returns with its earlier device-to-host copies
//     still queued on `out`;
//   * the member list comes from the ingest's scanner thread, which reads the
//     start offset when it starts (the late start is injected in the
//     extracted ingest, dcr_test_r3_member_scan_start below).
// Knobs (environment): DCR_R3_LATE_MS=n  the member scanner sleeps n ms before
// it reads its start offset; DCR_R3_COPY_US=n  each queued device-to-host copy
// takes n µs more (a busy copy engine).
#include <zlib.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dcr_inflate.h"

namespace {

int env_int(const char *k) {
    const char *v = std::getenv(k);
    return v ? std::atoi(v) : 0;
}

// one in-order queue (a HIP stream)
struct Queue {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    bool quit = false;
    int64_t queued = 0, ran = 0;
    Queue() {
        th = std::thread([this] {
            for (;;) {
                std::function<void()> f;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return quit || !q.empty(); });
                    if (q.empty()) return;
                    f = std::move(q.front());
                    q.pop_front();
                }
                f();
                {
                    std::lock_guard<std::mutex> g(mu);
                    ++ran;
                }
                cv.notify_all();
            }
        });
    }
    void push(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu);
            q.push_back(std::move(f));
            ++queued;
        }
        cv.notify_all();
    }
    void sync() {   // hipStreamSynchronize
        std::unique_lock<std::mutex> lk(mu);
        const int64_t want = queued;
        cv.wait(lk, [&] { return ran >= want; });
    }
    ~Queue() {
        {
            std::lock_guard<std::mutex> g(mu);
            quit = true;
        }
        cv.notify_all();
        th.join();
    }
};

struct Event {   // hipEvent_t with blocking sync
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    void record() {
        {
            std::lock_guard<std::mutex> g(mu);
            done = true;
        }
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return done; });
    }
};

int inflate_member(const uint8_t *in, uint32_t in_len, uint8_t *out, uint32_t isize, uint32_t crc) {
    z_stream z{};
    if (inflateInit2(&z, -15) != Z_OK) return 1;
    z.next_in = const_cast<uint8_t *>(in);
    z.avail_in = in_len;
    uint8_t dummy;
    z.next_out = isize ? out : &dummy;
    z.avail_out = isize;
    const int r = inflate(&z, Z_FINISH);
    const uLong got = z.total_out;
    inflateEnd(&z);
    if (r != Z_STREAM_END || got != isize) return 1;
    return (uint32_t)crc32(0L, out, isize) == crc ? 0 : 2;
}

void drain_device();

// a buffer that moves when it grows (round 3's grow / pinned_grow: hipFree and
// hipHostFree wait for the device first)
void grow(uint8_t *&p, size_t &cap, size_t n) {
    if (n <= cap) return;
    drain_device();
    std::free(p);
    p = (uint8_t *)std::malloc(n);
    cap = n;
}

constexpr int kSlots = 4;

// the inflater's slots (round 3: InflSlots, kept across streams)
struct Slots {
    uint8_t *h_stage[kSlots] = {}, *h_st[kSlots] = {}, *d_in[kSlots] = {}, *d_out[kSlots] = {}, *d_st[kSlots] = {};
    size_t cap_stage[kSlots] = {}, cap_hst[kSlots] = {}, cap_in[kSlots] = {}, cap_out[kSlots] = {}, cap_dst[kSlots] = {};
    std::vector<dcr_bgzf_member> d_m[kSlots];
    Queue s_k, s_out;
    bool busy = false;
    ~Slots() {
        s_k.sync();
        s_out.sync();
        for (int i = 0; i < kSlots; ++i) {
            std::free(h_stage[i]);
            std::free(h_st[i]);
            std::free(d_in[i]);
            std::free(d_out[i]);
            std::free(d_st[i]);
        }
    }
};

struct Totals {
    std::mutex mu;
    int64_t streams = 0, spans = 0, members = 0, bytes = 0;
} g_tot;

std::mutex g_inf_mu;   // round 3: dcr_inflater::mu
Slots *g_slots = nullptr;
std::string g_err;

void drain_device() {
    if (g_slots) {
        g_slots->s_k.sync();
        g_slots->s_out.sync();
    }
}

struct R3Stream {
    Slots *sl = nullptr;
    const uint8_t *file = nullptr;
    std::vector<dcr_bgzf_member> m;
    bool m_done = false;
    struct Span {
        int32_t m0 = 0, m1 = 0;
        int64_t out0 = 0, out1 = 0, in0 = 0, in1 = 0;
        bool launched = false, checked = false;
        int rc = 0;
        std::shared_ptr<Event> done;
    };
    std::deque<Span> spans;
    std::vector<dcr_bgzf_member> mrel[kSlots];
    std::thread producer;
    std::mutex mu;
    std::condition_variable cv;
    int64_t fetched = 0;
    bool stop = false, produced = false;
    int err = 0;
    int copy_us = env_int("DCR_R3_COPY_US");
};

void produce(R3Stream *st) {
    Slots &S = *st->sl;
    int32_t mnext = 0;
    for (size_t k = 0;; ++k) {
        const int32_t want = k == 0 ? 128 : k == 1 ? 1024 : 4096;
        R3Stream::Span *spp;
        {
            std::unique_lock<std::mutex> lk(st->mu);
            st->cv.wait(lk, [&] { return st->stop || st->m_done || (int32_t)st->m.size() - mnext >= want; });
            if (st->stop || (st->m_done && mnext == (int32_t)st->m.size())) break;
            R3Stream::Span sp;
            sp.m0 = mnext;
            sp.m1 = std::min((int32_t)st->m.size(), mnext + want);
            sp.out0 = st->m[sp.m0].out_off;
            sp.out1 = st->m[sp.m1 - 1].out_off + st->m[sp.m1 - 1].isize;
            sp.in0 = st->m[sp.m0].in_off;
            sp.in1 = sp.in0;
            for (int32_t i = sp.m0; i < sp.m1; ++i)
                sp.in1 = std::max<int64_t>(sp.in1, st->m[i].in_off + st->m[i].in_len);
            sp.done = std::make_shared<Event>();
            st->spans.push_back(sp);
            spp = &st->spans.back();
            st->cv.wait(lk, [&] {
                return st->stop || k < (size_t)kSlots || st->fetched >= st->spans[k - kSlots].out1;
            });
            if (st->stop) break;
        }
        auto &sp = *spp;
        mnext = sp.m1;
        const int slot = (int)(k % kSlots);
        const int32_t n = sp.m1 - sp.m0;
        const size_t nin = (size_t)(sp.in1 - sp.in0), nout = (size_t)(sp.out1 - sp.out0);
        grow(S.h_stage[slot], S.cap_stage[slot], nin + 16);
        grow(S.h_st[slot], S.cap_hst[slot], (size_t)n);
        grow(S.d_in[slot], S.cap_in[slot], nin + 1024);
        grow(S.d_out[slot], S.cap_out[slot], nout + 16);
        grow(S.d_st[slot], S.cap_dst[slot], (size_t)n);
        std::memcpy(S.h_stage[slot], st->file + sp.in0, nin);
        auto &mr = st->mrel[slot];
        {
            std::lock_guard<std::mutex> g(st->mu);
            mr.assign(st->m.begin() + sp.m0, st->m.begin() + sp.m1);
        }
        for (auto &x : mr) {
            x.in_off -= sp.in0;
            x.out_off -= sp.out0;
        }
        // hipMemcpyAsync of pinned staging (read when the queue runs it); the
        // member table is pageable, so its copy is taken now, as HIP stages it
        uint8_t *hs = S.h_stage[slot], *din = S.d_in[slot], *dout = S.d_out[slot], *dst_ = S.d_st[slot],
                *hst = S.h_st[slot];
        S.s_k.push([hs, din, nin] { std::memcpy(din, hs, nin); });
        auto rel = std::make_shared<std::vector<dcr_bgzf_member>>(mr);
        S.s_k.push([rel, din, dout, dst_] {
            for (size_t i = 0; i < rel->size(); ++i) {
                const dcr_bgzf_member &x = (*rel)[i];
                dst_[i] = (uint8_t)inflate_member(din + x.in_off, x.in_len, dout + x.out_off, x.isize, x.crc);
            }
        });
        S.s_k.push([hst, dst_, n] { std::memcpy(hst, dst_, (size_t)n); });
        auto done = sp.done;
        S.s_k.push([done] { done->record(); });
        {
            std::lock_guard<std::mutex> g(st->mu);
            sp.launched = true;
        }
        {
            std::lock_guard<std::mutex> g(g_tot.mu);
            ++g_tot.spans;
            g_tot.members += n;
        }
        st->cv.notify_all();
    }
    std::lock_guard<std::mutex> g(st->mu);
    st->produced = true;
    st->cv.notify_all();
}

int fetch(R3Stream *st, int64_t out_off, int64_t n, uint8_t *dst) {
    if (n == 0) return 0;
    Slots &S = *st->sl;
    const int64_t end = out_off + n;
    for (size_t k = 0;; ++k) {
        R3Stream::Span *spp;
        {
            std::unique_lock<std::mutex> lk(st->mu);
            st->cv.wait(lk, [&] { return st->spans.size() > k || st->produced || st->err; });
            if (st->spans.size() <= k) {
                g_err = "dcr_inflate_stream_fetch: range past the stream's members";
                return -1;             // round 3: returns with copies still queued on out
            }
            spp = &st->spans[k];
            if (spp->out0 >= end) break;
            if (spp->out1 <= out_off) continue;
            st->cv.wait(lk, [&] { return spp->launched || st->err; });
            if (!spp->launched) return -1;
        }
        auto &sp = *spp;
        const int slot = (int)(k % kSlots);
        if (!sp.checked) {
            sp.done->wait();
            for (int32_t i = 0; i < sp.m1 - sp.m0; ++i)
                if (S.h_st[slot][i] != 0) {
                    sp.rc = sp.m0 + i + 1;
                    break;
                }
            sp.checked = true;
        }
        if (sp.rc) return sp.rc;     // round 3: same, copies still queued
        const int64_t a = std::max(out_off, sp.out0), b = std::min(end, sp.out1);
        uint8_t *to = dst + (a - out_off);
        const uint8_t *from = S.d_out[slot] + (a - sp.out0);
        const size_t len = (size_t)(b - a);
        const int us = st->copy_us;
        S.s_out.push([to, from, len, us] {
            if (us) std::this_thread::sleep_for(std::chrono::microseconds(us));
            std::memcpy(to, from, len);
        });
        if (sp.out1 >= end) break;
    }
    S.s_out.sync();
    {
        std::lock_guard<std::mutex> g(st->mu);
        st->fetched = std::max(st->fetched, end);
    }
    st->cv.notify_all();
    std::lock_guard<std::mutex> g(g_tot.mu);
    g_tot.bytes += n;
    return 0;
}

void *r3_open(void *, const uint8_t *file) {
    {
        std::lock_guard<std::mutex> g(g_inf_mu);
        if (!g_slots) g_slots = new Slots;
        if (g_slots->busy) return nullptr;
        g_slots->busy = true;
    }
    auto *st = new R3Stream;
    st->sl = g_slots;
    st->file = file;
    st->producer = std::thread(produce, st);
    std::lock_guard<std::mutex> g(g_tot.mu);
    ++g_tot.streams;
    return st;
}
int r3_add(void *s, const dcr_bgzf_member *m, int32_t n, int32_t last) {
    auto *st = (R3Stream *)s;
    {
        std::lock_guard<std::mutex> g(st->mu);
        st->m.insert(st->m.end(), m, m + n);
        if (last) st->m_done = true;
    }
    st->cv.notify_all();
    return 0;
}
int r3_fetch(void *s, int64_t off, int64_t n, uint8_t *dst) { return fetch((R3Stream *)s, off, n, dst); }
void r3_close(void *s) {
    auto *st = (R3Stream *)s;
    {
        std::lock_guard<std::mutex> g(st->mu);
        st->stop = true;
    }
    st->cv.notify_all();
    if (st->producer.joinable()) st->producer.join();
    st->sl->s_k.sync();
    st->sl->s_out.sync();
    {
        std::lock_guard<std::mutex> g(g_inf_mu);
        st->sl->busy = false;
    }
    delete st;
}
int r3_run(void *, const uint8_t *in, int64_t, const dcr_bgzf_member *m, int32_t n, uint8_t *out, int64_t) {
    for (int32_t i = 0; i < n; ++i)
        if (inflate_member(in + m[i].in_off, m[i].in_len, out + m[i].out_off, m[i].isize, m[i].crc)) return i + 1;
    return 0;
}
// page-locked chunk buffers: hipHostFree waits for the device, so the
// emulation drains both queues before it frees
void *r3_alloc(void *, size_t bytes) { return std::malloc(bytes); }
void r3_free(void *, void *p) {
    drain_device();
    std::free(p);
}

}  // namespace

extern "C" {
void dcr_test_stream_hook(dcr_inflate_hook *hook) {
    hook->user = nullptr;
    hook->run = r3_run;
    hook->host_alloc = r3_alloc;
    hook->host_free = r3_free;
    hook->stream_open = r3_open;
    hook->stream_add = r3_add;
    hook->stream_fetch = r3_fetch;
    hook->stream_close = r3_close;
}
void dcr_test_stream_stats(int64_t *out4) {
    std::lock_guard<std::mutex> g(g_tot.mu);
    out4[0] = g_tot.streams;
    out4[1] = g_tot.spans;
    out4[2] = g_tot.members;
    out4[3] = g_tot.bytes;
}
// called by the extracted round-3 ingest's member scanner thread right before
// it reads its start offset (Makefile target r3 inserts the call)
void dcr_test_r3_member_scan_start(void) {
    const int ms = env_int("DCR_R3_LATE_MS");
    if (ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(ms));
}
}
