// dcr_span_stream.h — the scheduling protocol behind dcr_inflate_hook.stream_*
// (include/dcr_inflate.h), independent of where the members are inflated.
//
// The reader's helper thread appends the input's BGZF members as it walks the
// headers (add).  A producer thread forms spans of them and launches each span
// into one of kSlots output slots of the backend; fetch waits for the spans
// that cover an output range, checks their members' statuses and copies the
// range out.  The first spans are small (the reader starts early: on the GPU a
// member takes ~4 ms of serial decode whatever the launch size), the others
// hold 4,096 members.
//
// Slot reuse: span k goes into slot k % kSlots once span k - kSlots is done
// (its launch has completed) AND every byte of it has been copied out.
// `fetched` is advanced per span, as soon as a span's last byte is copied, not
// once per fetch: a fetch that covers more than kSlots spans (small BGZF
// blocks: a 64 MiB chunk of 4 KiB members is 16 k members) would otherwise
// wait for a span the producer can only launch after that same fetch returns.
//
// Backend B (csrc/dcr_inflate.hip: the device; tests/native/stream_host.cpp:
// a host emulation run under ThreadSanitizer) provides
//   using Event;                         a completion handle
//   bool new_events(Event &start, Event &done);  void free_events(Event&, Event&)
//   bool ensure(int slot, size_t nin, size_t nout, int32_t n)   slot buffers
//   uint8_t *stage(int slot)             host staging for the compressed bytes
//   bool launch(int slot, const dcr_bgzf_member *rel, int32_t n, size_t nin,
//               Event start, Event done)  inflate stage(slot) into the slot,
//                                        statuses into status(slot); async
//   bool wait(Event start, Event done, float *ms)   block until done
//   const uint8_t *status(int slot)      per-member status (0 = ok) after wait
//   bool copy_out(uint8_t *dst, int slot, int64_t off, int64_t n)  async copy
//   bool sync_out()                      every queued copy_out has landed
//   void drain()                         nothing of the backend is in flight
//   void account(float ms, int32_t members, int64_t fetched_bytes)
//   void error(const std::string &)      set the thread's error message
#ifndef DCR_SPAN_STREAM_H
#define DCR_SPAN_STREAM_H

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dcr_inflate.h"

namespace dcr_span {

constexpr int kSlots = 4;

inline int32_t span_members(size_t k) { return k == 0 ? 128 : k == 1 ? 1024 : 4096; }

// Every slot's buffers are sized once, for the largest span, by start() on
// the opening thread before the producer exists: a span holds at most
// kSpanMembers members, at most kSpanIn compressed bytes (a span ends early
// past it) and so at most kSpanMembers * 64 KiB of output (isize <= 65536).
// The producer's ensure() calls then never allocate or free (on the device:
// no hipFree / hipHostMalloc on the producer thread while kernels run,
// DESIGN.md §5, the round-3 exit suspect).
#ifndef DCR_SPAN_MEMBERS
#define DCR_SPAN_MEMBERS 4096   // A/B builds only
#endif
constexpr int32_t kSpanMembers = DCR_SPAN_MEMBERS;
constexpr size_t kSpanIn = (size_t)128 << 20;
constexpr size_t kSpanOut = (size_t)kSpanMembers * 65536;

template <class B>
struct Stream {
    using Event = typename B::Event;
    struct Span {
        int32_t m0 = 0, m1 = 0;
        int64_t out0 = 0, out1 = 0, in0 = 0, in1 = 0;
        bool launched = false;      // under mu
        bool checked = false;       // reader thread only
        int rc = 0;                 // reader thread only
        Event start{}, done{};
    };

    B &be;
    const uint8_t *file;
    std::vector<dcr_bgzf_member> m;     // appended by add (under mu)
    bool m_done = false;
    std::deque<Span> spans;             // formed by the producer; references stay valid
    std::vector<dcr_bgzf_member> rel[kSlots];   // producer thread only
    std::thread producer;
    std::mutex mu;
    std::condition_variable cv;
    int64_t fetched = 0;                // output bytes copied out, in order (monotonic)
    bool stop = false, produced = false;
    int err = 0;                        // producer-side runtime error

    Stream(B &b, const uint8_t *f) : be(b), file(f) {}
    ~Stream() { close(); }

    void start() {
        for (int slot = 0; slot < kSlots; ++slot)
            if (!be.ensure(slot, kSpanIn, kSpanOut, kSpanMembers)) {
                be.error("dcr_inflate_stream: slot buffers could not be allocated");
                err = -1;               // every fetch fails; no producer runs
                return;
            }
        producer = std::thread([this] { produce(); });
    }

    int add(const dcr_bgzf_member *mm, int32_t n, int32_t last) {
        {
            std::lock_guard<std::mutex> g(mu);
            m.insert(m.end(), mm, mm + n);
            if (last) m_done = true;
        }
        cv.notify_all();
        return 0;
    }

    void fail_producer() {
        std::lock_guard<std::mutex> g(mu);
        err = -1;
        cv.notify_all();
    }

    void produce() {
        int32_t mnext = 0;
        for (size_t k = 0;; ++k) {
            const int32_t want = span_members(k);
            Span *spp;
            Span *prev = nullptr;       // the slot's previous span
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || m_done || (int32_t)m.size() - mnext >= want; });
                if (stop || (m_done && mnext == (int32_t)m.size())) break;
                Span sp;
                sp.m0 = mnext;
                sp.m1 = std::min((int32_t)m.size(), mnext + want);
                // a span ends at a gap in the compressed input (members the
                // reader inflates on the host): its staging copy is
                // contiguous; and before kSpanIn compressed bytes (the slots'
                // sized capacity)
                for (int32_t i = sp.m0 + 1; i < sp.m1; ++i)
                    if (m[i].in_off > m[i - 1].in_off + (int64_t)m[i - 1].in_len + 64 ||
                        m[i].in_off + (int64_t)m[i].in_len - m[sp.m0].in_off > (int64_t)kSpanIn - 16) {
                        sp.m1 = i;
                        break;
                    }
                sp.out0 = m[sp.m0].out_off;
                sp.out1 = m[sp.m1 - 1].out_off + m[sp.m1 - 1].isize;
                sp.in0 = m[sp.m0].in_off;
                sp.in1 = sp.in0;
                for (int32_t i = sp.m0; i < sp.m1; ++i)
                    sp.in1 = std::max<int64_t>(sp.in1, m[i].in_off + m[i].in_len);
                if (!be.new_events(sp.start, sp.done)) {
                    err = -1;
                    cv.notify_all();
                    return;
                }
                spans.push_back(sp);
                spp = &spans.back();
                if (k >= (size_t)kSlots) {
                    prev = &spans[k - kSlots];
                    cv.wait(lk, [&] { return stop || fetched >= prev->out1; });
                    if (stop) break;
                }
            }
            // every byte of the previous span is copied out; its launch must
            // also be complete before its staging and output are touched (a
            // span with no output bytes is "fetched" before it even starts)
            if (prev && !be.wait(prev->start, prev->done, nullptr)) {
                fail_producer();
                return;
            }
            Span &sp = *spp;
            mnext = sp.m1;
            const int slot = (int)(k % kSlots);
            const int32_t n = sp.m1 - sp.m0;
            const size_t nin = (size_t)(sp.in1 - sp.in0), nout = (size_t)(sp.out1 - sp.out0);
            if (!be.ensure(slot, nin, nout, n)) {
                fail_producer();
                return;
            }
            std::memcpy(be.stage(slot), file + sp.in0, nin);
            auto &r = rel[slot];
            {
                std::lock_guard<std::mutex> g(mu);
                r.assign(m.begin() + sp.m0, m.begin() + sp.m1);
            }
            for (auto &x : r) {
                x.in_off -= sp.in0;
                x.out_off -= sp.out0;
            }
            if (!be.launch(slot, r.data(), n, nin, sp.start, sp.done)) {
                fail_producer();
                return;
            }
            {
                std::lock_guard<std::mutex> g(mu);
                sp.launched = true;
            }
            cv.notify_all();
        }
        std::lock_guard<std::mutex> g(mu);
        produced = true;
        cv.notify_all();
    }

    // output bytes [out_off, out_off + n) into dst; 0, the index + 1 of a
    // failed member, or -1.  Every return waits for the copies it queued
    // (dst is the caller's buffer, reused once this returns).
    int fetch(int64_t out_off, int64_t n, uint8_t *dst) {
        if (n == 0) return 0;
        const int64_t end = out_off + n;
        bool queued = false;
        auto leave = [&](int rc) {
            if (queued) be.sync_out();
            return rc;
        };
        for (size_t k = 0;; ++k) {
            Span *spp;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return spans.size() > k || produced || err; });
                if (spans.size() <= k) {
                    if (!err) be.error("dcr_inflate_stream_fetch: range past the stream's members");
                    else be.error("dcr_inflate_stream_fetch: the stream failed");
                    return leave(-1);
                }
                spp = &spans[k];
                if (spp->out0 >= end) break;
                if (spp->out1 <= out_off) continue;
                cv.wait(lk, [&] { return spp->launched || err; });
                if (!spp->launched) return leave(-1);
            }
            Span &sp = *spp;
            const int slot = (int)(k % kSlots);
            if (!sp.checked) {
                float ms = 0;
                if (!be.wait(sp.start, sp.done, &ms)) return leave(-1);
                const uint8_t *st = be.status(slot);
                for (int32_t i = 0; i < sp.m1 - sp.m0; ++i)
                    if (st[i] != 0) {
                        sp.rc = sp.m0 + i + 1;
                        break;
                    }
                sp.checked = true;
                be.account(ms, sp.m1 - sp.m0, 0);
            }
            if (sp.rc) {
                be.error("BGZF member " + std::to_string(sp.rc - 1) + " failed to inflate or CRC mismatch");
                return leave(sp.rc);
            }
            const int64_t a = std::max(out_off, sp.out0), b = std::min(end, sp.out1);
            if (!be.copy_out(dst + (a - out_off), slot, a - sp.out0, b - a)) return leave(-1);
            queued = true;
            if (b == sp.out1) {
                // the span is out: its slot may take span k + kSlots
                if (!be.sync_out()) return -1;
                queued = false;
                {
                    std::lock_guard<std::mutex> g(mu);
                    fetched = std::max(fetched, sp.out1);
                }
                cv.notify_all();
            }
            if (sp.out1 >= end) break;
        }
        if (queued && !be.sync_out()) return -1;
        {
            std::lock_guard<std::mutex> g(mu);
            fetched = std::max(fetched, end);
        }
        cv.notify_all();
        be.account(0, 0, n);
        return 0;
    }

    void close() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        if (producer.joinable()) producer.join();
        be.drain();
        for (auto &sp : spans) be.free_events(sp.start, sp.done);
        spans.clear();
    }
};

}  // namespace dcr_span

#endif  // DCR_SPAN_STREAM_H
