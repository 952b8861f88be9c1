// batcher.cpp — publish micro-batcher (hard part H5).
//
// The reference matches one topic per call, synchronously, inside the
// publishing connection's process (emqx_broker:publish/1 ->
// emqx_router:match_routes/1, src/emqx_broker.erl:148-157).  A GPU batch
// takes longer than a BEAM scheduler slice, so the NIF must not block: it
// submits the topic here and returns; this batcher gathers the topics of
// thousands of publisher processes into one device batch (sealed at
// max_topics / max_bytes, or deadline_us after its first topic), runs it on
// the GPU and hands every caller its own ordered result through a completion
// callback (the NIF's callback builds the list and enif_send()s it).
//
// Submission is striped: a producer thread appends to one of NSTRIPE
// buffers (its own lock), so thousands of publishers do not serialise on one
// mutex; a seal takes every stripe.  One worker thread per batcher gathers
// the stripes into pinned host memory, copies the batch to HBM, runs the
// stream-ordered device path (tm_match_batch_device, or
// tm_match_routes_batch_device with TM_BATCHER_ROUTES) and reads the results
// back with one synchronisation, into pinned memory, sized from the previous
// batches (a rare overflow is re-read).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/topicmatch.h"

namespace {

using clk = std::chrono::steady_clock;
constexpr int NSTRIPE = 16;

struct Req {
    tm_batch_done_fn fn;
    void* ctx;
    uint64_t ticket;
};

struct alignas(64) Stripe {
    std::mutex mu;
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> lens;
    std::vector<Req> reqs;
};

// pinned host buffer / device buffer that only grow
struct Pinned {
    void* p = nullptr;
    size_t bytes = 0;
    bool ensure(size_t need) {
        if (need <= bytes) return true;
        if (p) (void)hipHostFree(p);
        size_t want = need + need / 2 + 4096;
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            bytes = 0;
            return false;
        }
        bytes = want;
        return true;
    }
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
};
struct Dev {
    void* p = nullptr;
    size_t bytes = 0;
    bool ensure(size_t need) {
        if (need <= bytes) return true;
        if (p) (void)hipFree(p);
        size_t want = need + need / 2 + 4096;
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            bytes = 0;
            return false;
        }
        bytes = want;
        return true;
    }
    ~Dev() {
        if (p) (void)hipFree(p);
    }
};

std::atomic<uint32_t> g_stripe_rr{0};
thread_local int t_stripe = -1;

}  // namespace

struct tm_batcher {
    tm_engine* eng = nullptr;
    tm_batcher_config cfg{};
    int device = -1;
    hipStream_t stream = nullptr;
    Stripe stripes[NSTRIPE];
    std::atomic<uint64_t> pending{0}, pending_bytes{0}, next_ticket{1};
    std::atomic<int64_t> first_ns{0};

    std::mutex mu;                    // worker state, stats, wake-ups
    std::condition_variable cv_work, cv_idle;
    bool stop = false, busy = false;
    tm_batcher_stats st{};
    std::thread worker;

    // the batch being run (worker only)
    std::vector<Req> reqs;
    struct Taken {
        std::vector<uint8_t> bytes;
        std::vector<uint32_t> lens;
    } taken[NSTRIPE];
    Pinned h_bytes, h_off, h_counts, h_outoff, h_src, h_dest, h_total;
    Dev d_bytes, d_off, d_counts, d_outoff, d_src, d_dest, d_total;
    double ids_per_topic = 64.0;      // sizing estimate of the result read-back
    uint64_t rotate = 0;              // first stripe of the next gather

    int64_t now_ns() const { return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now().time_since_epoch()).count(); }

    bool due() const {
        const uint64_t n = pending.load(std::memory_order_acquire);
        if (n == 0) return false;
        if (n >= cfg.max_topics || pending_bytes.load(std::memory_order_relaxed) >= cfg.max_bytes) return true;
        return now_ns() - first_ns.load(std::memory_order_acquire) >= (int64_t)cfg.deadline_us * 1000;
    }

    // move every stripe's topics into the pinned batch; returns the count
    uint32_t gather() {
        reqs.clear();
        uint64_t nb = 0, n = 0;
        // under each stripe's lock: move its topics out, oldest first, up to
        // max_topics (pending counts them under the same lock, so the
        // subtraction never underflows)
        const uint64_t cap = cfg.max_topics;
        const int start = (int)(rotate++ % NSTRIPE);   // no stripe starves under overload
        for (int i = 0; i < NSTRIPE && n < cap; ++i) {
            const int s = (start + i) % NSTRIPE;
            Stripe& x = stripes[s];
            std::lock_guard<std::mutex> lk(x.mu);
            const size_t have = x.lens.size();
            if (have == 0) continue;
            const size_t k = (size_t)std::min<uint64_t>(have, cap - n);
            Taken& t = taken[s];
            if (k == have) {   // the whole stripe
                t.bytes.swap(x.bytes);
                t.lens.swap(x.lens);
                reqs.insert(reqs.end(), x.reqs.begin(), x.reqs.end());
                x.reqs.clear();
                x.bytes.clear();
                x.lens.clear();
            } else {           // its oldest k topics (the batch stays within max_topics)
                size_t kb = 0;
                for (size_t i = 0; i < k; ++i) kb += x.lens[i];
                t.bytes.assign(x.bytes.begin(), x.bytes.begin() + kb);
                t.lens.assign(x.lens.begin(), x.lens.begin() + k);
                reqs.insert(reqs.end(), x.reqs.begin(), x.reqs.begin() + k);
                x.bytes.erase(x.bytes.begin(), x.bytes.begin() + kb);
                x.lens.erase(x.lens.begin(), x.lens.begin() + k);
                x.reqs.erase(x.reqs.begin(), x.reqs.begin() + k);
            }
            nb += t.bytes.size();
            n += t.lens.size();
            // pending is counted under this lock: subtract while holding it
            pending.fetch_sub(t.lens.size(), std::memory_order_acq_rel);
            pending_bytes.fetch_sub(t.bytes.size(), std::memory_order_relaxed);
        }
        // topics left behind keep their first_ns: they are due at once
        if (device < 0) {   // nothing to stage: the batch fails with TM_EDEVICE
            for (auto& t : taken) {
                t.bytes.clear();
                t.lens.clear();
            }
            return (uint32_t)n;
        }
        if (!h_bytes.ensure(nb + 16) || !h_off.ensure((n + 1) * 8)) return UINT32_MAX;
        uint8_t* hb = (uint8_t*)h_bytes.p;
        uint64_t* ho = (uint64_t*)h_off.p;
        uint64_t o = 0, k = 0;
        ho[0] = 0;
        for (int i = 0; i < NSTRIPE; ++i) {   // same stripe order as reqs
            Taken& t = taken[(start + i) % NSTRIPE];
            if (!t.bytes.empty()) std::memcpy(hb + o, t.bytes.data(), t.bytes.size());
            for (uint32_t len : t.lens) {
                o += len;
                ho[++k] = o;
            }
            t.bytes.clear();
            t.lens.clear();
        }
        return (uint32_t)n;
    }

    int run_device(uint32_t n, uint64_t nbytes, bool routes, bool deliv, uint64_t& total) {
        auto chk = [](hipError_t e) { return e == hipSuccess; };
        if (!d_bytes.ensure(nbytes + 16) || !d_off.ensure((n + 1) * 8) || !d_counts.ensure(n * 4 + 4) ||
            !d_outoff.ensure((n + 1) * 8) || !d_total.ensure(64) || !h_counts.ensure(n * 4 + 4) ||
            !h_outoff.ensure((n + 1) * 8) || !h_total.ensure(64))
            return TM_ENOMEM;
        uint64_t cap = (uint64_t)(ids_per_topic * n * 1.25) + 1024;
        for (int pass = 0; pass < 2; ++pass) {
            if (!d_src.ensure(cap * 4) || !h_src.ensure(cap * 4) ||
                (routes && (!d_dest.ensure(cap * 4) || !h_dest.ensure(cap * 4))))
                return TM_ENOMEM;
            if (!chk(hipMemcpyAsync(d_bytes.p, h_bytes.p, nbytes, hipMemcpyHostToDevice, stream)) ||
                !chk(hipMemcpyAsync(d_off.p, h_off.p, (n + 1) * 8, hipMemcpyHostToDevice, stream)))
                return TM_EDEVICE;
            int rc = deliv ? tm_match_deliveries_batch_device(eng, (const uint8_t*)d_bytes.p, (const uint64_t*)d_off.p,
                                                              n, nbytes, (uint32_t*)d_counts.p, (uint64_t*)d_outoff.p,
                                                              (uint32_t*)d_src.p, (uint32_t*)d_dest.p, cap,
                                                              (uint64_t*)d_total.p, stream)
                     : routes ? tm_match_routes_batch_device(eng, (const uint8_t*)d_bytes.p, (const uint64_t*)d_off.p, n,
                                                           nbytes, (uint32_t*)d_counts.p, (uint64_t*)d_outoff.p,
                                                           (uint32_t*)d_src.p, (uint32_t*)d_dest.p, cap,
                                                           (uint64_t*)d_total.p, stream)
                            : tm_match_batch_device(eng, (const uint8_t*)d_bytes.p, (const uint64_t*)d_off.p, n,
                                                    nbytes, (uint32_t*)d_counts.p, (uint64_t*)d_outoff.p,
                                                    (uint32_t*)d_src.p, cap, (uint64_t*)d_total.p, stream);
            if (rc != TM_OK) return rc;
            // results up to cap in the same synchronisation
            if (!chk(hipMemcpyAsync(h_total.p, d_total.p, 8, hipMemcpyDeviceToHost, stream)) ||
                !chk(hipMemcpyAsync(h_counts.p, d_counts.p, n * 4, hipMemcpyDeviceToHost, stream)) ||
                !chk(hipMemcpyAsync(h_outoff.p, d_outoff.p, (n + 1) * 8, hipMemcpyDeviceToHost, stream)) ||
                !chk(hipMemcpyAsync(h_src.p, d_src.p, cap * 4, hipMemcpyDeviceToHost, stream)) ||
                (routes && !chk(hipMemcpyAsync(h_dest.p, d_dest.p, cap * 4, hipMemcpyDeviceToHost, stream))) ||
                !chk(hipStreamSynchronize(stream)))
                return TM_EDEVICE;
            total = *(const uint64_t*)h_total.p;
            ids_per_topic = 0.9 * ids_per_topic + 0.1 * ((double)total / n);
            if (total <= cap) return TM_OK;
            cap = total + total / 4 + 1024;   // overflow: rerun with room (rare)
        }
        return TM_OK;
    }

    void run() {
        const uint32_t n = gather();
        const bool deliv = (cfg.flags & TM_BATCHER_DELIVERIES) != 0;
        const bool routes = deliv || (cfg.flags & TM_BATCHER_ROUTES) != 0;
        uint64_t total = 0;
        int rc = n == UINT32_MAX ? TM_ENOMEM : TM_OK;
        if (rc == TM_OK && n) {
            if (device < 0) {
                rc = TM_EDEVICE;   // host-only engine: the match path runs on the GPU only
            } else {
                (void)hipSetDevice(device);
                rc = run_device(n, ((uint64_t*)h_off.p)[n], routes, deliv, total);
                if (rc == TM_OK && deliv) {   // lists sit at route offsets: count the entries
                    total = 0;
                    for (uint32_t i = 0; i < n; ++i) total += ((const uint32_t*)h_counts.p)[i];
                }
            }
        }
        const uint32_t m = rc == TM_ENOMEM && n == UINT32_MAX ? (uint32_t)reqs.size() : n;
        {
            std::lock_guard<std::mutex> lk(mu);
            st.batches++;
            st.topics += m;
            if (m > st.max_batch) st.max_batch = m;
            if (rc == TM_OK) st.results += total;
            else st.failed_batches++;
        }
        const uint32_t* cnt = (const uint32_t*)h_counts.p;
        const uint64_t* off = (const uint64_t*)h_outoff.p;
        const uint32_t* src = (const uint32_t*)h_src.p;
        const uint32_t* dst = (const uint32_t*)h_dest.p;
        for (uint32_t i = 0; i < m; ++i) {
            const Req& r = reqs[i];
            if (rc == TM_OK)
                r.fn(r.ctx, r.ticket, TM_OK, src + off[i], routes ? dst + off[i] : nullptr, cnt[i]);
            else
                r.fn(r.ctx, r.ticket, rc, nullptr, nullptr, 0);
        }
        reqs.clear();
    }

    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            if (due()) {
                busy = true;
                if (pending.load() >= cfg.max_topics) st.size_seals++;
                else st.deadline_seals++;
                lk.unlock();
                run();
                lk.lock();
                busy = false;
                continue;
            }
            if (pending.load(std::memory_order_acquire) == 0) {
                cv_idle.notify_all();
                if (stop) return;
                sleep_for(lk, std::chrono::milliseconds(50));
            } else {
                const int64_t left = first_ns.load() + (int64_t)cfg.deadline_us * 1000 - now_ns();
                if (left > 0) sleep_for(lk, std::chrono::nanoseconds(left));
            }
        }
    }

    // timed wait on the system clock (pthread_cond_timedwait): libstdc++'s
    // steady-clock wait uses pthread_cond_clockwait, which GCC 11's TSan does
    // not intercept (bogus "double lock" reports); a woken-early wait just loops
    template <class D>
    void sleep_for(std::unique_lock<std::mutex>& lk, D d) {
        cv_work.wait_until(lk, std::chrono::system_clock::now() + d);
    }

    void kick() {
        std::lock_guard<std::mutex> lk(mu);
        cv_work.notify_one();
    }
};

extern "C" {

int tm_batcher_open(tm_engine* e, const tm_batcher_config* cfg, tm_batcher** out) {
    if (!e || !out) return TM_EINVAL;
    tm_batcher* b = new (std::nothrow) tm_batcher();
    if (!b) return TM_ENOMEM;
    b->eng = e;
    if (cfg) b->cfg = *cfg;
    if (b->cfg.max_topics == 0) b->cfg.max_topics = 65536;
    if (b->cfg.max_bytes == 0) b->cfg.max_bytes = 64ull << 20;
    if (b->cfg.deadline_us == 0) b->cfg.deadline_us = 200;
    b->device = tm_engine_device(e);
    if (b->device >= 0) {
        if (hipSetDevice(b->device) != hipSuccess ||
            hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
            delete b;
            return TM_EDEVICE;
        }
    }
    try {
        b->worker = std::thread([b] { b->loop(); });
    } catch (...) {
        if (b->stream) (void)hipStreamDestroy(b->stream);
        delete b;
        return TM_ENOMEM;
    }
    *out = b;
    return TM_OK;
}

int tm_batcher_submit(tm_batcher* b, const uint8_t* topic, uint32_t len, tm_batch_done_fn fn, void* ctx,
                      uint64_t* ticket_out) {
    if (!b || !fn || (!topic && len)) return TM_EINVAL;
    if (t_stripe < 0) t_stripe = (int)(g_stripe_rr.fetch_add(1, std::memory_order_relaxed) % NSTRIPE);
    const uint64_t t = b->next_ticket.fetch_add(1, std::memory_order_relaxed);
    Stripe& s = b->stripes[t_stripe];
    uint64_t was;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        s.bytes.insert(s.bytes.end(), topic, topic + len);
        s.lens.push_back(len);
        s.reqs.push_back(Req{fn, ctx, t});
        b->pending_bytes.fetch_add(len, std::memory_order_relaxed);
        was = b->pending.fetch_add(1, std::memory_order_acq_rel);
        if (was == 0) b->first_ns.store(b->now_ns(), std::memory_order_release);
    }
    if (was == 0) {
        b->kick();   // arm the deadline
    } else if (was + 1 == b->cfg.max_topics) {
        b->kick();   // full
    }
    if (ticket_out) *ticket_out = t;
    return TM_OK;
}

int tm_batcher_flush(tm_batcher* b) {
    if (!b) return TM_EINVAL;
    std::unique_lock<std::mutex> lk(b->mu);
    // everything submitted before this call completes: force the deadline now
    b->first_ns.store(0, std::memory_order_release);
    b->cv_work.notify_one();
    b->cv_idle.wait(lk, [b] { return b->pending.load() == 0 && !b->busy; });
    return TM_OK;
}

int tm_batcher_get_stats(tm_batcher* b, tm_batcher_stats* out) {
    if (!b || !out) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(b->mu);
    *out = b->st;
    return TM_OK;
}

void tm_batcher_close(tm_batcher* b) {
    if (!b) return;
    tm_batcher_flush(b);
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
        b->cv_work.notify_all();
    }
    if (b->worker.joinable()) b->worker.join();
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
}

}  // extern "C"
