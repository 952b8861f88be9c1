// batcher.cpp — publish micro-batcher (hard part H5).
//
// The reference matches one topic per call, synchronously, inside the
// publishing connection's process (emqx_broker:publish/1 ->
// emqx_router:match_routes/1, src/emqx_broker.erl:148-157).  A GPU batch
// takes longer than a BEAM scheduler slice, so the NIF must not block: it
// submits the topic here and returns; this batcher gathers the topics of
// thousands of publisher processes into one device batch (sealed at
// max_topics / max_bytes, or deadline_us after its first topic), runs it
// through tm_match_batch (or tm_match_routes_batch), and hands every caller
// its own ordered result through a completion callback (the NIF's callback
// builds the list and enif_send()s it to the waiting pid).
//
// One worker thread per batcher.  While it runs batch k on the GPU, new
// submissions fill batch k+1 (double buffering).  Written against the public
// C-ABI only (include/topicmatch.h).
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/topicmatch.h"

namespace {

struct Req {
    tm_batch_done_fn fn;
    void* ctx;
    uint64_t ticket;
};

struct Batch {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> off{0};
    std::vector<Req> reqs;
    std::chrono::steady_clock::time_point first;
    size_t n() const { return reqs.size(); }
    void clear() {
        bytes.clear();
        off.assign(1, 0);
        reqs.clear();
    }
};

}  // namespace

struct tm_batcher {
    tm_engine* eng = nullptr;
    tm_batcher_config cfg{};
    std::mutex mu;
    std::condition_variable cv_work, cv_idle;
    Batch open;                       // filling
    std::deque<Batch> sealed;         // waiting for the worker
    std::vector<Batch> spare;         // recycled buffers
    bool stop = false, busy = false;
    uint64_t next_ticket = 1;
    tm_batcher_stats st{};
    std::thread worker;

    // output buffers of the worker (grown on demand)
    std::vector<uint32_t> counts, src, dest;
    std::vector<uint64_t> outoff;

    void seal_locked() {
        if (open.n() == 0) return;
        sealed.push_back(std::move(open));
        if (!spare.empty()) {
            open = std::move(spare.back());
            spare.pop_back();
        } else {
            open = Batch{};
        }
        open.clear();
        cv_work.notify_one();
    }

    void run(Batch& b) {
        const uint32_t n = (uint32_t)b.n();
        counts.resize(n);
        outoff.resize(n + 1);
        const bool routes = (cfg.flags & TM_BATCHER_ROUTES) != 0;
        uint64_t need = src.size();
        int rc;
        for (;;) {
            if (routes)
                rc = tm_match_routes_batch(eng, b.bytes.data(), b.off.data(), n, counts.data(), outoff.data(),
                                           src.data(), dest.data(), src.size(), &need);
            else
                rc = tm_match_batch(eng, b.bytes.data(), b.off.data(), n, counts.data(), outoff.data(), src.data(),
                                    src.size(), &need);
            if (rc != TM_ENOSPC) break;
            src.resize(need + need / 4 + 64);
            if (routes) dest.resize(src.size());
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            st.batches++;
            st.topics += n;
            if (n > st.max_batch) st.max_batch = n;
            if (rc == TM_OK) st.results += outoff[n];
            else st.failed_batches++;
        }
        for (uint32_t i = 0; i < n; ++i) {
            const Req& r = b.reqs[i];
            if (rc == TM_OK)
                r.fn(r.ctx, r.ticket, TM_OK, src.data() + outoff[i], routes ? dest.data() + outoff[i] : nullptr,
                     counts[i]);
            else
                r.fn(r.ctx, r.ticket, rc, nullptr, nullptr, 0);
        }
    }

    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            if (sealed.empty()) {
                if (open.n()) {
                    const auto due = open.first + std::chrono::microseconds(cfg.deadline_us);
                    if (std::chrono::steady_clock::now() >= due) {
                        st.deadline_seals++;
                        seal_locked();
                        continue;
                    }
                    cv_work.wait_until(lk, due);
                } else if (stop) {
                    return;
                } else {
                    cv_idle.notify_all();
                    cv_work.wait(lk);
                }
                continue;
            }
            Batch b = std::move(sealed.front());
            sealed.pop_front();
            busy = true;
            lk.unlock();
            run(b);
            b.clear();
            lk.lock();
            spare.push_back(std::move(b));
            busy = false;
            if (sealed.empty() && open.n() == 0) cv_idle.notify_all();
        }
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
    b->src.resize((size_t)b->cfg.max_topics * 16 + 1024);
    if (b->cfg.flags & TM_BATCHER_ROUTES) b->dest.resize(b->src.size());
    try {
        b->worker = std::thread([b] { b->loop(); });
    } catch (...) {
        delete b;
        return TM_ENOMEM;
    }
    *out = b;
    return TM_OK;
}

int tm_batcher_submit(tm_batcher* b, const uint8_t* topic, uint32_t len, tm_batch_done_fn fn, void* ctx,
                      uint64_t* ticket_out) {
    if (!b || !fn || (!topic && len)) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(b->mu);
    if (b->stop) return TM_EINVAL;
    Batch& o = b->open;
    if (o.n() == 0) {
        o.first = std::chrono::steady_clock::now();
        b->cv_work.notify_one();   // arm the deadline
    }
    o.bytes.insert(o.bytes.end(), topic, topic + len);
    o.off.push_back(o.bytes.size());
    const uint64_t t = b->next_ticket++;
    o.reqs.push_back(Req{fn, ctx, t});
    if (ticket_out) *ticket_out = t;
    if (o.n() >= b->cfg.max_topics || o.bytes.size() >= b->cfg.max_bytes) {
        b->st.size_seals++;
        b->seal_locked();
    }
    return TM_OK;
}

int tm_batcher_flush(tm_batcher* b) {
    if (!b) return TM_EINVAL;
    std::unique_lock<std::mutex> lk(b->mu);
    b->seal_locked();
    b->cv_idle.wait(lk, [b] { return b->sealed.empty() && b->open.n() == 0 && !b->busy; });
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
    {
        std::unique_lock<std::mutex> lk(b->mu);
        b->seal_locked();
        b->stop = true;
        b->cv_work.notify_all();
    }
    if (b->worker.joinable()) b->worker.join();
    delete b;
}

}  // extern "C"
