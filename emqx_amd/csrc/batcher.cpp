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
// chunks (its stripe's lock), so thousands of publishers do not serialise on
// one mutex.  A seal is O(stripes): the sealing thread moves each stripe's
// whole chunk out (a vector swap; only a stripe holding more than the batch
// has room for copies its oldest topics out) and hands the chunks to a free
// LANE; the lane (a thread, a stream and its own pinned / HBM buffers, bound
// to one of the engine's replicas, lanes_per_replica per GPU) packs them into
// its pinned memory, copies the batch to HBM, runs the stream-ordered device
// path (tm_match_batch_device, tm_match_routes_batch_device,
// tm_match_deliveries_batch_device), reads back counts, offsets and the
// total, then exactly `total` ids (no capacity-sized read-back), runs the
// batch's callbacks and recycles the chunks.  So several batches are in
// flight at once (one per lane: packing, upload, walk, read-back and
// callbacks of neighbouring batches overlap, and every GPU of a multi-device
// engine works), and no per-topic work runs on the single sealing thread.
#include <cstdlib>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstddef>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/topicmatch.h"

namespace {

using clk = std::chrono::steady_clock;
constexpr int NSTRIPE = 16;
// engine workspaces reserved at open: batches up to this many topics (a
// 256K-topic flood batch) run without growing them; larger ones grow on demand
constexpr uint64_t TM_BATCHER_RESERVE_TOPICS = 262144;

struct Req {
    tm_batch_done_fn fn;
    void* ctx;
    uint64_t ticket;
};

// Topics of one stripe, oldest first, from `head` on (a partial take
// advances head instead of moving the rest to the front).
struct Chunk {
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> lens;
    std::vector<Req> reqs;
    size_t head = 0, bhead = 0;   // topics / bytes already taken
    size_t size() const { return lens.size() - head; }
    size_t nbytes() const { return bytes.size() - bhead; }
    void reset() {
        bytes.clear();
        lens.clear();
        reqs.clear();
        head = bhead = 0;
    }
    void compact() {   // drop the taken prefix once it is the larger part
        if (head == 0 || head < lens.size() / 2) return;
        bytes.erase(bytes.begin(), bytes.begin() + bhead);
        lens.erase(lens.begin(), lens.begin() + head);
        reqs.erase(reqs.begin(), reqs.begin() + head);
        head = bhead = 0;
    }
};

// A producer thread appends to its own stripe; everything a submit touches
// lives in the stripe's cache lines (no shared counter is written per
// publish): its lock, its chunk, its pending count / bytes, the arrival
// time of its oldest topic and its ticket sequence.
struct alignas(64) Stripe {
    std::mutex mu;
    Chunk cur;
    std::atomic<uint64_t> pending{0}, pending_bytes{0};
    std::atomic<int64_t> first_ns{INT64_MAX};   // INT64_MAX: empty
    uint64_t seq = 0;                           // under mu
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

// one batch in flight: its requests, pinned staging and device buffers
struct Lane {
    int device = -1;
    hipStream_t stream = nullptr;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool full = false, stop = false;   // a batch has been handed over / shut down
    uint32_t n = 0;
    std::vector<Chunk> chunks;        // the batch: stripe chunks in gather order
    std::condition_variable cb_cv;    // callback parts still running on the callback threads (under mu)
    uint32_t cb_left = 0;
    Pinned h_bytes, h_off, h_counts, h_outoff, h_src, h_dest, h_total;
    Dev d_bytes, d_off, d_counts, d_outoff, d_src, d_dest, d_total;
    // small match/1 batches (fused transfers): offsets + bytes up in one copy,
    // total + offsets + counts + ids down in one copy
    Pinned h_io, h_out;
    Dev d_io, d_out;
    // the batch's results as the callbacks read them (into h_out, or the separate buffers)
    const uint32_t* r_counts = nullptr;
    const uint64_t* r_off = nullptr;
    const uint32_t* r_src = nullptr;
    const uint32_t* r_dst = nullptr;
    double ids_per_topic = 64.0;      // sizing estimate of the device result buffers
    clk::time_point sealed;           // when the batch was handed over
    uint64_t launch_ns = 0, sync_ns = 0;   // this batch: host time enqueueing the device work, waiting on it
};
inline uint64_t ns_since(clk::time_point a) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - a).count();
}

std::atomic<uint32_t> g_stripe_rr{0};
thread_local int t_stripe = -1;

}  // namespace

struct tm_batcher {
    tm_engine* eng = nullptr;
    tm_batcher_config cfg{};
    bool host_only = false;
    Stripe stripes[NSTRIPE];
    std::atomic<bool> sealer_idle{false};   // the sealer sleeps with nothing pending: the next submit wakes it
    std::atomic<bool> force{false};         // flush: seal whatever is pending now

    std::mutex mu;                    // sealer state, stats, wake-ups, lane hand-over
    std::condition_variable cv_work, cv_idle, cv_lane;
    bool stop = false;
    int sealing = 0, in_flight = 0;   // batches being gathered / on lanes
    tm_batcher_stats st{};
    std::thread worker;
    std::vector<std::unique_ptr<Lane>> lanes;
    std::vector<int> free_lanes;      // guarded by mu
    uint64_t rotate = 0;              // first stripe of the next gather (sealer only)
    uint64_t next_lane = 0;

    struct CbJob {
        Lane* L;
        int rc;
        bool routes;
        uint32_t lo, hi;
    };
    std::mutex cb_mu;                 // callback threads: parts of lanes' batches
    std::condition_variable cb_cv;
    std::deque<CbJob> cb_q;
    bool cb_stop = false;
    std::vector<std::thread> cb_threads;

    std::mutex pool_mu;               // emptied chunks (capacity kept) for the stripes
    std::vector<Chunk> pool;

    // Chunks are never freed while the batcher runs: every chunk in flight
    // (a stripe's, the lanes' batches) fits in the pool, so the heap pages
    // behind them stay mapped (a freed multi-MB vector goes back to the OS
    // and its replacement page-faults all over again), and a new chunk starts
    // at twice a stripe's share of a batch instead of growing by doubling.
    size_t pool_cap() const { return (size_t)NSTRIPE * (lanes.size() + 2); }
    Chunk spare() {
        std::lock_guard<std::mutex> lk(pool_mu);
        if (pool.empty()) {
            Chunk c;
            const size_t k = 2 * (size_t)cfg.max_topics / NSTRIPE + 64;
            c.lens.reserve(k);
            c.reqs.reserve(k);
            c.bytes.reserve(k * 64);
            return c;
        }
        Chunk c = std::move(pool.back());
        pool.pop_back();
        return c;
    }
    void recycle(std::vector<Chunk>& cs) {
        for (Chunk& c : cs) c.reset();
        std::lock_guard<std::mutex> lk(pool_mu);
        for (Chunk& c : cs)
            if (pool.size() < pool_cap()) pool.push_back(std::move(c));
        cs.clear();
    }

    int64_t now_ns() const { return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now().time_since_epoch()).count(); }

    // pending topics / bytes over the stripes and the oldest arrival
    uint64_t pending(uint64_t* bytes = nullptr, int64_t* oldest = nullptr) const {
        uint64_t n = 0, b = 0;
        int64_t o = INT64_MAX;
        for (const Stripe& x : stripes) {
            n += x.pending.load(std::memory_order_seq_cst);
            b += x.pending_bytes.load(std::memory_order_relaxed);
            o = std::min<int64_t>(o, x.first_ns.load(std::memory_order_acquire));
        }
        if (bytes) *bytes = b;
        if (oldest) *oldest = o;
        return n;
    }
    bool due() const {
        uint64_t b;
        int64_t o;
        const uint64_t n = pending(&b, &o);
        if (n == 0) return false;
        if (n >= cfg.max_topics || b >= cfg.max_bytes || force.load(std::memory_order_acquire)) return true;
        const int64_t age = now_ns() - o;
        // TM_BATCHER_EAGER: a free lane takes what is pending once the oldest
        // topic has waited eager_us or a fair batch is there (under mu)
        if (eager_ready() && (age >= (int64_t)cfg.eager_us * 1000 || n >= TM_BATCHER_EAGER_TOPICS)) return true;
        return age >= (int64_t)cfg.deadline_us * 1000;
    }
    bool eager_ready() const { return (cfg.flags & TM_BATCHER_EAGER) && !free_lanes.empty(); }

    // move stripes' topics (oldest first, up to max_topics) into lane L's
    // chunk list: a stripe that fits whole is swapped out, one holding more
    // than the batch has room for gives its oldest topics; sets L.n
    void gather(Lane& L) {
        L.chunks.clear();
        uint64_t n = 0;
        const uint64_t cap = cfg.max_topics;
        const int start = (int)(rotate++ % NSTRIPE);   // no stripe starves under overload
        for (int i = 0; i < NSTRIPE && n < cap; ++i) {
            const int s = (start + i) % NSTRIPE;
            Stripe& x = stripes[s];
            if (x.pending.load(std::memory_order_acquire) == 0) continue;
            Chunk fresh = spare();   // outside the stripe lock
            std::lock_guard<std::mutex> lk(x.mu);
            const size_t have = x.cur.size();
            if (have == 0) {
                recycle_one(std::move(fresh));
                continue;
            }
            const size_t k = (size_t)std::min<uint64_t>(have, cap - n);
            size_t kb;
            if (k == have) {   // the whole stripe
                kb = x.cur.nbytes();
                L.chunks.push_back(std::move(x.cur));
                x.cur = std::move(fresh);
            } else {           // its oldest k topics (the batch stays within max_topics)
                Chunk& c = fresh;
                const size_t h = x.cur.head;
                kb = 0;
                for (size_t j = 0; j < k; ++j) kb += x.cur.lens[h + j];
                const uint8_t* b0 = x.cur.bytes.data() + x.cur.bhead;
                c.bytes.assign(b0, b0 + kb);
                c.lens.assign(x.cur.lens.begin() + h, x.cur.lens.begin() + h + k);
                c.reqs.assign(x.cur.reqs.begin() + h, x.cur.reqs.begin() + h + k);
                x.cur.head += k;
                x.cur.bhead += kb;
                x.cur.compact();
                L.chunks.push_back(std::move(c));
            }
            n += k;
            // pending is counted under this lock: subtract while holding it;
            // topics left behind keep their stripe's first_ns (due at once)
            x.pending.store(x.pending.load(std::memory_order_relaxed) - k, std::memory_order_release);
            x.pending_bytes.store(x.pending_bytes.load(std::memory_order_relaxed) - kb, std::memory_order_relaxed);
            if (x.cur.size() == 0) x.first_ns.store(INT64_MAX, std::memory_order_release);
        }
        L.n = (uint32_t)n;
    }
    void recycle_one(Chunk&& c) {
        std::lock_guard<std::mutex> lk(pool_mu);
        if (pool.size() < pool_cap()) pool.push_back(std::move(c));
    }

    // the lane packs its chunks into pinned memory (bytes, offsets); false:
    // staging memory ran out
    static bool fused(const Lane& L, bool routes) { return !routes && L.n <= EAGER_TOPICS; }
    bool pack(Lane& L, bool routes) {
        uint64_t nb = 0;
        for (const Chunk& c : L.chunks) nb += c.nbytes();
        uint8_t* hb;
        uint64_t* ho;
        if (fused(L, routes)) {   // [offsets (n+1) u64][bytes] in one pinned block
            const uint64_t offb = ((uint64_t)L.n + 1) * 8;
            if (!L.h_io.ensure(offb + nb + 16)) return false;
            ho = (uint64_t*)L.h_io.p;
            hb = (uint8_t*)L.h_io.p + offb;
        } else {
            if (!L.h_bytes.ensure(nb + 16) || !L.h_off.ensure(((uint64_t)L.n + 1) * 8)) return false;
            hb = (uint8_t*)L.h_bytes.p;
            ho = (uint64_t*)L.h_off.p;
        }
        uint64_t o = 0, k = 0;
        ho[0] = 0;
        for (const Chunk& c : L.chunks) {
            if (c.nbytes()) std::memcpy(hb + o, c.bytes.data() + c.bhead, c.nbytes());
            for (size_t j = c.head; j < c.lens.size(); ++j) {
                o += c.lens[j];
                ho[++k] = o;
            }
        }
        return true;
    }

    // the lane's batch on its GPU; results in the lane's pinned buffers
    static constexpr uint32_t EAGER_TOPICS = 32768;   // batches up to this size read their lists back with the counts
    // a small match/1 batch: one copy up, the walk, one copy down (a small
    // batch's device time is mostly per-operation latency, not bytes)
    int run_fused(Lane& L, uint64_t& total) {
        auto chk = [](hipError_t e) { return e == hipSuccess; };
        const uint32_t n = L.n;
        const uint64_t offb = ((uint64_t)n + 1) * 8;
        const uint64_t nbytes = ((const uint64_t*)L.h_io.p)[n];
        const uint64_t cntb = ((uint64_t)n * 4 + 7) & ~7ull;
        if (!L.d_io.ensure(offb + nbytes + 16)) return TM_ENOMEM;
        hipStream_t s = L.stream;
        clk::time_point t0 = clk::now();
        if (!chk(hipMemcpyAsync(L.d_io.p, L.h_io.p, offb + nbytes + 8, hipMemcpyHostToDevice, s))) return TM_EDEVICE;
        uint64_t cap = (uint64_t)(L.ids_per_topic * n * 1.25) + 1024;
        for (int pass = 0; pass < 2; ++pass) {
            if (pass) t0 = clk::now();
            const uint64_t outb = 8 + offb + cntb + cap * 4;
            if (!L.d_out.ensure(outb) || !L.h_out.ensure(outb)) return TM_ENOMEM;
            uint8_t* d = (uint8_t*)L.d_out.p;
            // one launch (tm_match_small_device: lists in completion order,
            // read by (offset, count) per topic), or the CSR path (A/B)
            auto* const match = (cfg.flags & TM_BATCHER_CSR) ? tm_match_batch_device : tm_match_small_device;
            int rc = match(eng, (const uint8_t*)L.d_io.p + offb, (const uint64_t*)L.d_io.p, n, nbytes,
                           (uint32_t*)(d + 8 + offb), (uint64_t*)(d + 8), (uint32_t*)(d + 8 + offb + cntb), cap,
                           (uint64_t*)d, s);
            if (rc != TM_OK) return rc;
            if (!chk(hipMemcpyAsync(L.h_out.p, L.d_out.p, outb, hipMemcpyDeviceToHost, s))) return TM_EDEVICE;
            L.launch_ns += ns_since(t0);
            t0 = clk::now();
            if (!chk(hipStreamSynchronize(s))) return TM_EDEVICE;
            L.sync_ns += ns_since(t0);
            const uint8_t* h = (const uint8_t*)L.h_out.p;
            total = *(const uint64_t*)h;
            L.ids_per_topic = 0.9 * L.ids_per_topic + 0.1 * ((double)total / n);
            L.r_off = (const uint64_t*)(h + 8);
            L.r_counts = (const uint32_t*)(h + 8 + offb);
            L.r_src = (const uint32_t*)(h + 8 + offb + cntb);
            L.r_dst = nullptr;
            if (total <= cap) return TM_OK;
            cap = total + total / 4 + 1024;   // overflow: rerun with room (rare)
        }
        return TM_EDEVICE;
    }
    int run_device(Lane& L, bool routes, bool deliv, uint64_t& total) {
        if (fused(L, routes)) return run_fused(L, total);
        L.r_counts = (const uint32_t*)L.h_counts.p;
        L.r_off = (const uint64_t*)L.h_outoff.p;
        L.r_src = (const uint32_t*)L.h_src.p;
        L.r_dst = (const uint32_t*)L.h_dest.p;
        auto chk = [](hipError_t e) { return e == hipSuccess; };
        const uint32_t n = L.n;
        const uint64_t nbytes = ((const uint64_t*)L.h_off.p)[n];
        if (!L.d_bytes.ensure(nbytes + 16) || !L.d_off.ensure((n + 1) * 8) || !L.d_counts.ensure(n * 4 + 4) ||
            !L.d_outoff.ensure((n + 1) * 8) || !L.d_total.ensure(64) || !L.h_counts.ensure(n * 4 + 4) ||
            !L.h_outoff.ensure((n + 1) * 8) || !L.h_total.ensure(64))
            return TM_ENOMEM;
        hipStream_t s = L.stream;
        clk::time_point t0 = clk::now();
        if (!chk(hipMemcpyAsync(L.d_bytes.p, L.h_bytes.p, nbytes, hipMemcpyHostToDevice, s)) ||
            !chk(hipMemcpyAsync(L.d_off.p, L.h_off.p, (n + 1) * 8, hipMemcpyHostToDevice, s)))
            return TM_EDEVICE;
        uint64_t cap = (uint64_t)(L.ids_per_topic * n * 1.25) + 1024;
        for (int pass = 0; pass < 2; ++pass) {
            if (pass) t0 = clk::now();
            if (!L.d_src.ensure(cap * 4) || (routes && !L.d_dest.ensure(cap * 4))) return TM_ENOMEM;
            int rc = deliv ? tm_match_deliveries_batch_device(eng, (const uint8_t*)L.d_bytes.p, (const uint64_t*)L.d_off.p,
                                                              n, nbytes, (uint32_t*)L.d_counts.p, (uint64_t*)L.d_outoff.p,
                                                              (uint32_t*)L.d_src.p, (uint32_t*)L.d_dest.p, cap,
                                                              (uint64_t*)L.d_total.p, s)
                     : routes ? tm_match_routes_batch_device(eng, (const uint8_t*)L.d_bytes.p, (const uint64_t*)L.d_off.p, n,
                                                           nbytes, (uint32_t*)L.d_counts.p, (uint64_t*)L.d_outoff.p,
                                                           (uint32_t*)L.d_src.p, (uint32_t*)L.d_dest.p, cap,
                                                           (uint64_t*)L.d_total.p, s)
                            : tm_match_batch_device(eng, (const uint8_t*)L.d_bytes.p, (const uint64_t*)L.d_off.p, n,
                                                    nbytes, (uint32_t*)L.d_counts.p, (uint64_t*)L.d_outoff.p,
                                                    (uint32_t*)L.d_src.p, cap, (uint64_t*)L.d_total.p, s);
            if (rc != TM_OK) return rc;
            // the total, counts and offsets first: the list read-back is sized
            // by them; a small batch also reads its lists back speculatively
            // (up to the capacity) in the same round trip
            const bool eager = n <= EAGER_TOPICS;
            if (eager && (!L.h_src.ensure(cap * 4 + 4) || (routes && !L.h_dest.ensure(cap * 4 + 4))))
                return TM_ENOMEM;
            if (!chk(hipMemcpyAsync(L.h_total.p, L.d_total.p, 8, hipMemcpyDeviceToHost, s)) ||
                !chk(hipMemcpyAsync(L.h_counts.p, L.d_counts.p, n * 4, hipMemcpyDeviceToHost, s)) ||
                !chk(hipMemcpyAsync(L.h_outoff.p, L.d_outoff.p, (n + 1) * 8, hipMemcpyDeviceToHost, s)) ||
                (eager && !chk(hipMemcpyAsync(L.h_src.p, L.d_src.p, cap * 4, hipMemcpyDeviceToHost, s))) ||
                (eager && routes && !chk(hipMemcpyAsync(L.h_dest.p, L.d_dest.p, cap * 4, hipMemcpyDeviceToHost, s))))
                return TM_EDEVICE;
            L.launch_ns += ns_since(t0);
            t0 = clk::now();
            if (!chk(hipStreamSynchronize(s))) return TM_EDEVICE;
            L.sync_ns += ns_since(t0);
            total = *(const uint64_t*)L.h_total.p;
            L.ids_per_topic = 0.9 * L.ids_per_topic + 0.1 * ((double)total / n);
            if (total <= cap) {
                if (eager) {   // the lists came with the counts
                    L.r_src = (const uint32_t*)L.h_src.p;
                    L.r_dst = (const uint32_t*)L.h_dest.p;
                    L.r_counts = (const uint32_t*)L.h_counts.p;
                    L.r_off = (const uint64_t*)L.h_outoff.p;
                    return TM_OK;
                }
                break;
            }
            cap = total + total / 4 + 1024;   // overflow: rerun with room (rare)
        }
        if (!L.h_src.ensure(total * 4 + 4) || (routes && !L.h_dest.ensure(total * 4 + 4))) return TM_ENOMEM;
        t0 = clk::now();
        if ((total && !chk(hipMemcpyAsync(L.h_src.p, L.d_src.p, total * 4, hipMemcpyDeviceToHost, s))) ||
            (total && routes && !chk(hipMemcpyAsync(L.h_dest.p, L.d_dest.p, total * 4, hipMemcpyDeviceToHost, s))) ||
            !chk(hipStreamSynchronize(s)))
            return TM_EDEVICE;
        L.sync_ns += ns_since(t0);
        L.r_counts = (const uint32_t*)L.h_counts.p;
        L.r_off = (const uint64_t*)L.h_outoff.p;
        L.r_src = (const uint32_t*)L.h_src.p;
        L.r_dst = (const uint32_t*)L.h_dest.p;
        return TM_OK;
    }

    // callbacks of topics [lo, hi) of lane L's batch (gather order)
    void callbacks(const Lane& L, int rc, bool routes, uint32_t lo, uint32_t hi) {
        const uint32_t* cnt = L.r_counts;
        const uint64_t* off = L.r_off;
        const uint32_t* src = L.r_src;
        const uint32_t* dst = L.r_dst;
        uint32_t i = 0;
        for (const Chunk& c : L.chunks) {
            const uint32_t cn = (uint32_t)c.size();
            if (i + cn <= lo) {
                i += cn;
                continue;
            }
            for (size_t j = c.head + (lo > i ? lo - i : 0u); j < c.reqs.size() && i + (j - c.head) < hi; ++j) {
                const uint32_t k = i + (uint32_t)(j - c.head);
                const Req& r = c.reqs[j];
                if (rc == TM_OK)
                    r.fn(r.ctx, r.ticket, TM_OK, src + off[k], routes ? dst + off[k] : nullptr, cnt[k]);
                else
                    r.fn(r.ctx, r.ticket, rc, nullptr, nullptr, 0);
            }
            i += cn;
            if (i >= hi) break;
        }
    }

    // a batch's callbacks: on the lane, or cut into parts of >= CB_MIN topics
    // shared with the callback threads (the lane takes part 0 and waits for
    // the rest: its buffers are reused by the next batch)
    static constexpr uint32_t CB_MIN = 8192;
    void run_callbacks(Lane& L, int rc, bool routes, uint32_t m) {
        const uint32_t parts = std::min<uint32_t>((uint32_t)cb_threads.size() + 1, std::max<uint32_t>(1, m / CB_MIN));
        if (parts <= 1) {
            callbacks(L, rc, routes, 0, m);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(L.mu);
            L.cb_left = parts - 1;
        }
        {
            std::lock_guard<std::mutex> lk(cb_mu);
            for (uint32_t p = 1; p < parts; ++p)
                cb_q.push_back(CbJob{&L, rc, routes, (uint32_t)((uint64_t)m * p / parts),
                                     (uint32_t)((uint64_t)m * (p + 1) / parts)});
        }
        cb_cv.notify_all();
        callbacks(L, rc, routes, 0, (uint32_t)((uint64_t)m / parts));
        std::unique_lock<std::mutex> lk(L.mu);
        L.cb_cv.wait(lk, [&] { return L.cb_left == 0; });
    }
    void cb_loop() {
        for (;;) {
            CbJob j;
            {
                std::unique_lock<std::mutex> lk(cb_mu);
                cb_cv.wait(lk, [&] { return cb_stop || !cb_q.empty(); });
                if (cb_q.empty()) return;
                j = cb_q.front();
                cb_q.pop_front();
            }
            callbacks(*j.L, j.rc, j.routes, j.lo, j.hi);
            std::lock_guard<std::mutex> lk(j.L->mu);
            if (--j.L->cb_left == 0) j.L->cb_cv.notify_all();
        }
    }

    // lane worker: run handed-over batches and their callbacks
    void lane_loop(Lane& L, int idx) {
        if (L.device >= 0) (void)hipSetDevice(L.device);
        const bool deliv = (cfg.flags & TM_BATCHER_DELIVERIES) != 0;
        const bool routes = deliv || (cfg.flags & TM_BATCHER_ROUTES) != 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(L.mu);
                L.cv.wait(lk, [&] { return L.full || L.stop; });
                if (!L.full) return;
            }
            const uint32_t n = L.n;
            uint64_t total = 0, results = 0;
            L.launch_ns = L.sync_ns = 0;
            const clk::time_point t_start = clk::now();
            clk::time_point t_packed = t_start, t_dev = t_start;
            int rc = host_only ? TM_EDEVICE : TM_OK;   // host-only: the GPU path only
            // the batch's filter ids stay bound to their bytes until its
            // callbacks have gathered them (tm_lease_begin)
            uint64_t lease = 0;
            const bool leased = rc == TM_OK && n && tm_lease_begin(eng, &lease) == TM_OK;
            if (rc == TM_OK && n) {
                const bool packed = pack(L, routes);
                t_packed = clk::now();
                rc = packed ? run_device(L, routes, deliv, total) : TM_ENOMEM;
                t_dev = clk::now();
                if (rc == TM_OK)   // deliveries sit at route offsets: count the entries
                    for (uint32_t i = 0; i < n; ++i) results += L.r_counts[i];
            }
            const uint32_t m = n;
            run_callbacks(L, rc, routes, m);
            const clk::time_point t_cb = clk::now();
            if (leased) tm_lease_end(eng, lease);
            recycle(L.chunks);
            {
                std::lock_guard<std::mutex> lk(L.mu);
                L.full = false;
            }
            std::lock_guard<std::mutex> lk(mu);
            auto ns = [](clk::duration d) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(); };
            const uint64_t w_ns = ns(t_start - L.sealed), p_ns = ns(t_packed - t_start), d_ns = ns(t_dev - t_packed),
                           c_ns = ns(t_cb - t_dev);
            st.wait_ns += w_ns;
            st.pack_ns += p_ns;
            st.device_ns += d_ns;
            st.callback_ns += c_ns;
            st.launch_ns += L.launch_ns;
            st.sync_ns += L.sync_ns;
            st.max_wait_ns = std::max(st.max_wait_ns, w_ns);
            st.max_pack_ns = std::max(st.max_pack_ns, p_ns);
            st.max_device_ns = std::max(st.max_device_ns, d_ns);
            st.max_callback_ns = std::max(st.max_callback_ns, c_ns);
            st.max_sync_ns = std::max(st.max_sync_ns, L.sync_ns);
            st.batches++;
            st.topics += m;
            if (m > st.max_batch) st.max_batch = m;
            if (rc == TM_OK) st.results += results;
            else st.failed_batches++;
            free_lanes.push_back(idx);
            --in_flight;
            cv_lane.notify_all();
            cv_idle.notify_all();
            if (cfg.flags & TM_BATCHER_EAGER) cv_work.notify_one();   // the sealer may seal at once now
        }
    }

    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            if (due()) {
                // a free lane (every lane busy: the sealed batch waits, and
                // keeps filling to max_topics meanwhile)
                cv_lane.wait(lk, [&] { return !free_lanes.empty(); });
                const int li = free_lanes.back();
                free_lanes.pop_back();
                if (pending() >= cfg.max_topics) st.size_seals++;
                else st.deadline_seals++;
                ++sealing;
                lk.unlock();
                Lane& L = *lanes[li];
                gather(L);
                {
                    std::lock_guard<std::mutex> l2(L.mu);
                    L.full = true;
                    L.sealed = clk::now();
                }
                L.cv.notify_one();
                lk.lock();
                --sealing;
                ++in_flight;
                continue;
            }
            int64_t oldest;
            if (pending(nullptr, &oldest) == 0) {
                force.store(false, std::memory_order_release);
                cv_idle.notify_all();
                if (stop) return;
                // seq_cst store then re-check: either the submitter's pending++
                // is seen here, or its exchange() sees idle and wakes us
                sealer_idle.store(true, std::memory_order_seq_cst);
                if (pending() == 0) sleep_for(lk, std::chrono::milliseconds(50));
                sealer_idle.store(false, std::memory_order_release);
            } else {
                // until the deadline, or the eager age when a lane is free
                // (a lane freed or a batch's worth arriving meanwhile wakes it)
                const uint32_t us = eager_ready() ? std::min(cfg.eager_us, cfg.deadline_us) : cfg.deadline_us;
                const int64_t left = oldest + (int64_t)us * 1000 - now_ns();
                if (left > 0) sleep_for(lk, std::chrono::nanoseconds(std::min<int64_t>(left, 1000000)));
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

    void shutdown_lanes() {   // lanes first: a lane mid-batch may wait on the callback threads
        for (auto& L : lanes) {
            {
                std::lock_guard<std::mutex> lk(L->mu);
                L->stop = true;
            }
            L->cv.notify_all();
            if (L->th.joinable()) L->th.join();
            if (L->stream) {
                (void)hipSetDevice(L->device);
                (void)hipStreamDestroy(L->stream);
            }
        }
        {
            std::lock_guard<std::mutex> lk(cb_mu);
            cb_stop = true;
        }
        cb_cv.notify_all();
        for (auto& t : cb_threads)
            if (t.joinable()) t.join();
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
    if (b->cfg.eager_us == 0) b->cfg.eager_us = 40;   // profiles/r05_f/latency.jsonl
    const uint32_t per = b->cfg.lanes_per_replica ? b->cfg.lanes_per_replica : 2u;
    const int R = tm_engine_replicas(e);
    b->host_only = R == 0;
    std::vector<int32_t> devs(R > 0 ? R : 1, -1);
    if (R > 0 && tm_engine_devices(e, devs.data(), (uint32_t)R) != R) {
        delete b;
        return TM_EDEVICE;
    }
    // lanes round-robin over the replicas: lane k on replica k % R
    for (uint32_t k = 0; k < per * (uint32_t)devs.size(); ++k) {
        std::unique_ptr<Lane> L(new (std::nothrow) Lane());
        if (!L) {
            b->shutdown_lanes();
            delete b;
            return TM_ENOMEM;
        }
        L->device = devs[k % devs.size()];
        // normal priority (A/B: TM_BATCHER_PRIO=1 makes the lanes
        // high-priority streams, as bench.py's, each on a hardware queue of
        // its own; profiles/r05_y)
        static const bool prio = [] {
            const char* v = std::getenv("TM_BATCHER_PRIO");
            return v && v[0] == '1';
        }();
        int least = 0, greatest = 0;
        if (L->device >= 0 &&
            (hipSetDevice(L->device) != hipSuccess ||
             (prio ? (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
                      hipStreamCreateWithPriority(&L->stream, hipStreamNonBlocking, greatest) != hipSuccess)
                   : hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess))) {
            b->shutdown_lanes();
            delete b;
            return TM_EDEVICE;
        }
        b->lanes.push_back(std::move(L));
    }
    // the workspaces sized up front (the engine's for batches of up to
    // TM_BATCHER_RESERVE_TOPICS, each lane's for batches of up to 32768
    // topics at 64 B and 64 ids per topic): a buffer grown later frees and
    // reallocates device or pinned memory, which waits for the whole device
    // -- stalls of up to ~16 ms in a new batcher's first second (the latency
    // tail of profiles/r05_z).  Best effort: a reservation that does not fit
    // leaves the buffers to grow on demand, as before, and the open succeeds.
    if (R > 0) {
        const uint64_t mt = b->cfg.max_topics;
        const uint64_t pre = std::min<uint64_t>(mt, 32768);
        const uint64_t offb = (pre + 1) * 8, nbytes = pre * 64, cntb = pre * 4 + 8, cap = pre * 64 + 1024;
        const uint64_t eng = std::min<uint64_t>(mt, TM_BATCHER_RESERVE_TOPICS);
        (void)tm_reserve(e, (uint32_t)eng, eng * 64);
        for (auto& L : b->lanes) {
            if (L->device < 0 || hipSetDevice(L->device) != hipSuccess) continue;
            (void)(L->h_io.ensure(offb + nbytes + 16) && L->d_io.ensure(offb + nbytes + 16) &&
                   L->h_out.ensure(8 + offb + cntb + cap * 4) && L->d_out.ensure(8 + offb + cntb + cap * 4) &&
                   L->h_bytes.ensure(nbytes + 16) && L->h_off.ensure(offb) && L->d_bytes.ensure(nbytes + 16) &&
                   L->d_off.ensure(offb) && L->d_counts.ensure(pre * 4 + 4) && L->d_outoff.ensure(offb) &&
                   L->d_total.ensure(64) && L->h_counts.ensure(pre * 4 + 4) && L->h_outoff.ensure(offb) &&
                   L->h_total.ensure(64) && L->d_src.ensure(cap * 4) && L->h_src.ensure(cap * 4 + 4));
        }
    }
    try {
        for (Stripe& x : b->stripes) x.cur = b->spare();
        for (size_t k = 0; k < b->lanes.size(); ++k) {
            b->free_lanes.push_back((int)(b->lanes.size() - 1 - k));   // lane 0 first
            b->lanes[k]->th = std::thread([b, k] { b->lane_loop(*b->lanes[k], (int)k); });
        }
        for (uint32_t k = 0; k < std::min<uint32_t>(b->cfg.callback_threads, 256u); ++k)
            b->cb_threads.emplace_back([b] { b->cb_loop(); });
        b->worker = std::thread([b] { b->loop(); });
    } catch (...) {
        b->shutdown_lanes();
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
    Stripe& s = b->stripes[t_stripe];
    uint64_t t, was;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        t = ++s.seq * NSTRIPE + (uint64_t)t_stripe;   // unique per batcher, no shared counter
        s.cur.bytes.insert(s.cur.bytes.end(), topic, topic + len);
        s.cur.lens.push_back(len);
        s.cur.reqs.push_back(Req{fn, ctx, t});
        // the counters change only under the stripe lock: plain load + store
        // (no read-modify-write per publish); the 0 -> 1 step is seq_cst for
        // the sealer's idle hand-shake below
        s.pending_bytes.store(s.pending_bytes.load(std::memory_order_relaxed) + len, std::memory_order_relaxed);
        was = s.pending.load(std::memory_order_relaxed);
        s.pending.store(was + 1, was == 0 ? std::memory_order_seq_cst : std::memory_order_release);
        if (was == 0) s.first_ns.store(b->now_ns(), std::memory_order_release);
    }
    // wake the sealer only when it sleeps with nothing pending (it times the
    // deadline itself), or when this stripe alone could fill a batch
    if ((was == 0 && b->sealer_idle.exchange(false, std::memory_order_seq_cst)) ||
        was + 1 == b->cfg.max_topics / NSTRIPE ||
        ((b->cfg.flags & TM_BATCHER_EAGER) && was + 1 == TM_BATCHER_EAGER_TOPICS / NSTRIPE))
        b->kick();
    if (ticket_out) *ticket_out = t;
    return TM_OK;
}

int tm_batcher_flush(tm_batcher* b) {
    if (!b) return TM_EINVAL;
    std::unique_lock<std::mutex> lk(b->mu);
    // everything submitted before this call completes: force the seal now
    b->force.store(true, std::memory_order_release);
    b->cv_work.notify_one();
    b->cv_idle.wait(lk, [b] { return b->pending() == 0 && b->sealing == 0 && b->in_flight == 0; });
    return TM_OK;
}

static_assert(offsetof(tm_batcher_stats, max_wait_ns) == TM_BATCHER_STATS_V1_BYTES, "round-4 stats prefix");

int tm_batcher_get_stats(tm_batcher* b, tm_batcher_stats* out) {
    return tm_batcher_get_stats2(b, out, TM_BATCHER_STATS_V1_BYTES, 0);
}

int tm_batcher_get_stats2(tm_batcher* b, tm_batcher_stats* out, uint32_t out_size, uint32_t flags) {
    if (!b || !out || out_size < TM_BATCHER_STATS_V1_BYTES) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(b->mu);
    std::memcpy(out, &b->st, std::min<size_t>(out_size, sizeof(tm_batcher_stats)));
    if (flags & TM_BATCHER_STATS_RESET_MAX)
        b->st.max_wait_ns = b->st.max_pack_ns = b->st.max_device_ns = b->st.max_callback_ns = b->st.max_sync_ns = 0;
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
    b->shutdown_lanes();
    delete b;
}

}  // extern "C"
