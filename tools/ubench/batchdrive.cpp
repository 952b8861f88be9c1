// batchdrive.cpp — measurement helper (not product code): drives an
// engine's micro-batcher (tm_batcher_*) the way the NIF does — P producer
// threads, one tm_batcher_submit per publish, a completion callback per
// topic — over a packed topic batch, and reports end-to-end topics/s and
// submit->callback latency (every 16th topic).  bench.py loads it with ctypes to add the
// batcher leg (PCIe and host threads included) to its line.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/topicmatch.h"

namespace {
using clk = std::chrono::steady_clock;
// the latency sample: every LAT_EVERY-th topic reads the clock at submit and
// in its callback (a clock read costs about as much as a submit: reading it
// per topic would measure the driver, not the batcher)
constexpr uint64_t LAT_EVERY = 16;
struct Rec {
    clk::time_point t0;
    int64_t lat_ns = -1;
    uint32_t n = 0;
    bool timed = false;
};
void on_done(void* ctx, uint64_t, int status, const uint32_t*, const uint32_t*, uint32_t n) {
    Rec* r = (Rec*)ctx;
    r->n = status == TM_OK ? n : 0xFFFFFFFFu;
    if (r->timed) r->lat_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - r->t0).count();
}
}  // namespace

// out[14]: seconds, topics/s, batches, mean batch, p50 us, p99 us, failed,
// matches, then per batch (us): sealed -> lane, pack, device path (H2D,
// kernels, D2H), callbacks, and within the device path the host time
// enqueueing it and waiting on the stream
extern "C" int tm_bench_batcher(tm_engine* e, const uint8_t* tb, const uint64_t* to, uint64_t nt, int producers,
                                uint32_t deadline_us, uint32_t max_topics, uint32_t lanes, uint32_t flags,
                                uint32_t cb_threads, double* out) {
    tm_batcher_config bc{};
    bc.callback_threads = cb_threads;
    bc.max_topics = max_topics;
    bc.deadline_us = deadline_us;
    bc.lanes_per_replica = lanes;
    bc.flags = flags;
    tm_batcher* b;
    int rc = tm_batcher_open(e, &bc, &b);
    if (rc != TM_OK) return rc;
    {   // warm-up outside the timed run: one whole pass of the same submits,
        // so the lanes' pinned / device buffers, the stripes' chunks and the
        // heap pages behind them have reached the timed run's sizes
        std::vector<Rec> warm(nt);
        std::vector<std::thread> th;
        for (int k = 0; k < producers; ++k)
            th.emplace_back([&, k] {
                for (uint64_t i = nt * k / producers; i < nt * (k + 1) / producers; ++i)
                    tm_batcher_submit(b, tb + to[i], (uint32_t)(to[i + 1] - to[i]), on_done, &warm[i], nullptr);
            });
        for (auto& x : th) x.join();
        tm_batcher_flush(b);
    }
    tm_batcher_stats st0;
    tm_batcher_get_stats2(b, &st0, sizeof st0, TM_BATCHER_STATS_RESET_MAX);
    std::vector<Rec> recs(nt);
    const auto t0 = clk::now();
    std::vector<std::thread> th;
    for (int k = 0; k < producers; ++k)   // contiguous blocks: no false sharing between producers
        th.emplace_back([&, k] {
            for (uint64_t i = nt * k / producers; i < nt * (k + 1) / producers; ++i) {
                if (i % LAT_EVERY == 0) {
                    recs[i].timed = true;
                    recs[i].t0 = clk::now();
                }
                tm_batcher_submit(b, tb + to[i], (uint32_t)(to[i + 1] - to[i]), on_done, &recs[i], nullptr);
            }
        });
    for (auto& x : th) x.join();
    tm_batcher_flush(b);
    const double secs = std::chrono::duration<double>(clk::now() - t0).count();
    tm_batcher_stats st;
    tm_batcher_get_stats2(b, &st, sizeof st, TM_BATCHER_STATS_RESET_MAX);
    tm_batcher_close(b);
    st.batches -= st0.batches;
    st.topics -= st0.topics;
    const double nb = st.batches ? (double)st.batches : 1.0;
    out[8] = (st.wait_ns - st0.wait_ns) / nb / 1e3;
    out[9] = (st.pack_ns - st0.pack_ns) / nb / 1e3;
    out[10] = (st.device_ns - st0.device_ns) / nb / 1e3;
    out[11] = (st.callback_ns - st0.callback_ns) / nb / 1e3;
    out[12] = (st.launch_ns - st0.launch_ns) / nb / 1e3;
    out[13] = (st.sync_ns - st0.sync_ns) / nb / 1e3;
    std::vector<int64_t> lat;
    lat.reserve(nt / LAT_EVERY + 1);
    uint64_t fails = 0, ids = 0;
    for (uint64_t i = 0; i < nt; ++i) {
        if (recs[i].timed) lat.push_back(recs[i].lat_ns);
        if (recs[i].n == 0xFFFFFFFFu) ++fails;
        else ids += recs[i].n;
    }
    std::sort(lat.begin(), lat.end());
    const size_t nl = lat.size() ? lat.size() : 1;
    if (lat.empty()) lat.push_back(0);
    out[0] = secs;
    out[1] = nt / secs;
    out[2] = (double)st.batches;
    out[3] = (double)st.topics / (st.batches ? st.batches : 1);
    out[4] = lat[(size_t)(0.5 * (nl - 1))] / 1e3;
    out[5] = lat[(size_t)(0.99 * (nl - 1))] / 1e3;
    out[6] = (double)fails;
    out[7] = (double)ids;
    return TM_OK;
}

// ---- open loop: publishes arrive at a fixed rate ------------------------
// P producers submit topic i at its scheduled time t0 + i / rate (the topic
// batch is cycled); latency = callback time - scheduled time (not submit
// time: a producer that falls behind its schedule is counted, as a publisher
// kept waiting would be).  Every LAT_EVERY-th topic is timed.
namespace {
struct OLRec {
    clk::time_point due;
    int64_t lat_ns = -1;
};
std::atomic<uint64_t> g_ol_fail{0}, g_ol_done{0};
void on_done_ol(void* ctx, uint64_t, int status, const uint32_t*, const uint32_t*, uint32_t) {
    if (status != TM_OK) g_ol_fail.fetch_add(1, std::memory_order_relaxed);
    if (ctx) {
        OLRec* r = (OLRec*)ctx;
        r->lat_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - r->due).count();
    }
    g_ol_done.fetch_add(1, std::memory_order_relaxed);
}
}  // namespace

// out[16]: seconds, achieved topics/s, batches, mean batch, p50 us, p99 us,
//          p999 us, max us, failed, max producer lag us, and per batch (us):
//          sealed -> lane, pack, device path, callbacks, device enqueue, device wait
extern "C" int tm_bench_batcher_open_loop(tm_engine* e, const uint8_t* tb, const uint64_t* to, uint64_t nt,
                                          int producers, double rate, uint64_t total, uint32_t deadline_us,
                                          uint32_t max_topics, uint32_t lanes, uint32_t flags, uint32_t cb_threads,
                                          double* out) {
    tm_batcher_config bc{};
    bc.callback_threads = cb_threads;
    bc.max_topics = max_topics;
    bc.deadline_us = deadline_us;
    bc.lanes_per_replica = lanes;
    bc.flags = flags & 0xFFFFu;
    bc.eager_us = flags >> 16;   // (this driver's convention: eager_us in the flags' high half)
    tm_batcher* b;
    int rc = tm_batcher_open(e, &bc, &b);
    if (rc != TM_OK) return rc;
    {   // warm-up: the lanes' buffers at their sizes
        std::vector<std::thread> th;
        const uint64_t w = std::min<uint64_t>(nt, 1u << 20);
        for (int k = 0; k < producers; ++k)
            th.emplace_back([&, k] {
                for (uint64_t i = w * k / producers; i < w * (k + 1) / producers; ++i)
                    tm_batcher_submit(b, tb + to[i], (uint32_t)(to[i + 1] - to[i]), on_done_ol, nullptr, nullptr);
            });
        for (auto& x : th) x.join();
        tm_batcher_flush(b);
    }
    tm_batcher_stats st0;
    tm_batcher_get_stats2(b, &st0, sizeof st0, TM_BATCHER_STATS_RESET_MAX);
    g_ol_fail = 0;
    g_ol_done = 0;
    // a settling phase of 100 ms at the offered rate before the measured
    // publishes: the warm-up's flood leaves device and pinned allocations
    // (hipHostMalloc / hipHostFree of the lanes' grown buffers) whose
    // runtime locks held the first copies of the open loop for 9-11 ms
    // (profiles/r05_latency/hip_api_long_calls.txt); they are not the
    // steady state this driver measures
    const uint64_t settle = (uint64_t)(rate * 0.1);
    total += settle;
    std::vector<OLRec> recs(total / LAT_EVERY + 1);
    std::vector<int64_t> lag(producers, 0);
    const auto t0 = clk::now() + std::chrono::milliseconds(2);
    const double ns_per = 1e9 / rate;
    std::vector<std::thread> th;
    for (int k = 0; k < producers; ++k)   // producer k: topics i = k, k + P, ... (interleaved schedule)
        th.emplace_back([&, k] {
            // paced by sleeping, never spinning: a spinning producer burns the
            // process's CPU quota (cgroup cpu.max) and the throttling then
            // stalls every thread, the batcher's included, for the rest of the
            // period.  A producer wakes at most every PACE_US and submits every
            // publish that has come due; the wait counts in the latency (it
            // runs from the scheduled time).
            constexpr int64_t PACE_US = 20;
            int64_t mylag = 0;
            auto now = clk::now();
            for (uint64_t i = (uint64_t)k; i < total; i += (uint64_t)producers) {
                const auto due = t0 + std::chrono::nanoseconds((int64_t)(i * ns_per));
                if (now < due) {
                    now = clk::now();
                    while (now < due) {
                        const auto gap = std::chrono::duration_cast<std::chrono::microseconds>(due - now).count();
                        std::this_thread::sleep_for(std::chrono::microseconds(std::min<int64_t>(std::max<int64_t>(gap, 1),
                                                                                                PACE_US)));
                        now = clk::now();
                    }
                }
                mylag = std::max<int64_t>(mylag, std::chrono::duration_cast<std::chrono::nanoseconds>(now - due).count());
                const uint64_t j = i % nt;
                OLRec* r = nullptr;
                if (i % LAT_EVERY == 0 && i >= settle) {
                    r = &recs[i / LAT_EVERY];
                    r->due = due;
                }
                tm_batcher_submit(b, tb + to[j], (uint32_t)(to[j + 1] - to[j]), on_done_ol, r, nullptr);
            }
            lag[k] = mylag;
        });
    // the per-batch means and maxima from the end of the settling phase
    std::this_thread::sleep_until(t0 + std::chrono::nanoseconds((int64_t)(settle * ns_per)));
    tm_batcher_get_stats2(b, &st0, sizeof st0, TM_BATCHER_STATS_RESET_MAX);
    const auto t_meas = clk::now();
    for (auto& x : th) x.join();
    tm_batcher_flush(b);
    const double secs = std::chrono::duration<double>(clk::now() - t_meas).count();
    tm_batcher_stats st;
    tm_batcher_get_stats2(b, &st, sizeof st, TM_BATCHER_STATS_RESET_MAX);
    tm_batcher_close(b);
    std::vector<int64_t> lat;
    for (const OLRec& r : recs)
        if (r.lat_ns >= 0) lat.push_back(r.lat_ns);
    std::sort(lat.begin(), lat.end());
    if (lat.empty()) lat.push_back(0);
    const size_t nl = lat.size();
    out[0] = secs;
    out[1] = (total - settle) / secs;
    out[2] = (double)(st.batches - st0.batches);
    out[3] = (double)(st.topics - st0.topics) / std::max<double>(1, st.batches - st0.batches);
    out[4] = lat[(size_t)(0.5 * (nl - 1))] / 1e3;
    out[5] = lat[(size_t)(0.99 * (nl - 1))] / 1e3;
    out[6] = lat[(size_t)(0.999 * (nl - 1))] / 1e3;
    out[7] = lat[nl - 1] / 1e3;
    out[8] = (double)g_ol_fail.load();
    out[9] = *std::max_element(lag.begin(), lag.end()) / 1e3;
    const double nb = std::max<double>(1, st.batches - st0.batches);
    out[10] = (st.wait_ns - st0.wait_ns) / nb / 1e3;
    out[11] = (st.pack_ns - st0.pack_ns) / nb / 1e3;
    out[12] = (st.device_ns - st0.device_ns) / nb / 1e3;
    out[13] = (st.callback_ns - st0.callback_ns) / nb / 1e3;
    out[14] = (st.launch_ns - st0.launch_ns) / nb / 1e3;
    out[15] = (st.sync_ns - st0.sync_ns) / nb / 1e3;
    // the worst single batch of the run (us; since the stats read after the warm-up)
    out[16] = st.max_wait_ns / 1e3;
    out[17] = st.max_pack_ns / 1e3;
    out[18] = st.max_device_ns / 1e3;
    out[19] = st.max_callback_ns / 1e3;
    out[20] = st.max_sync_ns / 1e3;
    return TM_OK;
}
