// batcher_bench.cpp — the micro-batcher (tm_batcher_*) driven the way the
// NIF drives it: P producer threads submit single publish topics, one call
// per publish, and every completion callback records the submit->callback
// latency.  Reports topics/s end to end and latency percentiles, per
// deadline setting.  Filters / topics come from the same synthetic generator
// as bench.py (emqx_amd/libtmwork.so, config C3 unless overridden).
//
// build: make tools/ubench/batcher_bench ; run: tools/ubench/batcher_bench [filters topics producers]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/topicmatch.h"

extern "C" {
struct wk_params {
    uint32_t levels, share_groups;
    double p_plus, p_hash, sys_frac, share_frac;
    uint32_t vocab[64];
};
int wk_generate(const wk_params* p, int kind, uint64_t n, uint64_t seed, int distinct, uint8_t** bytes,
                uint64_t** offs, uint64_t* nbytes);
void wk_free(void* p);
}

using clk = std::chrono::steady_clock;

struct Slot {
    clk::time_point t0;
    std::atomic<int64_t> lat_ns{-1};
    uint32_t n = 0;
};

static void on_done(void* ctx, uint64_t, int status, const uint32_t*, const uint32_t*, uint32_t n) {
    Slot* s = (Slot*)ctx;
    s->n = status == TM_OK ? n : 0xFFFFFFFFu;
    s->lat_ns.store(std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - s->t0).count(),
                    std::memory_order_release);
}

int main(int argc, char** argv) {
    const uint64_t nf = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ull;
    const uint64_t nt = argc > 2 ? strtoull(argv[2], 0, 10) : 2000000ull;
    const int P = argc > 3 ? atoi(argv[3]) : 16;
    wk_params p{};
    p.levels = 8;
    p.share_groups = 8;
    p.p_plus = 0.20;
    p.p_hash = 0.05;
    const uint32_t voc[8] = {16, 64, 256, 1024, 4096, 4096, 4096, 4096};
    for (int i = 0; i < 8; ++i) p.vocab[i] = voc[i];
    uint8_t *fb, *tb;
    uint64_t *fo, *to, fbn, tbn;
    if (wk_generate(&p, 0, nf, 0xE3A10000ull + 3, 1, &fb, &fo, &fbn) || wk_generate(&p, 1, nt, 0xE3A11000ull + 3, 0, &tb, &to, &tbn)) {
        fprintf(stderr, "generator failed\n");
        return 1;
    }
    tm_config cfg{};
    cfg.device = 0;
    cfg.filters_hint = nf;
    tm_engine* e;
    if (tm_open(&cfg, &e) != TM_OK || tm_insert_batch(e, fb, fo, (uint32_t)nf) != TM_OK) {
        fprintf(stderr, "engine failed\n");
        return 1;
    }
    uint64_t ep;
    tm_commit(e, &ep);
    printf("{\"filters\": %llu, \"topics\": %llu, \"producers\": %d, \"runs\": [", (unsigned long long)nf,
           (unsigned long long)nt, P);
    const uint32_t deadlines[] = {50, 200, 1000};
    bool first = true;
    for (uint32_t dl : deadlines) {
        tm_batcher_config bc{};
        bc.max_topics = 65536;
        bc.deadline_us = dl;
        tm_batcher* b;
        if (tm_batcher_open(e, &bc, &b) != TM_OK) return 1;
        std::vector<Slot> slots(nt);
        const auto t0 = clk::now();
        std::vector<std::thread> th;
        for (int k = 0; k < P; ++k)
            th.emplace_back([&, k] {
                for (uint64_t i = k; i < nt; i += P) {
                    slots[i].t0 = clk::now();
                    tm_batcher_submit(b, tb + to[i], (uint32_t)(to[i + 1] - to[i]), on_done, &slots[i], nullptr);
                }
            });
        for (auto& x : th) x.join();
        tm_batcher_flush(b);
        const double secs = std::chrono::duration<double>(clk::now() - t0).count();
        tm_batcher_stats st;
        tm_batcher_get_stats2(b, &st, sizeof st, 0);
        tm_batcher_close(b);
        std::vector<int64_t> lat(nt);
        uint64_t fails = 0, ids = 0;
        for (uint64_t i = 0; i < nt; ++i) {
            lat[i] = slots[i].lat_ns.load(std::memory_order_acquire);
            if (slots[i].n == 0xFFFFFFFFu) ++fails;
            else ids += slots[i].n;
        }
        std::sort(lat.begin(), lat.end());
        auto pct = [&](double q) { return lat[(size_t)(q * (nt - 1))] / 1e3; };
        printf("%s{\"deadline_us\": %u, \"topics_per_s\": %.0f, \"secs\": %.3f, \"batches\": %llu, "
               "\"mean_batch\": %.0f, \"max_batch\": %llu, \"lat_us_p50\": %.0f, \"lat_us_p99\": %.0f, "
               "\"lat_us_max\": %.0f, \"failed\": %llu, \"matches\": %llu}",
               first ? "" : ", ", dl, nt / secs, secs, (unsigned long long)st.batches,
               (double)st.topics / (st.batches ? st.batches : 1), (unsigned long long)st.max_batch, pct(0.5),
               pct(0.99), lat[nt - 1] / 1e3, (unsigned long long)fails, (unsigned long long)ids);
        fflush(stdout);
        first = false;
    }
    printf("]}\n");
    tm_close(e);
    wk_free(fb);
    wk_free(fo);
    wk_free(tb);
    wk_free(to);
    return 0;
}
