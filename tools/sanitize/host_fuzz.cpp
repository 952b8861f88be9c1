// host_fuzz.cpp — sanitizer driver for the host side of libtopicmatch (no GPU):
// randomized emqx_trie insert / delete / lookup, route add / del / get, the
// pure topic functions, the ACL rule builder, and the micro-batcher with
// producer threads on a host-only engine (every batch completes with
// TM_EDEVICE).  Built with ASan+UBSan (memory errors, UB) and TSan (races)
// by tools/sanitize/run.sh; exits non-zero on a bookkeeping inconsistency.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/topicmatch.h"

static std::string rand_filter(std::mt19937& g) {
    static const char* W[] = {"a", "b", "", "+", "#", "$SYS", "c", "dd", "%c"};
    std::string s;
    int n = 1 + (int)(g() % 6);
    for (int i = 0; i < n; ++i) {
        if (i) s += '/';
        const char* w = W[g() % 9];
        if (!std::strcmp(w, "#") && i + 1 < n) w = "x";
        s += w;
    }
    return s;
}

static void on_done(void* ctx, uint64_t, int status, const uint32_t* ids, const uint32_t*, uint32_t n) {
    auto* c = (std::atomic<uint64_t>*)ctx;
    if (status == TM_EDEVICE && ids == nullptr && n == 0) c->fetch_add(1);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937 g(12345);
    tm_config cfg{};
    cfg.device = -1;
    tm_engine* e = nullptr;
    if (tm_open(&cfg, &e) != TM_OK) return 1;
    std::set<std::string> live;                           // filters in the trie (expected)
    std::map<std::string, std::set<std::string>> routes;   // the route bag (expected)
    for (int i = 0; i < iters; ++i) {
        std::string f = rand_filter(g);
        const uint8_t* p = (const uint8_t*)f.data();
        switch (g() % 8) {
            case 0: case 1: case 2:
                if (tm_insert(e, p, (uint32_t)f.size()) != TM_OK) return 2;
                live.insert(f);
                break;
            case 3:
                if (tm_delete(e, p, (uint32_t)f.size()) != TM_OK) return 3;
                live.erase(f);
                break;
            case 4: {
                tm_node_info info;
                (void)tm_lookup(e, p, (uint32_t)f.size(), &info);
                break;
            }
            case 5: {   // emqx_router: the trie follows a wildcard topic's first / last route
                const std::string d = (g() & 1) ? "n1" : "n2";
                const bool add = g() & 1;
                const bool wild = tm_topic_wildcard(p, (uint32_t)f.size()) != 0;
                std::set<std::string>& bag = routes[f];
                if (add && !bag.count(d)) {
                    if (wild && bag.empty()) live.insert(f);
                    bag.insert(d);
                } else if (!add && bag.count(d)) {
                    if (wild && bag.size() == 1) live.erase(f);
                    bag.erase(d);
                }
                if ((add ? tm_route_add : tm_route_del)(e, p, (uint32_t)f.size(), (const uint8_t*)d.data(), 2) != TM_OK)
                    return 4;
                uint32_t out[8], k = 0;
                (void)tm_get_routes(e, p, (uint32_t)f.size(), out, 8, &k);
                break;
            }
            case 6: {
                std::string t = rand_filter(g);
                (void)tm_topic_match((const uint8_t*)t.data(), (uint32_t)t.size(), p, (uint32_t)f.size());
                (void)tm_topic_wildcard(p, (uint32_t)f.size());
                const uint8_t *in, *grp;
                uint32_t il, gl;
                std::string sh = "$share/g/" + f;
                (void)tm_topic_parse((const uint8_t*)sh.data(), (uint32_t)sh.size(), &in, &il, &grp, &gl);
                break;
            }
            default: {
                uint64_t ep;
                if (tm_commit(e, &ep) != TM_OK) return 5;
            }
        }
    }
    // ids of live filters gather back to their bytes
    std::vector<uint32_t> ids;
    for (const auto& f : live) {
        tm_node_info info;
        if (tm_lookup(e, (const uint8_t*)f.data(), (uint32_t)f.size(), &info) == TM_OK && info.filter_id != TM_NO_FILTER)
            ids.push_back(info.filter_id);
    }
    std::vector<uint64_t> off(ids.size() + 1);
    std::vector<uint8_t> buf(1 << 20);
    if (tm_filters_gather(e, ids.data(), (uint32_t)ids.size(), buf.data(), buf.size(), off.data()) != TM_OK) return 6;
    if (tm_filter_count(e) != ids.size()) {
        fprintf(stderr, "filter count %llu != live %zu\n", (unsigned long long)tm_filter_count(e), ids.size());
        return 7;
    }
    // ACL builder
    tm_acl* a;
    if (tm_acl_open(-1, &a) != TM_OK) return 8;
    for (int r = 0; r < 50; ++r) {
        tm_acl_rule_begin(a, r & 1, 1 + (r % 3));
        tm_acl_who(a, TM_ACL_WHO_AND, nullptr, 0, 0);
        tm_acl_who(a, TM_ACL_WHO_USER, (const uint8_t*)"u1", 2, 0);
        tm_acl_who(a, TM_ACL_WHO_IPADDR, (const uint8_t*)"10.0.0.0", 8, 8);
        tm_acl_who(a, TM_ACL_WHO_END, nullptr, 0, 0);
        std::string t = rand_filter(g);
        tm_acl_topic(a, r % 5 == 0, (const uint8_t*)t.data(), (uint32_t)t.size());
        if (tm_acl_rule_end(a) != TM_OK) return 9;
    }
    tm_acl_close(a);
    // micro-batcher: 8 producers on a host-only engine
    tm_batcher_config bc{};
    bc.max_topics = 256;
    bc.deadline_us = 100;
    tm_batcher* b;
    if (tm_batcher_open(e, &bc, &b) != TM_OK) return 10;
    std::atomic<uint64_t> done{0};
    std::vector<std::thread> th;
    for (int k = 0; k < 8; ++k)
        th.emplace_back([&, k] {
            std::mt19937 gg(k);
            for (int i = 0; i < 5000; ++i) {
                std::string t = rand_filter(gg);
                tm_batcher_submit(b, (const uint8_t*)t.data(), (uint32_t)t.size(), on_done, &done, nullptr);
            }
        });
    for (auto& t : th) t.join();
    tm_batcher_flush(b);
    tm_batcher_close(b);
    tm_close(e);
    if (done.load() != 40000) {
        fprintf(stderr, "batcher completions %llu != 40000\n", (unsigned long long)done.load());
        return 11;
    }
    printf("host_fuzz ok: %d ops, %zu live filters, 40000 batched submits\n", iters, ids.size());
    return 0;
}
