// walksim.cpp — cache and latency model of the walk kernel (diagnostic tool,
// not product code): replays tm_walk_queue's per-lane walk (kernels.hip
// walk_step / walk_pop, summaries on) over the host mirror of a committed
// image (tm_debug_image) and feeds its loads, in the order a GPU's lanes issue
// them, through a model of one XCD: per-CU L1 (32 KiB) and the XCD's L2
// (4 MiB, 16-way, LRU).  L2 misses model the fabric read requests
// (TCC_EA0_RDREQ: one 64 B request per missed 16 B gather, calibrated in
// profiles/r02_gather).
//
// Time: the lanes of a wave run in lockstep, so one walk step of a wave
// lasts, for each round of dependent loads in it, as long as the slowest
// lane's load of that round (the max over 64 random gathers); the model
// sums, per wave, the latency class (L1 hit / L2 hit / miss) of the slowest
// load of every round, and reports the mean over waves.
//
// Walk variants are evaluated as modes over the same logical walk, before
// any of them is built into the engine.
//
// Build: g++ -O2 -std=c++17 -shared -fPIC tools/sim/walksim.cpp -o tools/sim/libwalksim.so
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

// image.h names HIP vector types in its route views: host stand-ins
struct uint4 { unsigned x, y, z, w; };
struct uint2 { unsigned x, y; };
#include "../../emqx_amd/csrc/image.h"

using namespace tmx;

namespace {

struct View {
    const Node* nodes;
    uint64_t n_nodes;
    const EdgeSlot* cold;
    uint64_t cold_slots;
    const EdgeSlot* hot;
    uint64_t hot_slots;
    uint32_t hot_limit;
    uint32_t aux_stride;
    const uint8_t* aux;
};

enum Kind : uint8_t { K_INNER = 0, K_LEAF = 1, K_COLD = 2, K_HOT = 3, K_PAIR = 4, K_NKIND = 5 };
constexpr uint8_t K_FIXK = K_PAIR;   // M_FIX quads (the pair kind is unused with it): address space 4

// one load: its record, kind and dependent round within its step
struct Acc {
    uint32_t idx;   // node id / slot index (bit 31: second 16 B half of a 32 B slot)
    uint8_t kind;
    uint8_t round;
    uint8_t reach;  // node loads: how the walk got there (R_*)
};
enum Reach : uint8_t { R_ROOT = 0, R_PLUS_NOW = 1, R_PLUS_POP = 2, R_LIT_INLINE = 3, R_LIT_TABLE = 4, R_NREACH = 5 };

// set-associative LRU cache of 2^shift-byte lines
struct Cache {
    uint32_t ways = 16, sets = 1, shift = 6;
    std::vector<uint64_t> tag;   // sets * ways, MRU first; ~0 = empty
    void init(uint64_t bytes, uint32_t w, uint32_t sh) {
        ways = w;
        shift = sh;
        sets = (uint32_t)std::max<uint64_t>(1, (bytes >> sh) / w);
        tag.assign((size_t)sets * ways, ~0ull);
    }
    bool access(uint64_t addr) {   // true on hit; the line becomes MRU
        const uint64_t line = addr >> shift;
        const uint64_t set = (line * 0x9E3779B97F4A7C15ull >> 20) % sets;
        uint64_t* t = &tag[set * ways];
        for (uint32_t i = 0; i < ways; ++i) {
            if (t[i] == line) {
                std::memmove(t + 1, t, i * sizeof(uint64_t));
                t[0] = line;
                return true;
            }
        }
        std::memmove(t + 1, t, (ways - 1) * sizeof(uint64_t));
        t[0] = line;
        return false;
    }
};

// walk variants
enum Mode : int {
    M_SLOTREC = 1,   // TM_SLOT_RECORD: 32 B slots carry the child's record, the walk goes on in the same step
    M_PAIR = 2,      // a node's '+' child at id + 1, both halves loaded in one round; an immediate '+' step is free
    M_SPECPROBE = 4, // the parent's reference says "WIDE": the home slot is loaded with the node (no Bloom)
    M_BLOCKS = 8,    // per-node child blocks: a WIDE node's literal / '#' edges in a contiguous open-addressing
                     // block of its own (blocks in node order = heat order), not one shared table
    M_NOFP = 128,
    M_GFPTR = 512,   // with M_GF: the regions packed in node order (heat order) at 16 bits per child and found
                     // through a pointer in the node (its useless Bloom bits): the filter load is a round of
                     // its own after the node's half
    M_GF = 256,      // a per-node filter for nodes with >= GF_MIN literal children: a region of a global bit
                     // array at a hash of the node id, sized by a 2-bit class the reference to the node
                     // carries, so the filter word is loaded beside the node's half (same round); an
                     // absent word that passes the in-node Bloom but not the region costs no probe    // upper bound of a perfect per-node filter: a Bloom pass for an absent word costs no probe
    M_FIX = 64,      // a fixed 64 B block per node id (no pointer: address = v * 64): up to 8 literal children
                     // as 8 B {word, child} in 4 quads, home quad by word hash, quads probed in order (one
                     // round each); nodes with more children: the shared table (with M_BLOCKS: their own
                     // variable block, found through a header in the fixed block, one extra round)
};

// per-node child blocks (M_BLOCKS): 16 B slots {word, child, S(child), -}
struct Blocks {
    std::vector<uint64_t> base;    // per node: first slot (cells), ~0 = none
    std::vector<uint32_t> size;    // per node: slots (power of two)
    std::vector<uint32_t> word, child, sum;
    uint32_t div = 2;              // block size >= div * edges
    // M_FIX: per node, its literal children placed in the fixed block's quads (quad of child i), or
    // cnt > 8 (big: variable block / shared table)
    std::vector<uint32_t> cnt;
    std::vector<std::vector<std::pair<uint32_t, uint8_t>>> fixq;   // per node with <= 8 children: (word, quad)
    static uint32_t qhome(uint32_t w) { return (w * 0x9E3779B1u) >> 30; }
    static uint32_t home(uint32_t w, uint32_t mask) { return (w * 0x9E3779B1u >> 7) & mask; }
    void build(const View& v, uint32_t d) {
        div = d;
        const uint64_t n = v.n_nodes;
        cnt.assign(n, 0);
        auto each = [&](auto f) {
            for (const EdgeSlot* t : {v.cold, v.hot}) {
                const uint64_t ns = t == v.cold ? v.cold_slots : v.hot_slots;
                for (uint64_t s = 0; s < ns; ++s)
                    if (t[s].parent != EDGE_EMPTY) f(t[s]);
            }
        };
        each([&](const EdgeSlot& e) { ++cnt[e.parent]; });
        base.assign(n, ~0ull);
        size.assign(n, 0);
        uint64_t cur = 0;
        for (uint64_t x = 0; x < n; ++x) {
            if (!cnt[x]) continue;
            uint32_t sz = 1;
            while (sz < cnt[x] * div) sz <<= 1;
            if (sz < 4) sz = 4;
            // a block of <= 4 slots never crosses a 64 B line
            if (sz <= 4 && ((cur & 3) + sz > 4)) cur = (cur + 3) & ~3ull;
            base[x] = cur;
            size[x] = sz;
            cur += sz;
        }
        word.assign(cur, EDGE_EMPTY);
        child.assign(cur, NODE_NONE);
        sum.assign(cur, 0);
        fixq.assign(n, {});
        std::vector<uint8_t> fill(n * 4, 0);
        each([&](const EdgeSlot& e) {
            if (cnt[e.parent] > 8 || e.word == WORD_HASH) return;
            uint32_t q = qhome(e.word);
            while (fill[(uint64_t)e.parent * 4 + q] >= 2) q = (q + 1) & 3;
            ++fill[(uint64_t)e.parent * 4 + q];
            fixq[e.parent].push_back({e.word, (uint8_t)q});
        });
        each([&](const EdgeSlot& e) {
            const uint32_t m = size[e.parent] - 1;
            uint32_t p = home(e.word, m);
            while (word[base[e.parent] + p] != EDGE_EMPTY) p = (p + 1) & m;
            word[base[e.parent] + p] = e.word;
            child[base[e.parent] + p] = e.child;
            sum[base[e.parent] + p] = e.plus;
        });
    }
};

// M_GF: the global filter (built from the shared edge tables)
struct GFilt {
    uint32_t gbits = 0;                       // 2^gbits u32 words
    std::vector<uint32_t> words;
    std::vector<uint8_t> cls;                 // per node: 0 (none), 1..3
    uint32_t min_children = 16;
    static uint32_t region_words(uint32_t c) { return c == 1 ? 16u : c == 2 ? 128u : 1024u; }
    static uint32_t cls_of(uint32_t children, uint32_t mn) {
        return children < mn ? 0u : children <= 32 ? 1u : children <= 256 ? 2u : 3u;
    }
    bool packed = false;
    std::vector<uint64_t> pbase;   // packed: per node its region's first word
    std::vector<uint32_t> pwords;  // packed: per node its region's words (power of two)
    uint32_t rwords(uint32_t v) const { return packed ? pwords[v] : region_words(cls[v]); }
    uint64_t base(uint32_t v) const {
        if (packed) return pbase[v];
        const uint32_t R = region_words(cls[v]);
        return (uint64_t)(fmix32(v * 0x9E3779B1u + 0x7F4A7C15u) & ((1u << gbits) - 1u)) & ~(uint64_t)(R - 1);
    }
    static uint32_t wpos(uint32_t w, uint32_t R) { return (w * 0x85EBCA77u >> 8) & (R - 1); }
    static uint32_t wbits(uint32_t w) {
        const uint32_t h = w * 0xC2B2AE35u;
        return (1u << (h >> 27)) | (1u << ((h >> 22) & 31u));
    }
    void build(const View& v, uint32_t mn, uint32_t gb, bool pk) {
        min_children = mn;
        packed = pk;
        const uint64_t n = v.n_nodes;
        std::vector<uint32_t> cnt(n, 0);
        for (const EdgeSlot* t : {v.cold, v.hot}) {
            const uint64_t ns = t == v.cold ? v.cold_slots : v.hot_slots;
            for (uint64_t s = 0; s < ns; ++s)
                if (t[s].parent != EDGE_EMPTY && t[s].word != WORD_HASH) ++cnt[t[s].parent];
        }
        cls.assign(n, 0);
        uint64_t eb = 0;
        for (uint64_t x = 0; x < n; ++x) {
            cls[x] = (uint8_t)cls_of(cnt[x], mn);
            if (cls[x]) eb += cnt[x];
        }
        gbits = gb ? gb : 16;
        while (!gb && (1ull << gbits) * 32 < eb * 2 * 24) ++gbits;   // ~8 % of the bits set
        if (packed) {   // 16 bits per child, a power of two of u32 words, regions in node order
            pbase.assign(n, 0);
            pwords.assign(n, 0);
            uint64_t cur = 0;
            for (uint64_t x = 0; x < n; ++x) {
                if (!cls[x]) continue;
                uint32_t R = 1;
                while (R * 32 < cnt[x] * 16) R <<= 1;
                pwords[x] = R;
                pbase[x] = cur;
                cur += R;
            }
            gbits = 1;
            while ((1ull << gbits) < cur) ++gbits;
        }
        words.assign(1ull << gbits, 0);
        for (const EdgeSlot* t : {v.cold, v.hot}) {
            const uint64_t ns = t == v.cold ? v.cold_slots : v.hot_slots;
            for (uint64_t s = 0; s < ns; ++s) {
                const EdgeSlot& e = t[s];
                if (e.parent == EDGE_EMPTY || e.word == WORD_HASH || !cls[e.parent]) continue;
                words[base(e.parent) + wpos(e.word, rwords(e.parent))] |= wbits(e.word);
            }
        }
    }
};

struct Walker {
    const View& v;
    const GFilt* gf = nullptr;
    int mode = 0;
    const Blocks* blk = nullptr;
    mutable uint64_t probes_ok = 0, probes_fail = 0, table_visits = 0, plus_now = 0, plus_pop = 0, lit_inline = 0;
    mutable uint64_t wide_hist[48] = {0};   // WIDE lookups by log2(children): lookups, bloom passes, hits
    explicit Walker(const View& vw, int m) : v(vw), mode(m) {}

    const uint32_t* aux(uint32_t id) const {
        return reinterpret_cast<const uint32_t*>(v.aux + (uint64_t)id * v.aux_stride);
    }
    struct Hit {
        uint32_t child, plus;
        bool delivered;
    };
    // probe_edge<false> (kernels.hip): linear probing from the home slot,
    // one dependent round per slot (from round rd0 on)
    Hit probe(uint32_t node, uint32_t w, std::vector<Acc>& acc, uint32_t& rd) const {
        if ((mode & M_FIX) && w != WORD_HASH) {
            const uint32_t c = blk->cnt[node];
            if (c && c <= 8) {
                // quads from the home one on: a quad holding the word ends it; a
                // quad with a free entry (fewer than 2) ends it too
                std::vector<uint8_t> per(4, 0);
                uint8_t wq = 255;
                for (const auto& pr : blk->fixq[node]) {
                    ++per[pr.second];
                    if (pr.first == w) wq = pr.second;
                }
                uint32_t q = Blocks::qhome(w);
                for (int k = 0; k < 4; ++k, q = (q + 1) & 3) {
                    acc.push_back(Acc{(uint32_t)q, (uint8_t)(K_NKIND + 0), (uint8_t)std::min<uint32_t>(rd, 255)});
                    acc.back().idx = node * 4 + q;
                    acc.back().kind = K_FIXK;
                    ++rd;
                    if (q == wq) {
                        ++probes_ok;
                        // the child: from the shared table's record (same child, same summary)
                        uint32_t r0 = 0;
                        std::vector<Acc> dummy;
                        const int m0 = mode;
                        const_cast<Walker*>(this)->mode = 0;
                        const Hit h = probe(node, w, dummy, r0);
                        const_cast<Walker*>(this)->mode = m0;
                        --probes_ok;
                        return Hit{h.child, SUM_ALL, false};   // 8 B entries: no per-child summary
                    }
                    if (per[q] < 2) break;
                }
                ++probes_fail;
                return Hit{NODE_NONE, 0, false};
            }
            if (c > 8 && (mode & M_BLOCKS)) {   // header round in the fixed block
                acc.push_back(Acc{node * 4, K_FIXK, (uint8_t)std::min<uint32_t>(rd, 255)});
                ++rd;
            }
        }
        if ((mode & M_BLOCKS) && (!(mode & M_FIX) || blk->cnt[node] > 8)) {
            const uint64_t b = blk->base[node];
            if (b == ~0ull) {
                ++probes_fail;
                return Hit{NODE_NONE, 0, false};
            }
            const uint32_t m = blk->size[node] - 1;
            uint32_t p = Blocks::home(w, m);
            for (;;) {
                acc.push_back(Acc{(uint32_t)(b + p), K_COLD, (uint8_t)std::min<uint32_t>(rd, 255)});
                ++rd;
                const uint32_t ww = blk->word[b + p];
                if (ww == w) {
                    ++probes_ok;
                    return Hit{blk->child[b + p], blk->sum[b + p], false};
                }
                if (ww == EDGE_EMPTY) {
                    ++probes_fail;
                    return Hit{NODE_NONE, 0, false};
                }
                p = (p + 1) & m;
            }
        }
        const bool hot = node < v.hot_limit;
        const EdgeSlot* tab = hot ? v.hot : v.cold;
        const uint64_t mask = (hot ? v.hot_slots : v.cold_slots) - 1;
        uint64_t s = edge_home(node, w, mask);
        for (;;) {
            const EdgeSlot& e = tab[s];
            acc.push_back(Acc{(uint32_t)s, hot ? K_HOT : K_COLD, (uint8_t)std::min<uint32_t>(rd, 255)});
            if (mode & M_SLOTREC)
                acc.push_back(Acc{(uint32_t)s | 0x80000000u, hot ? K_HOT : K_COLD, (uint8_t)std::min<uint32_t>(rd, 255)});
            ++rd;
            if (e.parent == node && e.word == w) {
                ++probes_ok;
                return Hit{e.child, e.plus, (mode & M_SLOTREC) != 0};
            }
            if (e.parent == EDGE_EMPTY) {
                ++probes_fail;
                return Hit{NODE_NONE, 0, false};
            }
            s = (s + 1) & mask;
        }
    }
    // lit_child<false>; spec: the home slot was loaded in round 0 with the node
    Hit lit(uint32_t node, uint32_t plus, uint32_t lw, uint32_t lc, uint32_t w, std::vector<Acc>& acc,
            uint32_t& rd) const {
        if (w < WORD_MAX) {
            if (!(plus & WIDE)) {
                if (lw == w) ++lit_inline;
                return Hit{lw == w ? lc : NODE_NONE, SUM_ALL, false};
            }
            const uint32_t c = aux(node)[3];
            const uint32_t bk = c ? std::min(15, 31 - __builtin_clz(c)) : 0;
            ++wide_hist[bk];
            if (mode & M_SPECPROBE) {   // no Bloom: the home slot is in flight beside the node's half
                uint32_t r0 = 0;
                const Hit h = probe(node, w, acc, r0);
                rd = std::max(rd, r0);
                if (h.child != NODE_NONE) ++wide_hist[32 + bk];
                return h;
            }
            const uint64_t b = word_bloom(w);
            const uint64_t mask = ((uint64_t)lc << 32) | lw;
            if ((mask & b) != b) return Hit{NODE_NONE, 0, false};
            if (gf && gf->cls[node] && w < WORD_MAX) {   // the filter word came with the node's half (round 0)
                const uint64_t i = gf->base(node) + GFilt::wpos(w, gf->rwords(node));
                if (gf->packed) {   // after the node's half: a round of its own
                    acc.push_back(Acc{(uint32_t)i, K_PAIR, (uint8_t)std::min<uint32_t>(rd, 255)});
                    ++rd;
                } else {
                    acc.push_back(Acc{(uint32_t)i, K_PAIR, 0});
                }
                const uint32_t bb = GFilt::wbits(w);
                if ((gf->words[i] & bb) != bb) {
                    ++probes_fail;
                    return Hit{NODE_NONE, 0, false};
                }
            }
            ++wide_hist[16 + bk];
            if (mode & M_NOFP) {   // the probe's outcome without its loads: an absent word stops here
                std::vector<Acc> dummy;
                uint32_t r0 = 0;
                const int m0 = mode;
                const_cast<Walker*>(this)->mode = m0 & M_BLOCKS;
                const uint64_t ok0 = probes_ok, f0 = probes_fail;
                const Hit h0 = probe(node, w, dummy, r0);
                const_cast<Walker*>(this)->mode = m0;
                probes_ok = ok0;
                probes_fail = f0;
                if (h0.child == NODE_NONE) {
                    ++probes_fail;
                    return Hit{NODE_NONE, 0, false};
                }
            }
            const Hit h = probe(node, w, acc, rd);
            if (h.child != NODE_NONE) ++wide_hist[32 + bk];
            return h;
        }
        if (w == WORD_PLUS) return Hit{plus & NODE_MASK, SUM_ALL, false};
        if (w == WORD_HASH) return probe(node, WORD_HASH, acc, rd);
        return Hit{NODE_NONE, 0, false};
    }

    // the whole walk of one topic: loads appended to `acc`, step boundaries
    // in `steps` (offset of each step's first load)
    void walk(const uint32_t* W, uint32_t n, bool dollar, std::vector<Acc>& acc, std::vector<uint32_t>& steps,
              uint64_t& matches) const {
        uint32_t path[64];
        uint64_t pend = 0;
        uint32_t cv, cr;
        if (!dollar) {
            cv = ROOT;
            cr = 0;
        } else {
            steps.push_back((uint32_t)acc.size());
            acc.push_back(Acc{ROOT, K_INNER, 0});
            uint32_t rd = 1;
            const Node& q = v.nodes[ROOT];
            cv = lit(ROOT, q.plus, q.lw, q.lc, W[0], acc, rd).child;
            cr = 1;
            if (cv == NODE_NONE) return;
        }
        bool have = false;          // slotrec: the node's record came with the previous probe
        uint8_t reach = R_ROOT;
        uint32_t pair_id = NODE_NONE;   // pair: the half already in registers
        for (;;) {
            const uint32_t node = cv, r = cr;
            const bool leaf = r == n;
            uint32_t rd = 0;
            if (!have) steps.push_back((uint32_t)acc.size());
            const Node& x = v.nodes[node];
            if (have) {
                ++table_visits;
                rd = acc.empty() ? 0 : acc.back().round + 1u;   // same step, after the delivering probe
            } else if (pair_id == node && !leaf) {
                rd = 0;   // in registers: no load
                pair_id = NODE_NONE;
            } else {
                const bool pair = (mode & M_PAIR) && !leaf && (x.plus & NODE_MASK) == node + 1;
                acc.push_back(Acc{node, leaf ? K_LEAF : K_INNER, 0, reach});
                if (pair) acc.push_back(Acc{node + 1, K_PAIR, 0, reach});
                rd = 1;
                pair_id = pair ? node + 1 : NODE_NONE;
            }
            have = false;
            bool next = false;
            if (!(x.hash_filter & SUM_TAG)) ++matches;
            if (leaf) {
                if (x.self_filter != FILTER_NONE) ++matches;
            } else {
                const uint32_t w = r < 64 ? W[r] : WORD_NONE;
                const uint32_t hf = x.hash_filter;
                bool lit_ok = true, plus_ok = true;
                if (hf & SUM_TAG) {
                    const uint32_t k = n - r - 1;
                    plus_ok = sum_useful(hf & SUM_ALL, k);
                    lit_ok = w < WORD_MAX ? sum_useful((hf >> 15) & SUM_ALL, k) : w == WORD_PLUS ? plus_ok : true;
                }
                Hit g = lit_ok ? lit(node, x.plus, x.lw, x.lc, w, acc, rd) : Hit{NODE_NONE, 0, false};
                if (g.child != NODE_NONE && !(mode & M_SLOTREC) && !sum_useful(g.plus & SUM_ALL, n - r - 1))
                    g.child = NODE_NONE;
                const uint32_t pc = plus_ok ? (x.plus & NODE_MASK) : NODE_NONE;
                if (g.child != NODE_NONE) {
                    path[r] = pc;
                    pend = pc != NODE_NONE ? (pend | (1ull << r)) : (pend & ~(1ull << r));
                    cv = g.child;
                    cr = r + 1;
                    have = g.delivered;
                    reach = (x.plus & WIDE) ? R_LIT_TABLE : R_LIT_INLINE;
                    if (pair_id != NODE_NONE) pair_id = NODE_NONE;   // the '+' half is not kept past a descent
                    next = true;
                } else if (pc != NODE_NONE) {
                    pend &= ~(1ull << r);
                    cv = pc;
                    cr = r + 1;
                    ++plus_now;
                    reach = R_PLUS_NOW;
                    next = true;
                }
            }
            if (!next) {   // pop
                const uint64_t m = pend & (r >= 64 ? ~0ull : (1ull << r) - 1);
                if (!m) break;
                const uint32_t k = 63u - (uint32_t)__builtin_clzll(m);
                pend &= ~(1ull << k);
                cv = path[k];
                cr = k + 1;
                ++plus_pop;
                reach = R_PLUS_POP;
                pair_id = NODE_NONE;
            }
        }
    }
};

}  // namespace

extern "C" {

struct SimOut {
    uint64_t req[K_NKIND], l1m[K_NKIND], l2m[K_NKIND];
    uint64_t topics, steps, matches, rounds;
    uint64_t probes_ok, probes_fail, table_visits, plus_now, plus_pop, lit_inline;
    uint64_t reach_req[R_NREACH], reach_l2m[R_NREACH];   // node loads by how the node was reached
    double wave_time;        // mean over waves of the summed per-round max latency (cycles)
    double wave_rounds;      // mean over waves of the dependent rounds executed
    uint64_t waves;
};

// One XCD: `lanes` lanes (waves of 64, lanes_per_cu per CU) take the topics in
// order; in each pass every busy wave runs one walk step.  lat: cycles of an
// L1 hit, an L2 hit and an L2 miss.
int sim_run(const void* view, const uint32_t* levels, const uint32_t* words, const uint8_t* dollar, uint32_t n_topics,
            uint32_t lanes, uint32_t lanes_per_cu, uint64_t l2_bytes, uint64_t l1_bytes, const double* lat, int mode,
            SimOut* out) {
    const View& vw = *reinterpret_cast<const View*>(view);
    Walker wk(vw, mode);
    Blocks blocks;
    GFilt gfilt;
    if (mode & M_GF) {
        gfilt.build(vw, (uint32_t)((mode >> 16) & 0xFF) ? (uint32_t)((mode >> 16) & 0xFF) : 16u,
                    (uint32_t)((mode >> 24) & 0x3F), (mode & M_GFPTR) != 0);
        wk.gf = &gfilt;
    }
    if (mode & (M_BLOCKS | M_FIX)) {
        blocks.build(vw, (uint32_t)((mode >> 8) & 0xFF) ? (uint32_t)((mode >> 8) & 0xFF) : 2u);
        wk.blk = &blocks;
    }
    std::memset(out, 0, sizeof(SimOut));
    std::vector<uint64_t> woff(n_topics + 1, 0);
    for (uint32_t t = 0; t < n_topics; ++t) woff[t + 1] = woff[t] + levels[t];
    Cache l2;
    l2.init(l2_bytes, 16, 6);
    const uint32_t ncu = (lanes + lanes_per_cu - 1) / lanes_per_cu;
    std::vector<Cache> l1(ncu);
    for (auto& c : l1) c.init(l1_bytes, 8, 7);
    const uint64_t sb = (mode & M_SLOTREC) ? 32 : 16;
    const uint64_t R = 1ull << 40;
    auto addr = [&](const Acc& a) -> uint64_t {
        const uint64_t i = a.idx & 0x7FFFFFFFu, hi = a.idx >> 31;
        switch (a.kind) {
            case K_INNER: return 0 * R + i * 16;
            case K_PAIR: return (mode & M_FIX)  ? 4 * R + (uint64_t)a.idx * 16
                                : (mode & M_GF) ? 5 * R + (uint64_t)a.idx * 4 : 0 * R + i * 16;
            case K_LEAF: return 1 * R + i * 16;
            case K_COLD: return 2 * R + i * sb + hi * 16;
            default: return 3 * R + i * sb + hi * 16;
        }
    };
    struct Lane {
        std::vector<Acc> acc;
        std::vector<uint32_t> steps;
        uint32_t si = 0;
        bool busy = false;
    };
    std::vector<Lane> L(lanes);
    const uint32_t nw = (lanes + 63) / 64;
    std::vector<double> wtime(nw, 0.0), wrounds(nw, 0.0);
    uint32_t next = 0;
    auto take = [&](Lane& ln) {
        ln.busy = false;
        while (next < n_topics) {
            const uint32_t t = next++;
            ln.acc.clear();
            ln.steps.clear();
            ln.si = 0;
            uint64_t m = 0;
            wk.walk(words + woff[t], levels[t], dollar[t] != 0, ln.acc, ln.steps, m);
            out->matches += m;
            ++out->topics;
            ln.steps.push_back((uint32_t)ln.acc.size());
            if (ln.steps.size() < 2) continue;
            ln.busy = true;
            return;
        }
    };
    for (auto& ln : L) take(ln);
    double rmax[256];
    for (;;) {
        bool any = false;
        ++out->rounds;
        for (uint32_t wv = 0; wv < nw; ++wv) {
            uint32_t top = 0;
            bool stepped = false;
            for (uint32_t i = wv * 64; i < std::min(lanes, wv * 64 + 64); ++i) {
                Lane& ln = L[i];
                if (!ln.busy) continue;
                any = stepped = true;
                ++out->steps;
                Cache& c1 = l1[i / lanes_per_cu];
                for (uint32_t k = ln.steps[ln.si]; k < ln.steps[ln.si + 1]; ++k) {
                    const Acc& a = ln.acc[k];
                    const uint64_t ad = addr(a);
                    ++out->req[a.kind];
                    const bool nodeload = a.kind == K_INNER || a.kind == K_LEAF;
                    if (nodeload) ++out->reach_req[a.reach];
                    double lt = lat[0];
                    if (!c1.access(ad)) {
                        ++out->l1m[a.kind];
                        lt = lat[1];
                        if (!l2.access(ad)) {
                            ++out->l2m[a.kind];
                            if (nodeload) ++out->reach_l2m[a.reach];
                            lt = lat[2];
                        }
                    }
                    const uint32_t rd = a.round;
                    while (top <= rd) rmax[top++] = 0.0;
                    rmax[rd] = std::max(rmax[rd], lt);
                }
                ++ln.si;
                if (ln.si + 1 >= ln.steps.size()) take(ln);
            }
            if (stepped && top == 0) wtime[wv] += lat[0];   // a step of register-held halves only
            for (uint32_t j = 0; j < top; ++j) {
                wtime[wv] += rmax[j];
                wrounds[wv] += rmax[j] > 0 ? 1 : 0;
            }
        }
        if (!any) break;
    }
    double st = 0, sr = 0;
    for (uint32_t wv = 0; wv < nw; ++wv) {
        st += wtime[wv];
        sr += wrounds[wv];
    }
    out->wave_time = st / nw;
    out->wave_rounds = sr / nw;
    out->waves = nw;
    out->probes_ok = wk.probes_ok;
    out->probes_fail = wk.probes_fail;
    out->table_visits = wk.table_visits;
    out->plus_now = wk.plus_now;
    out->plus_pop = wk.plus_pop;
    out->lit_inline = wk.lit_inline;
    return 0;
}

// per-topic walk steps (node visits) and loads, no caches
int sim_per_topic(const void* view, const uint32_t* levels, const uint32_t* words, const uint8_t* dollar,
                  uint32_t n_topics, uint32_t* steps_out, uint32_t* loads_out) {
    const View& vw = *reinterpret_cast<const View*>(view);
    Walker wk(vw, 0);
    std::vector<Acc> acc;
    std::vector<uint32_t> steps;
    uint64_t wo = 0;
    for (uint32_t t = 0; t < n_topics; ++t) {
        acc.clear();
        steps.clear();
        uint64_t m = 0;
        wk.walk(words + wo, levels[t], dollar[t] != 0, acc, steps, m);
        wo += levels[t];
        steps_out[t] = (uint32_t)steps.size();
        loads_out[t] = (uint32_t)acc.size();
    }
    return 0;
}

// the walk alone (no caches): WIDE lookups by children count
int sim_count(const void* view, const uint32_t* levels, const uint32_t* words, const uint8_t* dollar,
              uint32_t n_topics, SimOut* out, uint64_t* hist48) {
    const View& vw = *reinterpret_cast<const View*>(view);
    Walker wk(vw, 0);
    std::memset(out, 0, sizeof(SimOut));
    std::vector<Acc> acc;
    std::vector<uint32_t> steps;
    uint64_t wo = 0;
    for (uint32_t t = 0; t < n_topics; ++t) {
        acc.clear();
        steps.clear();
        uint64_t m = 0;
        wk.walk(words + wo, levels[t], dollar[t] != 0, acc, steps, m);
        out->steps += steps.size();
        wo += levels[t];
        out->matches += m;
        for (const Acc& a : acc) ++out->req[a.kind];
        ++out->topics;
    }
    if (hist48) std::memcpy(hist48, wk.wide_hist, sizeof(wk.wide_hist));
    out->probes_ok = wk.probes_ok;
    out->probes_fail = wk.probes_fail;
    return 0;
}

}  // extern "C"
