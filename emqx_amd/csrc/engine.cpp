// engine.cpp — host side of libtopicmatch: the C-ABI (include/topicmatch.h),
// the subscription-trie host mirror with emqx_trie's bookkeeping, the word
// dictionary, and the HBM image it commits to the device.
//
// Reference semantics (vus520/emqx @ 3.0-rc.3):
//   insert/1      src/emqx_trie.erl:62-73, add_path/1 :104-117
//   delete/1      src/emqx_trie.erl:88-96, delete_path/1 :149-163
//   lookup/1      src/emqx_trie.erl:83-84
//   match/1       src/emqx_trie.erl:77-79, 121-145 (device: kernels.hip)
//   words/1       src/emqx_topic.erl:141-147 (device tokenizer)
//   match/2, wildcard/1, parse/1,2   src/emqx_topic.erl:41-75, 180-200
//
// The host mirror IS the host copy of the device image (image.h): inserts and
// deletes patch it in place and mark 64 KiB pages dirty; tm_commit uploads
// the dirty pages (or the whole table after a resize) on the engine stream.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/topicmatch.h"
#include "image.h"
#include "kernels.h"

using namespace tmx;

extern "C" int tm_topic_wildcard(const uint8_t* topic, uint32_t len);

namespace {

constexpr size_t PAGE_ELEMS = 4096;  // dirty granule: 4096 elements (64 KiB of 16 B slots, 128 KiB of nodes)

struct DevError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct ArgError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct RangeError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIPCHK(x)                                                                       \
    do {                                                                                \
        hipError_t _e = (x);                                                            \
        if (_e != hipSuccess)                                                           \
            throw DevError(std::string(#x) + ": " + hipGetErrorString(_e));             \
    } while (0)

// ---- word hashing, identical to the device tokenizer (image.h) --------------
uint64_t word_hash(const uint8_t* p, uint32_t len) {
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (uint32_t i = 0; i < len; i += 8) {
        uint32_t k = std::min<uint32_t>(8, len - i);
        uint64_t c = 0;
        std::memcpy(&c, p + i, k);  // little-endian host (x86_64)
        h = word_hash_step(h, c);
    }
    return word_hash_final(h, len);
}

size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// dirty-page bitmap over a table of 16 B elements
struct Dirty {
    std::vector<uint8_t> pages;
    bool all = true;  // whole table must be (re)uploaded
    void mark(size_t idx) {
        size_t pg = idx / PAGE_ELEMS;
        if (pg >= pages.size()) pages.resize(pg + 1, 0);
        pages[pg] = 1;
    }
    void clear() {
        std::fill(pages.begin(), pages.end(), 0);
        all = false;
    }
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    // grow to at least `need` bytes (contents not preserved); true if reallocated
    bool ensure(size_t need, double slack = 1.25) {
        if (need <= bytes && p) return false;
        release();
        size_t want = std::max<size_t>(256, (size_t)(need * slack));
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            throw DevError(std::string("hipMalloc(") + std::to_string(want) + "): " + hipGetErrorString(e));
        }
        bytes = want;
        return true;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

constexpr EdgeSlot empty_slot() {
    EdgeSlot e{};
    e.parent = EDGE_EMPTY;
    return e;
}
constexpr EdgeSlot kEmptySlot = empty_slot();

struct NodeAux {
    uint32_t parent;      // parent node id (root: NODE_NONE)
    uint32_t word;        // word by which the parent reaches it (id, WORD_PLUS, WORD_HASH)
    uint32_t edge_count;  // #trie_node.edge_count
    uint32_t lit_count;   // literal children (inline when 1, WIDE + edges[] once 2 or more)
};

struct FilterRec {
    uint64_t off;   // into filter arena
    uint32_t len;
    uint32_t node;  // NODE_NONE when the id is free
};

struct KTimes {
    const char* name;
    hipEvent_t a, b;
};
constexpr int N_KERNEL_SLOTS = 4;   // tokenize, walk, scan, copy_out

}  // namespace

struct tm_engine {
    std::recursive_mutex mu;
    int device = -1;
    hipStream_t stream = nullptr;
    std::string last_error;
    uint64_t epoch = 0;

    // ---- word dictionary (host copy of dict/word_arena/word_off) ----
    std::vector<DictSlot> dict;
    size_t dict_used = 0;
    std::vector<uint8_t> word_arena;   // 8-aligned, zero-padded words
    std::vector<uint32_t> word_off;
    Dirty dict_dirty;
    size_t arena_uploaded = 0, woff_uploaded = 0;

    // ---- trie mirror / image ----
    std::vector<Node> nodes;
    std::vector<NodeAux> aux;
    std::vector<uint32_t> free_nodes;
    size_t live_nodes = 0;
    // literal / '#' edges: parents with id < hot_limit (the level-by-level
    // laid-out top of the trie, depths < hot_edge_depth) keep theirs in a
    // small `hot` table, so the probes every topic makes near the root hit a
    // few MB instead of lines scattered over the whole table
    struct EdgeTable {
        std::vector<EdgeSlot> slots;
        size_t used = 0;
        Dirty dirty;
    };
    EdgeTable cold, hot;
    uint32_t hot_limit = 0;
    uint32_t hot_edge_depth = 0;      // option "hot_edges": parents of depth < D use `hot` (0 = off; A/B: no gain at C3)
    Dirty node_dirty;
    EdgeTable& tab(uint32_t parent) { return parent < hot_limit ? hot : cold; }
    const EdgeTable& tab(uint32_t parent) const { return parent < hot_limit ? hot : cold; }

    // ---- filter registry ----
    std::vector<uint8_t> filter_arena;
    std::vector<FilterRec> filters;
    std::vector<uint32_t> free_filters;
    size_t live_filters = 0;

    // ---- device image ----
    DevBuf d_nodes, d_edges, d_hedges, d_dict, d_arena, d_woff;
    bool dev_dirty = true;
    int hist_enabled = 0;             // option "hist": per-level histogram in stats mode (diagnostic, slow)
    uint32_t walk_bpc = 0;            // option "walk_bpc": walk blocks per CU (0 = full occupancy)
    int xcdq = 1;                     // option "xcdq": per-XCD dequeue ranges in the queue walk (default on)
    int group = 0;                    // option "group": walk the batch in topic-group order (kernels.hip; A/B at C3: no gain, off)
    int layout_mode = 1;              // option "layout": 0 off, 1 auto, 2 every commit (tests)
    size_t created_since_layout = 0;  // nodes created since the last relayout
    uint32_t hot_levels = 4;          // option "hot_levels": relayout puts depths <= H level by level (BFS)
                                      // first, then DFS-preorder subtrees (0 = DFS throughout)
    uint32_t edge_div = 4;            // option "edge_load": edge tables kept at load <= 1/edge_div
    uint32_t layout_order = 15;       // option "order" (default 15; A/B at C3, walk ms: 0 3.90, 1 3.84, 7 3.51-3.66, 15 3.44): bit 0 = a node's '+' child directly follows it
                                      // (the walk's most frequent step, 67 of 101 visits per topic at
                                      // C3, then lands in the line the parent's load fetched); bit 1 =
                                      // '#' nodes (never visited with words left) moved to the end;
                                      // bit 2 = heat order (heat_sort); bit 3 = heat from filter counts
    bool force_relayout = false;
    int split_halves = 1;             // option "split": walk reads separate inner / leaf half arrays
    bool split_stale = true;
    DevBuf d_inner, d_leaf;

    // ---- route table: the emqx_route bag (src/emqx_router.erl:52-59) ----
    std::unordered_map<std::string, uint32_t> dest_index;   // dest bytes -> dest id
    std::vector<std::string> dest_names;
    std::unordered_map<std::string, std::vector<uint32_t>> route_bag;   // topic -> dests, insertion order
    size_t route_total = 0;
    bool routes_dirty = true;         // the route image must be rebuilt at commit
    DevBuf d_fr_meta, d_fr_dest, d_ex_slots, d_ex_arena, d_ex_dest;
    std::vector<uint32_t> h_fr_off;   // host copy of fr_meta's offsets (aggre rewrites the ranks)
    uint64_t ex_slot_mask = 0;
    uint32_t fr_filters = 0;          // filter ids covered by fr_meta
    bool route_image = false;
    DevBuf w_rexact, w_rscan, w_rids, w_rcounts, w_roff;
    // the route / aggre workspaces (w_r*, w_d*, w_a*) and images are shared by
    // every stream: rw_done is recorded after the last route or aggre kernel
    // of a batch; the host waits on it before the next batch reuses (or
    // reallocates) the workspaces and before it rewrites an image
    hipEvent_t rw_done = nullptr;
    bool rw_used = false;
    void rw_release(hipStream_t st) {
        if (!rw_done) HIPCHK(hipEventCreateWithFlags(&rw_done, hipEventDisableTiming));
        HIPCHK(hipEventRecord(rw_done, st));
        rw_used = true;
    }
    void rw_drain() {   // host: every route / aggre kernel issued so far has finished
        if (rw_used) HIPCHK(hipEventSynchronize(rw_done));
    }

    // ---- emqx_broker:aggre/1 targets (aggre.hip) ----
    // a dest aggregates to a target: a node (atom) or a $share group; targets
    // are interned as kind byte + key bytes, so string order is the Erlang
    // term order of the X in {To, X} (atom < binary, then bytewise)
    std::unordered_map<std::string, uint32_t> target_index;
    std::vector<std::string> target_names;
    std::vector<uint32_t> dest_target;      // dest id -> target id (TARGET_DEFAULT: node named by the dest bytes)
    static constexpr uint32_t TARGET_DEFAULT = 0xFFFFFFFFu;
    struct AggKey { const std::string* key; uint32_t dest_off; uint32_t fid; };
    std::vector<AggKey> agg_keys;           // route image entries (set by build_route_image)
    bool aggre_dirty = true;
    DevBuf d_ex_rank, d_dt;
    DevBuf d_rank_src, d_rank_tg;           // inverse ranks: to_rank -> route source, target rank -> target id
    DevBuf w_dsrc, w_dcount, w_akey, w_alarge;

    // ---- match workspace ----
    DevBuf w_mpre, w_mscan, w_bytes, w_off, w_counts, w_outoff, w_ids, w_total;
    // per-batch device workspace: consecutive batches rotate over `nslots`
    // slots, so batches issued on different streams overlap on the GPU (the
    // walk of one beside the tokenizer / copy-out of its neighbours); a
    // slot's next user waits for its previous batch (hipStreamWaitEvent)
    struct Slot {
        DevBuf twords, words, path, meta, scan, stage, kstage, ws, stats, perm;
        uint64_t* h_maxc = nullptr;     // pinned: largest match count of the slot's last walk
        hipEvent_t maxc_ev = nullptr, done = nullptr;
        bool maxc_pending = false, used = false, keyed = false;
    };
    static constexpr int MAX_SLOTS = 4;
    Slot slots[MAX_SLOTS];
    int nslots = 2, next_slot = 0, last_slot = 0;   // option "slots"
    uint32_t stage_k = 512;   // TM_STAGE_K: ids staged per topic before a re-walk (rows are
                              // written sparsely: HBM footprint, not traffic)
    uint32_t stage_k_min = 512;         // option "stage_k"
    int stage_auto = 1;                 // option "stage_auto": grow K to the largest list seen (no re-walks)
    static constexpr size_t STAGE_BUDGET = 16ull << 30;  // stage-row footprint cap (bytes, of 288 GB HBM)
    bool stats_enabled = false, timing_enabled = false;
    tm_batch_stats last_stats{};
    // per-batch event records, accumulated until tm_last_kernel_times()
    std::vector<KTimes> ev_pool;          // recycled events
    std::vector<KTimes> ev_pending;       // recorded, not yet read
    KTimes ev_cur[N_KERNEL_SLOTS];

    // scratch for words of one filter
    std::vector<uint32_t> tmp_words;

    tm_engine() {
        if (const char* v = std::getenv("TM_XCDQ")) xcdq = std::atoi(v) ? 1 : 0;
        if (const char* v = std::getenv("TM_STAGE_K")) {
            long k = std::atol(v);
            if (k >= 4 && k <= 4096 && !(k & 3)) {
                stage_k = stage_k_min = (uint32_t)k;
                stage_auto = 0;
            }
        }
        dict.assign(1024, DictSlot{0, WORD_NONE, 0, {0, 0}});
        nodes.reserve(1024);
        cold.slots.assign(1024, kEmptySlot);
        hot.slots.assign(1024, kEmptySlot);
        new_node(NODE_NONE, NODE_NONE);  // root = 0
    }

    // ------------------------------------------------------------------
    // dictionary
    uint32_t dict_find(const uint8_t* p, uint32_t len, uint64_t h) const {
        size_t mask = dict.size() - 1;
        for (size_t s = h & mask;; s = (s + 1) & mask) {
            const DictSlot& d = dict[s];
            if (d.word == WORD_NONE) return WORD_NONE;
            if (d.hash == h && d.len == len && std::memcmp(&word_arena[word_off[d.word]], p, len) == 0)
                return d.word;
        }
    }
    void dict_place(uint64_t h, uint32_t id, uint32_t len) {
        size_t mask = dict.size() - 1;
        size_t s = h & mask;
        while (dict[s].word != WORD_NONE) s = (s + 1) & mask;
        DictSlot d{h, id, len, {0, 0}};
        std::memcpy(d.head, &word_arena[word_off[id]], std::min<size_t>(16, (len + 7) & ~size_t(7)));
        dict[s] = d;
        dict_dirty.mark(s);
    }
    void dict_grow() {
        std::vector<DictSlot> old;
        old.swap(dict);
        dict.assign(old.size() * 2, DictSlot{0, WORD_NONE, 0, {0, 0}});
        for (const DictSlot& d : old)
            if (d.word != WORD_NONE) dict_place(d.hash, d.word, d.len);
        dict_dirty.all = true;
    }
    // word id of a level (interning it when `intern`)
    uint32_t word_id(const uint8_t* p, uint32_t len, bool intern) {
        if (len == 1 && p[0] == '+') return WORD_PLUS;
        if (len == 1 && p[0] == '#') return WORD_HASH;
        uint64_t h = word_hash(p, len);
        uint32_t id = dict_find(p, len, h);
        if (id != WORD_NONE || !intern) return id;
        if (word_off.size() >= WORD_MAX) throw RangeError("word dictionary full");
        id = (uint32_t)word_off.size();
        size_t off = word_arena.size();
        if (off > 0xFFFFFFF0ull) throw RangeError("word arena exceeds 4 GiB");
        size_t padded = (len + 7) & ~size_t(7);
        if (padded == 0) padded = 8;  // the empty word still owns one zero chunk
        word_arena.resize(off + padded, 0);
        if (len) std::memcpy(&word_arena[off], p, len);
        word_off.push_back((uint32_t)off);
        if ((dict_used + 1) * 2 > dict.size()) dict_grow();
        dict_place(h, id, len);
        ++dict_used;
        return id;
    }
    // emqx_topic:words/1 (src/emqx_topic.erl:141-147): split on every '/',
    // N slashes -> N+1 levels, empty levels kept.
    bool split_words(const uint8_t* p, uint32_t len, bool intern) {
        tmp_words.clear();
        uint32_t s = 0;
        for (uint32_t i = 0; i <= len; ++i) {
            if (i == len || p[i] == '/') {
                uint32_t w = word_id(p + s, i - s, intern);
                if (w == WORD_NONE) return false;  // cannot be on any trie path
                tmp_words.push_back(w);
                s = i + 1;
            }
        }
        return true;
    }

    // ------------------------------------------------------------------
    // edges (open addressing, linear probing over 16 B slots from the home
    // bucket's first slot; backward-shift deletion keeps probes tombstone-free)
    size_t edge_find_slot(uint32_t parent, uint32_t word) const {
        const std::vector<EdgeSlot>& edges = tab(parent).slots;
        size_t mask = edges.size() - 1;
        for (size_t s = edge_home(parent, word, mask);; s = (s + 1) & mask) {
            const EdgeSlot& e = edges[s];
            if (e.parent == EDGE_EMPTY) return SIZE_MAX;
            if (e.parent == parent && e.word == word) return s;
        }
    }
    static void place_in(EdgeTable& t, const EdgeSlot& x) {
        size_t mask = t.slots.size() - 1;
        size_t s = edge_home(x.parent, x.word, mask);
        while (t.slots[s].parent != EDGE_EMPTY) s = (s + 1) & mask;
        t.slots[s] = x;
        t.dirty.mark(s);
    }
    void edge_place(const EdgeSlot& x) { place_in(tab(x.parent), x); }
    static void edge_grow(EdgeTable& t) {
        std::vector<EdgeSlot> old;
        old.swap(t.slots);
        t.slots.assign(old.size() * 2, kEmptySlot);
        for (const EdgeSlot& e : old)
            if (e.parent != EDGE_EMPTY) place_in(t, e);
        t.dirty.all = true;
    }
    EdgeSlot slot_for(uint32_t parent, uint32_t word, uint32_t child) const {
        const Node& c = nodes[child];
        EdgeSlot e{};
        e.parent = parent;
        e.word = word;
        e.child = child;
        e.plus = c.plus;
#if TM_SLOT_RECORD
        e.hash_filter = c.hash_filter;
        e.lw = c.lw;
        e.lc = c.lc;
        e.self_filter = c.self_filter;
#endif
        return e;
    }
    void edge_insert(uint32_t parent, uint32_t word, uint32_t child) {
        EdgeTable& t = tab(parent);
        if ((t.used + 1) * edge_div > t.slots.size()) edge_grow(t);
        place_in(t, slot_for(parent, word, child));
        ++t.used;
    }
    // node x changed: mark its page and refresh the copy of its record in
    // its parent's edge slot (when it is a table child)
    void touched(uint32_t x) {
        node_dirty.mark(x);
        if (!SLOT_RECORD) return;
        const uint32_t p = aux[x].parent, w = aux[x].word;
        if (p == NODE_NONE || w == WORD_PLUS) return;
        if (w != WORD_HASH && !(nodes[p].plus & WIDE)) return;
        const size_t s = edge_find_slot(p, w);
        if (s == SIZE_MAX) return;
        tab(p).slots[s] = slot_for(p, w, x);
        tab(p).dirty.mark(s);
    }
    void edge_erase(uint32_t parent, uint32_t word) {
        size_t i = edge_find_slot(parent, word);
        if (i == SIZE_MAX) return;
        EdgeTable& t = tab(parent);
        std::vector<EdgeSlot>& edges = t.slots;
        Dirty& edge_dirty = t.dirty;
        size_t mask = edges.size() - 1;
        size_t j = i;
        for (;;) {
            j = (j + 1) & mask;
            if (edges[j].parent == EDGE_EMPTY) break;
            size_t k = edge_home(edges[j].parent, edges[j].word, mask);
            bool move = (i <= j) ? (k <= i || k > j) : (k <= i && k > j);
            if (move) {
                edges[i] = edges[j];
                edge_dirty.mark(i);
                i = j;
            }
        }
        edges[i] = kEmptySlot;
        edge_dirty.mark(i);
        --t.used;
    }

    // ------------------------------------------------------------------
    // nodes
    uint32_t new_node(uint32_t parent, uint32_t word) {
        uint32_t id;
        if (!free_nodes.empty()) {
            id = free_nodes.back();
            free_nodes.pop_back();
        } else {
            if (nodes.size() >= NODE_NONE) throw RangeError("trie exceeds 2^29-1 nodes");
            id = (uint32_t)nodes.size();
            nodes.push_back(Node{});
            aux.push_back(NodeAux{});
        }
        nodes[id] = empty_node();
        aux[id] = NodeAux{parent, word, 0, 0};
        node_dirty.mark(id);
        ++live_nodes;
        ++created_since_layout;
        return id;
    }
    static Node empty_node() {
        Node x;
        x.plus = NODE_NONE;
        x.hash_filter = FILTER_NONE;
        x.lw = WORD_NONE;
        x.lc = NODE_NONE;
        x.self_filter = FILTER_NONE;
        x.hash_filter2 = FILTER_NONE;
        x.hash = NODE_NONE;
        x.pad = 0;
        return x;
    }
    uint32_t child(uint32_t v, uint32_t w) const {
        const Node& x = nodes[v];
        if (w == WORD_PLUS) return x.plus & NODE_MASK;
        if (w == WORD_HASH) return x.hash;
        if (!(x.plus & WIDE)) return x.lw == w ? x.lc : NODE_NONE;
        size_t s = edge_find_slot(v, w);
        return s == SIZE_MAX ? NODE_NONE : tab(v).slots[s].child;
    }
    // literal child add / remove: one literal child lives inline (lw, lc);
    // from the second on, all of them live in edges[] (WIDE), and lw:lc
    // hold a Bloom mask of their words (a superset after deletes; rebuilt
    // exactly on relayout)
    static void bloom_add(Node& x, uint32_t w) {
        const uint64_t b = word_bloom(w);
        x.lw |= (uint32_t)b;
        x.lc |= (uint32_t)(b >> 32);
    }
    void lit_add(uint32_t v, uint32_t w, uint32_t c) {
        Node& x = nodes[v];
        if (!(x.plus & WIDE)) {
            if (x.lw == WORD_NONE) {
                x.lw = w;
                x.lc = c;
                return;
            }
            edge_insert(v, x.lw, x.lc);  // spill the inline pair to the table
            Node& y = nodes[v];
            const uint32_t w0 = y.lw;
            y.plus |= WIDE;
            y.lw = 0;
            y.lc = 0;
            bloom_add(y, w0);
        }
        edge_insert(v, w, c);
        bloom_add(nodes[v], w);
    }
    void lit_remove(uint32_t v, uint32_t w) {
        Node& x = nodes[v];
        if (x.plus & WIDE) {
            edge_erase(v, w);
        } else if (x.lw == w) {
            x.lw = WORD_NONE;
            x.lc = NODE_NONE;
        }
        if (--aux[v].lit_count == 0) {
            nodes[v].plus &= ~WIDE;
            nodes[v].lw = WORD_NONE;
            nodes[v].lc = NODE_NONE;
        }
    }
    // add_path/1 (emqx_trie.erl:104-117) for one (Node, Word, Child) triple:
    // a new edge bumps the parent's edge_count.
    uint32_t child_or_create(uint32_t v, uint32_t w) {
        uint32_t c = child(v, w);
        if (c != NODE_NONE) return c;
        c = new_node(v, w);
        if (w == WORD_PLUS) {
            nodes[v].plus = (nodes[v].plus & WIDE) | c;
        } else if (w == WORD_HASH) {
            nodes[v].hash = c;
            edge_insert(v, WORD_HASH, c);
        } else {
            lit_add(v, w, c);
            aux[v].lit_count++;
        }
        aux[v].edge_count++;
        touched(v);
        return c;
    }
    void unlink_child(uint32_t c) {
        uint32_t v = aux[c].parent, w = aux[c].word;
        if (w == WORD_PLUS) {
            nodes[v].plus = (nodes[v].plus & WIDE) | NODE_NONE;
        } else if (w == WORD_HASH) {
            nodes[v].hash = NODE_NONE;
            nodes[v].hash_filter = FILTER_NONE;
            nodes[v].hash_filter2 = FILTER_NONE;
            edge_erase(v, WORD_HASH);
        } else {
            lit_remove(v, w);
        }
        aux[v].edge_count--;
        touched(v);
        nodes[c] = empty_node();
        aux[c] = NodeAux{NODE_NONE, 0, 0, 0};
        node_dirty.mark(c);
        free_nodes.push_back(c);
        --live_nodes;
    }
    uint32_t walk(const std::vector<uint32_t>& ws) const {
        uint32_t v = ROOT;
        for (uint32_t w : ws) {
            v = child(v, w);
            if (v == NODE_NONE) return NODE_NONE;
        }
        return v;
    }
    // set/clear #trie_node.topic of node c (and the inline copy in the parent
    // when c is a '#' child)
    void set_topic(uint32_t c, uint32_t fid) {
        nodes[c].self_filter = fid;
        touched(c);
        if (aux[c].word == WORD_HASH && aux[c].parent != NODE_NONE) {
            nodes[aux[c].parent].hash_filter = fid;
            nodes[aux[c].parent].hash_filter2 = fid;
            touched(aux[c].parent);
        }
    }

    // ------------------------------------------------------------------
    // filters
    uint32_t new_filter(const uint8_t* p, uint32_t len, uint32_t node) {
        uint32_t id;
        if (!free_filters.empty()) {
            id = free_filters.back();
            free_filters.pop_back();
        } else {
            if (filters.size() >= 0xFFFFFFF0ull) throw RangeError("filter ids exhausted");
            id = (uint32_t)filters.size();
            filters.push_back(FilterRec{});
        }
        uint64_t off = filter_arena.size();
        filter_arena.insert(filter_arena.end(), p, p + len);
        filters[id] = FilterRec{off, len, node};
        ++live_filters;
        return id;
    }
    void free_filter(uint32_t id) {
        filters[id].node = NODE_NONE;
        free_filters.push_back(id);
        --live_filters;
    }

    // emqx_trie:insert/1 (src/emqx_trie.erl:62-73)
    void insert(const uint8_t* p, uint32_t len) {
        split_words(p, len, true);
        uint32_t v = ROOT;
        for (uint32_t w : tmp_words) v = child_or_create(v, w);
        if (nodes[v].self_filter == FILTER_NONE) set_topic(v, new_filter(p, len, v));
        dev_dirty = true;
        routes_dirty = true;   // filter ids may have changed
    }

    // emqx_trie:delete/1 (src/emqx_trie.erl:88-96) + delete_path/1 (:149-163)
    void remove(const uint8_t* p, uint32_t len) {
        if (!split_words(p, len, false)) return;  // [] -> ok
        uint32_t v = walk(tmp_words);
        if (v == NODE_NONE) return;               // [] -> ok
        uint32_t fid = nodes[v].self_filter;
        if (fid != FILTER_NONE) {
            set_topic(v, FILTER_NONE);
            free_filter(fid);
        }
        if (aux[v].edge_count == 0) {
            // [#trie_node{edge_count = 0}] -> delete node, then walk up removing
            // nodes whose edge_count drops to 0 with topic = undefined
            for (;;) {
                uint32_t parent = aux[v].parent;
                unlink_child(v);
                if (parent == ROOT || aux[parent].edge_count != 0 ||
                    nodes[parent].self_filter != FILTER_NONE)
                    break;
                v = parent;
            }
        }
        dev_dirty = true;
        routes_dirty = true;
    }

    // ------------------------------------------------------------------
    // routes (emqx_router.erl): add_route/del_route with the reference's
    // trie bookkeeping, get_routes/1, and the route image match_routes/1 reads
    uint32_t intern_dest(const uint8_t* d, uint32_t dlen) {
        std::string k(reinterpret_cast<const char*>(d), dlen);
        auto it = dest_index.find(k);
        if (it != dest_index.end()) return it->second;
        if (dest_names.size() >= 0xFFFFFFF0ull) throw RangeError("dest ids exhausted");
        const uint32_t id = (uint32_t)dest_names.size();
        dest_names.push_back(k);
        dest_index.emplace(std::move(k), id);
        return id;
    }
    // handle_cast({add_route, Route}) (:153-163) + add_trie_route/1 (:226-231)
    void route_add(const uint8_t* t, uint32_t tlen, const uint8_t* d, uint32_t dlen) {
        const uint32_t dest = intern_dest(d, dlen);
        std::string key(reinterpret_cast<const char*>(t), tlen);
        auto it = route_bag.find(key);
        if (it != route_bag.end() &&
            std::find(it->second.begin(), it->second.end(), dest) != it->second.end())
            return;   // lists:member(Route, get_routes(Topic)) -> ok
        const bool had = it != route_bag.end() && !it->second.empty();
        if (tm_topic_wildcard(t, tlen) && !had) insert(t, tlen);   // mnesia:wread -> [] -> emqx_trie:insert
        route_bag[key].push_back(dest);
        ++route_total;
        routes_dirty = true;
    }
    // handle_cast({del_route, Route}) (:165-187) + del_trie_route/1 (:252-260)
    // or del_direct_route/1 (:240-241); the emqx_subscriber check (:179) is
    // the broker's and stays in the caller
    void route_del(const uint8_t* t, uint32_t tlen, const uint8_t* d, uint32_t dlen) {
        auto di = dest_index.find(std::string(reinterpret_cast<const char*>(d), dlen));
        if (di == dest_index.end()) return;
        auto it = route_bag.find(std::string(reinterpret_cast<const char*>(t), tlen));
        if (it == route_bag.end()) return;   // [] -> ok
        std::vector<uint32_t>& bag = it->second;
        auto pos = std::find(bag.begin(), bag.end(), di->second);
        if (pos == bag.end()) return;        // delete_object of an absent route: no-op
        const bool last = bag.size() == 1;
        bag.erase(pos);
        --route_total;
        if (last) {
            route_bag.erase(it);
            if (tm_topic_wildcard(t, tlen)) remove(t, tlen);   // [Route] -> emqx_trie:delete(Topic)
        }
        routes_dirty = true;
    }
    const std::vector<uint32_t>* get_routes(const uint8_t* t, uint32_t tlen) const {
        auto it = route_bag.find(std::string(reinterpret_cast<const char*>(t), tlen));
        return it == route_bag.end() ? nullptr : &it->second;
    }
    // filter id of a trie filter (or FILTER_NONE)
    uint32_t filter_of(const uint8_t* p, uint32_t len) {
        if (!split_words(p, len, false)) return FILTER_NONE;
        const uint32_t v = walk(tmp_words);
        return v == NODE_NONE ? FILTER_NONE : nodes[v].self_filter;
    }
    // rebuild the route image: per-filter-id dest lists (CSR) and the
    // exact-topic table over every topic with routes
    void build_route_image() {
        rw_drain();   // no route / aggre kernel may read the image being replaced
        const uint32_t nf = (uint32_t)filters.size();
        std::vector<uint32_t> fr_off(nf + 1, 0);
        std::vector<std::pair<uint32_t, const std::vector<uint32_t>*>> by_fid;
        by_fid.reserve(route_bag.size());
        size_t cap = 16;
        while (cap < route_bag.size() * 2) cap <<= 1;
        std::vector<ExactSlot> slots(cap);
        for (auto& x : slots) x = ExactSlot{0, 0, 0, 0, 0, 0};
        std::vector<uint8_t> arena;
        std::vector<uint32_t> ex_dest;
        ex_dest.reserve(route_total);
        agg_keys.clear();
        agg_keys.reserve(route_bag.size());
        aggre_dirty = true;
        for (const auto& kv : route_bag) {
            const uint8_t* t = reinterpret_cast<const uint8_t*>(kv.first.data());
            const uint32_t tlen = (uint32_t)kv.first.size();
            uint32_t fid = FILTER_NONE;
            if (tm_topic_wildcard(t, tlen)) {
                fid = filter_of(t, tlen);
                if (fid != FILTER_NONE) {
                    fr_off[fid + 1] = (uint32_t)kv.second.size();
                    by_fid.emplace_back(fid, &kv.second);
                }
            }
            agg_keys.push_back(AggKey{&kv.first, (uint32_t)ex_dest.size(), fid});
            const uint64_t h = word_hash(t, tlen);
            size_t sl = h & (cap - 1);
            while (slots[sl].hash) sl = (sl + 1) & (cap - 1);
            ExactSlot& e = slots[sl];
            e.hash = h;
            e.len = tlen;
            e.count = (uint32_t)kv.second.size();
            e.arena = arena.size();
            e.dest_off = (uint32_t)ex_dest.size();
            arena.resize(arena.size() + std::max<size_t>(8, (tlen + 7) & ~size_t(7)), 0);
            if (tlen) std::memcpy(&arena[e.arena], t, tlen);
            ex_dest.insert(ex_dest.end(), kv.second.begin(), kv.second.end());
        }
        for (uint32_t f = 0; f < nf; ++f) fr_off[f + 1] += fr_off[f];
        std::vector<uint32_t> fr_dest(fr_off[nf]);
        for (const auto& x : by_fid) std::copy(x.second->begin(), x.second->end(), fr_dest.begin() + fr_off[x.first]);
        auto up = [&](DevBuf& b, const void* src, size_t bytes) {
            b.ensure(std::max<size_t>(bytes, 16));
            if (bytes) HIPCHK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, stream));
        };
        {
            std::vector<uint2> meta(fr_off.size());
            for (size_t f = 0; f < fr_off.size(); ++f) meta[f] = make_uint2(fr_off[f], 0u);
            up(d_fr_meta, meta.data(), meta.size() * sizeof(uint2));
            HIPCHK(hipStreamSynchronize(stream));
        }
        up(d_fr_dest, fr_dest.data(), fr_dest.size() * 4);
        up(d_ex_slots, slots.data(), slots.size() * sizeof(ExactSlot));
        up(d_ex_arena, arena.data(), arena.size());
        up(d_ex_dest, ex_dest.data(), ex_dest.size() * 4);
        ex_slot_mask = cap - 1;
        fr_filters = nf;
        route_image = !route_bag.empty();
        HIPCHK(hipStreamSynchronize(stream));   // host vectors die here
        h_fr_off.swap(fr_off);
        routes_dirty = false;
    }
    // ------------------------------------------------------------------
    // emqx_broker:aggre/1 (src/emqx_broker.erl:194-206) tables: to_rank of
    // every topic with routes (std::string order = Erlang binary order:
    // bytewise unsigned, a proper prefix first), and per dest its target's
    // rank and id.  Rebuilt after the route image or a target changes.
    uint32_t intern_target(uint32_t kind, const uint8_t* k, uint32_t klen) {
        std::string key(1, (char)kind);
        key.append(reinterpret_cast<const char*>(k), klen);
        auto it = target_index.find(key);
        if (it != target_index.end()) return it->second;
        if (target_names.size() >= 0x7FFFFFF0ull) throw RangeError("target ids exhausted");
        const uint32_t id = (uint32_t)target_names.size();
        target_names.push_back(key);
        target_index.emplace(std::move(key), id);
        return id;
    }
    void build_aggre_image() {
        rw_drain();
        const uint32_t nf = fr_filters;
        std::vector<uint32_t> order(agg_keys.size());
        for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
        std::sort(order.begin(), order.end(),
                  [&](uint32_t a, uint32_t b) { return *agg_keys[a].key < *agg_keys[b].key; });
        std::vector<uint2> fr_meta(h_fr_off.size());
        for (size_t f = 0; f < h_fr_off.size(); ++f) fr_meta[f] = make_uint2(h_fr_off[f], 0u);
        std::vector<uint32_t> ex_rank(std::max<size_t>(route_total, 1), 0);
        std::vector<uint32_t> rank_src(std::max<size_t>(order.size(), 1), TM_ROUTE_TOPIC_ID);
        for (uint32_t r = 0; r < order.size(); ++r) {
            const AggKey& a = agg_keys[order[r]];
            if (a.fid != FILTER_NONE && a.fid < nf) fr_meta[a.fid].y = r;
            if (a.dest_off < ex_rank.size()) ex_rank[a.dest_off] = r;
            // the To of rank r as a route source: its filter id when it is a
            // trie filter, else the literal topic (same To binary either way)
            rank_src[r] = a.fid != FILTER_NONE ? a.fid : TM_ROUTE_TOPIC_ID;
        }
        const size_t nd = dest_names.size();
        dest_target.resize(nd, TARGET_DEFAULT);
        for (size_t d = 0; d < nd; ++d)
            if (dest_target[d] == TARGET_DEFAULT)
                dest_target[d] = intern_target(0, reinterpret_cast<const uint8_t*>(dest_names[d].data()),
                                               (uint32_t)dest_names[d].size());
        if (target_names.size() >= (1u << 25))   // aggre.hip packs rank << 7 | index into 32 bits
            throw RangeError("aggre: more than 2^25 targets");
        std::vector<uint32_t> tord(target_names.size()), trank(target_names.size());
        for (uint32_t i = 0; i < tord.size(); ++i) tord[i] = i;
        std::sort(tord.begin(), tord.end(), [&](uint32_t a, uint32_t b) { return target_names[a] < target_names[b]; });
        for (uint32_t r = 0; r < tord.size(); ++r) trank[tord[r]] = r;
        std::vector<uint32_t> rank_tg(std::max<size_t>(tord.size(), 1), 0);
        for (uint32_t r = 0; r < tord.size(); ++r) rank_tg[r] = tord[r];
        std::vector<uint2> dt(std::max<size_t>(nd, 1));
        for (size_t d = 0; d < nd; ++d) {
            const uint32_t tid = dest_target[d];
            dt[d] = make_uint2(trank[tid], tid | (target_names[tid][0] ? 0x80000000u : 0u));
        }
        auto up = [&](DevBuf& b, const void* src, size_t bytes) {
            b.ensure(std::max<size_t>(bytes, 16));
            if (bytes) HIPCHK(hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, stream));
        };
        if (!fr_meta.empty()) up(d_fr_meta, fr_meta.data(), fr_meta.size() * sizeof(uint2));
        up(d_ex_rank, ex_rank.data(), ex_rank.size() * 4);
        up(d_dt, dt.data(), dt.size() * sizeof(uint2));
        up(d_rank_src, rank_src.data(), rank_src.size() * 4);
        up(d_rank_tg, rank_tg.data(), rank_tg.size() * 4);
        HIPCHK(hipStreamSynchronize(stream));   // host vectors die here
        aggre_dirty = false;
    }
    AggreView aggre_view() const {
        AggreView av;
        av.ex_rank = d_ex_rank.as<const uint32_t>();
        av.dt = d_dt.as<const uint2>();
        av.rank_src = d_rank_src.as<const uint32_t>();
        av.rank_tg = d_rank_tg.as<const uint32_t>();
        return av;
    }

    RouteView route_view() const {
        RouteView rv;
        rv.fr_meta = d_fr_meta.as<const uint2>();
        rv.fr_dest = d_fr_dest.as<const uint32_t>();
        rv.n_filters = route_image ? fr_filters : 0u;
        rv.ex_slots = route_image ? d_ex_slots.as<const ExactSlot>() : nullptr;
        rv.ex_slot_mask = ex_slot_mask;
        rv.ex_arena = d_ex_arena.as<const uint8_t>();
        rv.ex_dest = d_ex_dest.as<const uint32_t>();
        return rv;
    }

    // ------------------------------------------------------------------
    // Heat order (option "order" bit 2): nodes sorted by the estimated share
    // of publishes that visit them, hottest first, so each 64 B line of the
    // hot end of inner[] holds four hot halves and the set a cache level can
    // hold is as hot as it gets.  A topic visits v iff its words equal v's
    // literal levels ('+' levels take any word), so heat(v) = product over
    // v's literal levels of P(word); P is estimated from the trie itself (a
    // word's share of all literal edges: subscriptions and publishes draw on
    // one vocabulary).  '#' nodes are never visited with words left: last.
    // The sort is stable over the preorder built above, so a node and its
    // '+' child (equal heat) stay adjacent.
    void heat_sort(std::vector<uint32_t>& order, std::vector<uint32_t>& newid, uint32_t& new_hot_limit) {
        std::unordered_map<uint32_t, uint64_t> wcnt;
        uint64_t total = 0;
        if (layout_order & 8) {   // P(word) from the filters through each edge (subtree filter counts)
            std::vector<uint32_t> sub(nodes.size(), 0);
            for (size_t i = order.size(); i-- > 0;) {   // preorder reversed: children before parents
                const uint32_t v = order[i];
                sub[v] += nodes[v].self_filter != FILTER_NONE ? 1u : 0u;
                if (v == ROOT) continue;
                sub[aux[v].parent] += sub[v];
                if (aux[v].word < WORD_MAX) {
                    wcnt[aux[v].word] += sub[v];
                    total += sub[v];
                }
            }
        } else {                  // P(word) from the number of edges labelled with it
            for (uint32_t v : order)
                if (v != ROOT && aux[v].word < WORD_MAX) {
                    ++wcnt[aux[v].word];
                    ++total;
                }
        }
        std::unordered_map<uint32_t, double> wlog;
        wlog.reserve(wcnt.size());
        for (const auto& kv : wcnt) wlog[kv.first] = std::log((double)kv.second / (double)total);
        std::vector<double> heat(nodes.size(), 0.0);   // log P(visit)
        const double COLD = -1e300;
        for (uint32_t v : order) {
            if (v == ROOT) continue;
            const uint32_t p = aux[v].parent, w = aux[v].word;
            const double hp = heat[p];
            heat[v] = w == WORD_PLUS ? hp : w == WORD_HASH || hp == COLD ? COLD : hp + wlog[w];
        }
        struct Key {
            double h;
            uint32_t i;   // position in the preorder (ties keep it)
        };
        std::vector<Key> keys(order.size());
        for (size_t i = 0; i < order.size(); ++i) keys[i] = Key{heat[order[i]], (uint32_t)i};
        std::vector<double>().swap(heat);
        std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) { return a.h > b.h || (a.h == b.h && a.i < b.i); });
        std::vector<uint32_t> sorted(order.size());
        for (size_t i = 0; i < keys.size(); ++i) sorted[i] = order[keys[i].i];
        order.swap(sorted);
        for (size_t i = 0; i < order.size(); ++i) newid[order[i]] = (uint32_t)i;
        new_hot_limit = 0;   // the depth-based hot edge table does not apply
    }

    // ------------------------------------------------------------------
    // DFS-preorder relayout: renumber the live nodes so that every subtree is
    // a contiguous id range and a node's first child in walk order (its
    // literal children, then its '+' child: the walk runs in the reference's
    // discovery order) directly follows it, two 32 B records to a 64 B line;
    // topics with a common prefix walk a compact region.  Deleted ids are
    // dropped (compaction).  Filter ids are unchanged.
    void relayout() {
        const size_t N = nodes.size();
        // literal children per node (inline or table edges), CSR
        std::vector<uint32_t> start(N + 1, 0);
        for (size_t v = 0; v < N; ++v) {
            if (aux[v].parent == NODE_NONE && v != ROOT) continue;  // free slot
            if (!(nodes[v].plus & WIDE) && nodes[v].lw != WORD_NONE) start[v + 1]++;
        }
        for (const EdgeTable* t : {&cold, &hot})
            for (const EdgeSlot& e : t->slots)
                if (e.parent != EDGE_EMPTY && e.word != WORD_HASH) start[e.parent + 1]++;
        for (size_t v = 0; v < N; ++v) start[v + 1] += start[v];
        std::vector<uint32_t> kids(start[N]);
        {
            std::vector<uint32_t> fill(start.begin(), start.end() - 1);
            for (size_t v = 0; v < N; ++v) {
                if (aux[v].parent == NODE_NONE && v != ROOT) continue;
                if (!(nodes[v].plus & WIDE) && nodes[v].lw != WORD_NONE) kids[fill[v]++] = nodes[v].lc;
            }
            for (const EdgeTable* t : {&cold, &hot})
                for (const EdgeSlot& e : t->slots)
                    if (e.parent != EDGE_EMPTY && e.word != WORD_HASH) kids[fill[e.parent]++] = e.child;
        }
        // preorder: v, literal subtrees, '+' subtree, '#' subtree; with
        // hot_levels = H, depths 0..H first, level by level (each node's
        // children contiguous, in the same order), then the subtrees below
        // depth H in preorder
        std::vector<uint32_t> newid(N, NODE_NONE), order;
        order.reserve(live_nodes);
        std::vector<uint32_t> stack;
        const bool plus_first = layout_order & 1, hash_last = layout_order & 2;
        std::vector<uint32_t> deferred;   // '#' nodes (hash_last)
        auto children = [&](uint32_t v, std::vector<uint32_t>& out) {   // walk order
            uint32_t pc = nodes[v].plus & NODE_MASK;
            if (plus_first && pc != NODE_NONE) out.push_back(pc);
            for (uint32_t k = start[v]; k < start[v + 1]; ++k) out.push_back(kids[k]);
            if (!plus_first && pc != NODE_NONE) out.push_back(pc);
            if (nodes[v].hash != NODE_NONE) (hash_last ? deferred : out).push_back(nodes[v].hash);
        };
        uint32_t new_hot_limit = 0;
        if (hot_levels > 0) {
            std::vector<uint32_t> cur{ROOT}, next;
            for (uint32_t d = 0; d <= hot_levels && !cur.empty(); ++d) {
                next.clear();
                for (uint32_t v : cur) {
                    newid[v] = (uint32_t)order.size();
                    order.push_back(v);
                    children(v, next);
                }
                cur.swap(next);
                if (d + 1 == hot_edge_depth) new_hot_limit = (uint32_t)order.size();   // depths < D
            }
            if (hot_edge_depth > hot_levels + 1) new_hot_limit = (uint32_t)order.size();
            for (auto it = cur.rbegin(); it != cur.rend(); ++it) stack.push_back(*it);
        } else {
            stack.push_back(ROOT);
        }
        while (!stack.empty()) {
            uint32_t v = stack.back();
            stack.pop_back();
            newid[v] = (uint32_t)order.size();
            order.push_back(v);
            if (nodes[v].hash != NODE_NONE) (hash_last ? deferred : stack).push_back(nodes[v].hash);
            uint32_t pc = nodes[v].plus & NODE_MASK;
            if (!plus_first && pc != NODE_NONE) stack.push_back(pc);
            for (uint32_t k = start[v + 1]; k > start[v]; --k) stack.push_back(kids[k - 1]);
            if (plus_first && pc != NODE_NONE) stack.push_back(pc);
        }
        // '#' nodes have no children on valid filters; any subtree below one
        // (a literal "#" level in a filter) is laid out in preorder after it
        for (size_t i = 0; i < deferred.size(); ++i) {
            stack.push_back(deferred[i]);
            while (!stack.empty()) {
                uint32_t v = stack.back();
                stack.pop_back();
                if (newid[v] != NODE_NONE) continue;
                newid[v] = (uint32_t)order.size();
                order.push_back(v);
                if (nodes[v].hash != NODE_NONE) stack.push_back(nodes[v].hash);
                if ((nodes[v].plus & NODE_MASK) != NODE_NONE) stack.push_back(nodes[v].plus & NODE_MASK);
                for (uint32_t k = start[v + 1]; k > start[v]; --k) stack.push_back(kids[k - 1]);
            }
        }
        std::vector<uint32_t>().swap(kids);
        std::vector<uint32_t>().swap(start);
        if (layout_order & 4) heat_sort(order, newid, new_hot_limit);
        auto remap = [&](uint32_t id) { return id == NODE_NONE ? NODE_NONE : newid[id]; };
        std::vector<Node> nn(order.size());
        std::vector<NodeAux> na(order.size());
        for (size_t i = 0; i < order.size(); ++i) {
            Node x = nodes[order[i]];
            x.plus = (x.plus & WIDE) | remap(x.plus & NODE_MASK);
            x.hash = remap(x.hash);
            if (x.plus & WIDE) x.lw = x.lc = 0;   // Bloom rebuilt exactly below
            else if (x.lw != WORD_NONE) x.lc = remap(x.lc);
            nn[i] = x;
            NodeAux a = aux[order[i]];
            a.parent = remap(a.parent);
            na[i] = a;
        }
        // edge tables with the new ids: parents below the new hot limit in `hot`
        std::vector<EdgeSlot> old;
        old.reserve(cold.used + hot.used);
        for (EdgeTable* t : {&cold, &hot}) {
            for (const EdgeSlot& e : t->slots)
                if (e.parent != EDGE_EMPTY) old.push_back(e);
            std::vector<EdgeSlot>().swap(t->slots);
            t->used = 0;
        }
        for (const EdgeSlot& e : old)
            if (e.word != WORD_HASH) bloom_add(nn[newid[e.parent]], e.word);
        nodes.swap(nn);
        hot_limit = new_hot_limit;
        size_t nhot = 0;
        for (const EdgeSlot& e : old) nhot += newid[e.parent] < hot_limit;
        cold.slots.assign(std::max<size_t>(1024, next_pow2((old.size() - nhot) * edge_div + 1)), kEmptySlot);
        hot.slots.assign(std::max<size_t>(1024, next_pow2(nhot * edge_div + 1)), kEmptySlot);
        // placed in order of the children's new ids: under the heat order the
        // most visited edges are placed first and sit in their home slots
        std::sort(old.begin(), old.end(),
                  [&](const EdgeSlot& a, const EdgeSlot& b) { return newid[a.child] < newid[b.child]; });
        for (const EdgeSlot& e : old) {
            edge_place(slot_for(newid[e.parent], e.word, newid[e.child]));
            ++tab(newid[e.parent]).used;
        }
        for (FilterRec& f : filters)
            if (f.node != NODE_NONE) f.node = newid[f.node];
        aux.swap(na);
        free_nodes.clear();
        created_since_layout = 0;
        force_relayout = false;
        node_dirty.all = true;
        cold.dirty.all = true;
        hot.dirty.all = true;
    }

    // ------------------------------------------------------------------
    // device image
    struct Guard {
        int prev = -1;
        explicit Guard(int dev) {
            (void)hipGetDevice(&prev);
            HIPCHK(hipSetDevice(dev));
        }
        ~Guard() {
            if (prev >= 0) (void)hipSetDevice(prev);
        }
    };

    ImageView view() const {
        ImageView im;
        if (split_halves && d_inner.p && !split_stale) {
            im.inner = d_inner.as<const uint8_t>();
            im.leaf = d_leaf.as<const uint8_t>();
            im.node_shift = 4;
        } else {
            im.inner = d_nodes.as<const uint8_t>();
            im.leaf = d_nodes.as<const uint8_t>() + 16;
            im.node_shift = 5;
        }
        im.edges = d_edges.as<const EdgeSlot>();
        im.edge_slot_mask = cold.slots.size() - 1;
        im.hot_edges = d_hedges.as<const EdgeSlot>();
        im.hot_slot_mask = hot.slots.size() - 1;
        im.hot_limit = hot_limit;
        im.dict = d_dict.as<const DictSlot>();
        im.dict_slot_mask = dict.size() - 1;
        im.word_arena = d_arena.as<const uint8_t>();
        im.word_off = d_woff.as<const uint32_t>();
        return im;
    }

    template <class T>
    void upload_table(DevBuf& buf, const std::vector<T>& host, Dirty& dirty, size_t dev_elems_min) {
        size_t need = std::max(host.size(), dev_elems_min) * sizeof(T);
        bool re = buf.ensure(need);
        if (re || dirty.all) {
            HIPCHK(hipMemcpyAsync(buf.p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice, stream));
        } else {
            size_t np = dirty.pages.size();
            for (size_t pg = 0; pg < np;) {
                if (!dirty.pages[pg]) { ++pg; continue; }
                size_t q = pg;
                while (q < np && dirty.pages[q]) ++q;
                size_t a = pg * PAGE_ELEMS, b = std::min(host.size(), q * PAGE_ELEMS);
                if (a < b)
                    HIPCHK(hipMemcpyAsync(buf.as<T>() + a, host.data() + a, (b - a) * sizeof(T),
                                          hipMemcpyHostToDevice, stream));
                pg = q;
            }
        }
        dirty.clear();
    }

    void wait_matches() {
        for (Slot& w : slots)
            if (w.used) HIPCHK(hipEventSynchronize(w.done));
    }

    void maybe_relayout() {
        if (force_relayout || layout_mode == 2 ||
            (layout_mode == 1 && live_nodes >= 4096 && created_since_layout * 4 >= live_nodes))
            relayout();
    }

    void commit() {
        if (dev_dirty || !d_nodes.p) maybe_relayout();
        if (device < 0) {
            ++epoch;
            dev_dirty = false;
            return;
        }
        if (!dev_dirty && d_nodes.p) {
            if (split_halves && split_stale) {
                Guard g(device);
                wait_matches();
                split_image();
                HIPCHK(hipStreamSynchronize(stream));
            }
            return;
        }
        Guard g(device);
        wait_matches();  // never patch the image under a running walk
        rw_drain();
        upload_table(d_nodes, nodes, node_dirty, 0);
        upload_table(d_edges, cold.slots, cold.dirty, 0);
        upload_table(d_hedges, hot.slots, hot.dirty, 0);
        upload_table(d_dict, dict, dict_dirty, 0);
        // append-only arrays: upload the new tail (or all after a realloc)
        {
            bool re = d_arena.ensure(std::max<size_t>(word_arena.size(), 8) + 16);
            size_t from = re ? 0 : arena_uploaded;
            if (word_arena.size() > from)
                HIPCHK(hipMemcpyAsync(d_arena.as<uint8_t>() + from, word_arena.data() + from,
                                      word_arena.size() - from, hipMemcpyHostToDevice, stream));
            arena_uploaded = word_arena.size();
        }
        {
            bool re = d_woff.ensure(std::max<size_t>(word_off.size(), 1) * 4);
            size_t from = re ? 0 : woff_uploaded;
            if (word_off.size() > from)
                HIPCHK(hipMemcpyAsync(d_woff.as<uint32_t>() + from, word_off.data() + from,
                                      (word_off.size() - from) * 4, hipMemcpyHostToDevice, stream));
            woff_uploaded = word_off.size();
        }
        split_stale = true;
        if (split_halves) split_image();
        HIPCHK(hipStreamSynchronize(stream));
        dev_dirty = false;
        ++epoch;
    }

    // option "split": de-interleave the uploaded records into inner / leaf arrays
    void split_image() {
        d_inner.ensure(nodes.size() * 16);
        d_leaf.ensure(nodes.size() * 16);
        HIPCHK(launch_split_nodes(d_nodes.p, nodes.size(), d_inner.p, d_leaf.p, stream));
        split_stale = false;
    }

    // ------------------------------------------------------------------
    // the match pipeline on device buffers (all stream-ordered on st)
    KTimes take_event(const char* name) {
        KTimes k{name, nullptr, nullptr};
        if (!ev_pool.empty()) {
            k = ev_pool.back();
            ev_pool.pop_back();
            k.name = name;
        } else {
            HIPCHK(hipEventCreate(&k.a));
            HIPCHK(hipEventCreate(&k.b));
        }
        return k;
    }
    void ensure_workspace(uint32_t n, uint64_t nbytes) { w_total.ensure(64); }
    void ensure_slot(Slot& w, uint32_t n, uint64_t nbytes, uint32_t key_words) {
        w.twords.ensure((size_t)(n + 1) * WREG * 4);
        w.words.ensure((nbytes + n + 1) * 4);
        w.path.ensure((nbytes + 2ull * n + 2) * 4);
        w.stats.ensure(STATS_BYTES);
        w.meta.ensure((size_t)(n + 1) * 4);
        w.scan.ensure(scan_tmp_elems(n) * 8 + 8);
        w.stage.ensure(((size_t)n * stage_k + 4) * 4);
        if (key_words) w.kstage.ensure(((size_t)n * stage_k * key_words + 4) * 8);
        w.ws.ensure(QWS_BYTES);
        if (group) w.perm.ensure(((size_t)n + GROUP_WS_ELEMS) * 4);
        if (!w.done) HIPCHK(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    }

    // the whole hot path of one batch, stream-ordered on st: CSR of ordered
    // filter ids (ids past cap are dropped; *total always exact)
    // stage rows sized to the largest list of the previous walk (read back
    // asynchronously), within STAGE_BUDGET: fan-out beyond K costs a re-walk
    void adapt_stage_k(uint32_t n, uint32_t key_words) {
        if (!stage_auto) return;
        uint64_t mc = 0;
        for (Slot& w : slots) {
            if (!w.maxc_pending || hipEventQuery(w.maxc_ev) != hipSuccess) continue;
            w.maxc_pending = false;
            mc = std::max<uint64_t>(mc, *w.h_maxc);
        }
        if (!mc) return;
        uint64_t want = stage_k_min;
        while (want < mc && want < 4096) want <<= 1;
        uint64_t k = stage_k;
        const uint64_t per = (uint64_t)n * (4 + 8 * key_words);
        while (k < want && per * (k << 1) <= STAGE_BUDGET) k <<= 1;
        stage_k = (uint32_t)k;
    }
    void record_maxc(Slot& w, hipStream_t st) {
        if (!stage_auto) return;
        if (!w.h_maxc) HIPCHK(hipHostMalloc((void**)&w.h_maxc, 64, hipHostMallocDefault));
        if (!w.maxc_ev) HIPCHK(hipEventCreateWithFlags(&w.maxc_ev, hipEventDisableTiming));
        HIPCHK(hipMemcpyAsync(w.h_maxc, w.ws.as<uint64_t>() + QWS_MAXC, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(w.maxc_ev, st));
        w.maxc_pending = true;
    }

    void run_batch(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes, uint32_t* counts,
                   uint64_t* out_off, uint32_t* ids, uint64_t cap, uint64_t* total, hipStream_t st,
                   uint64_t* keys = nullptr, uint32_t key_words = 1) {
        const uint32_t kw = keys ? key_words : 0u;
        adapt_stage_k(n, kw);
        ensure_workspace(n, nbytes);
        const int si = next_slot;
        next_slot = (next_slot + 1) % nslots;
        Slot& w = slots[si];
        if (w.used) HIPCHK(hipStreamWaitEvent(st, w.done, 0));   // its previous batch, maybe on another stream
        ensure_slot(w, n, nbytes, kw);
        last_slot = si;
        ImageView im = view();
        unsigned long long* sp = w.stats.as<unsigned long long>();
        if (stats_enabled) HIPCHK(hipMemsetAsync(w.stats.p, 0, STATS_BYTES, st));
        static const char* kStage[4] = {"tokenize", "walk", "scan", "copy_out"};
        hipEvent_t marks[8];
        if (timing_enabled)
            for (int i = 0; i < 4; ++i) {
                ev_cur[i] = take_event(kStage[i]);
                marks[2 * i] = ev_cur[i].a;
                marks[2 * i + 1] = ev_cur[i].b;
            }
        QueueBufs qb;
        qb.twords = w.twords.as<uint32_t>();
        qb.words = w.words.as<uint32_t>();
        qb.meta = w.meta.as<uint32_t>();
        qb.path = w.path.as<uint32_t>();
        qb.stage = w.stage.as<uint32_t>();
        qb.kstage = keys ? w.kstage.as<uint64_t>() : nullptr;
        qb.scan_tmp = w.scan.as<uint64_t>();
        qb.ws = w.ws.as<unsigned long long>();
        qb.perm = group ? w.perm.as<uint32_t>() : nullptr;
        HIPCHK(launch_queue(stats_enabled, xcdq != 0, im, bytes, off, n, qb, stage_k, counts, out_off, ids, keys, cap,
                            total, sp, st, timing_enabled ? marks : nullptr, walk_bpc, hist_enabled != 0,
                            keys ? key_words : 1u));
        w.keyed = keys != nullptr;
        record_maxc(w, st);
        HIPCHK(hipEventRecord(w.done, st));
        w.used = true;
        if (timing_enabled)
            for (int i = 0; i < 4; ++i) ev_pending.push_back(ev_cur[i]);
    }
    // emqx_router:match_routes/1 over a device batch (stream-ordered except
    // for one read of the match total that sizes the ids workspace)
    void ensure_route_image() {
        if (routes_dirty) {
            if (route_bag.empty()) {
                route_image = false;
                routes_dirty = false;
                agg_keys.clear();
                aggre_dirty = true;
            } else {
                build_route_image();
            }
        }
    }
    void run_routes(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes, uint32_t* counts,
                    uint64_t* out_off, uint32_t* src, uint32_t* dest, uint64_t cap, uint64_t* total,
                    hipStream_t st, uint64_t* out_key = nullptr) {
        ensure_route_image();
        // this path reads the match total back anyway (host sync per batch):
        // wait for the previous route / aggre batch of any stream, so its
        // workspaces can be reused or reallocated
        rw_drain();
        w_rcounts.ensure((size_t)n * 4 + 4);
        w_roff.ensure((size_t)(n + 1) * 8);
        uint64_t want = std::max<uint64_t>(w_rids.bytes / 4, (uint64_t)n * 16 + 1024);
        w_rids.ensure(want * 4, 1.0);
        uint64_t icap = w_rids.bytes / 4, ids_total = 0;
        for (int pass = 0; pass < 2; ++pass) {
            run_batch(bytes, off, n, nbytes, w_rcounts.as<uint32_t>(), w_roff.as<uint64_t>(), w_rids.as<uint32_t>(),
                      icap, total, st);
            HIPCHK(hipMemcpyAsync(&ids_total, total, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (ids_total <= icap) break;
            w_rids.ensure(ids_total * 4, 1.25);
            icap = w_rids.bytes / 4;
        }
        w_rexact.ensure((size_t)n * 8 + 8);
        w_rscan.ensure(scan_tmp_elems(n) * 8 + 8);
        const AggreView av_tmp = aggre_view();
        HIPCHK(launch_routes(route_view(), bytes, off, n, w_rcounts.as<uint32_t>(), w_roff.as<uint64_t>(),
                             w_rids.as<uint32_t>(), w_rexact.as<uint2>(), counts, out_off, src, dest, cap, total,
                             w_rscan.as<uint64_t>(), st, out_key ? &av_tmp : nullptr, out_key));
        rw_release(st);
    }

    // aggre(match_routes(T)) over a device batch: the route lists and their
    // sort keys go to engine workspace (one read of the route total sizes
    // it), aggre.hip writes each topic's list at its route offset; *total =
    // route total
    void run_deliveries(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes, uint32_t* counts,
                        uint64_t* out_off, uint32_t* to, uint32_t* target, uint64_t cap, uint64_t* total,
                        hipStream_t st) {
        ensure_route_image();
        if (aggre_dirty) build_aggre_image();
        rw_drain();   // w_d* / w_a* may be reallocated below
        w_dcount.ensure((size_t)n * 4 + 4);
        uint64_t want = std::max<uint64_t>(w_dsrc.bytes / 8, (uint64_t)n * 16 + 1024);
        w_dsrc.ensure(want * 8, 1.0);
        w_akey.ensure(want * 8, 1.0);
        uint64_t rcap = std::min(w_dsrc.bytes / 8, w_akey.bytes / 8), rtotal = 0;
        for (int pass = 0; pass < 2; ++pass) {
            uint32_t* src = w_dsrc.as<uint32_t>();
            run_routes(bytes, off, n, nbytes, w_dcount.as<uint32_t>(), out_off, src, src + rcap, rcap, total, st,
                       w_akey.as<uint64_t>());
            HIPCHK(hipMemcpyAsync(&rtotal, total, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (rtotal <= rcap) break;
            w_dsrc.ensure(rtotal * 8, 1.25);
            w_akey.ensure(rtotal * 8, 1.25);
            rcap = std::min(w_dsrc.bytes / 8, w_akey.bytes / 8);
        }
        w_alarge.ensure((size_t)n * 4 + 16);
        const uint32_t* src = w_dsrc.as<uint32_t>();
        HIPCHK(launch_aggre(aggre_view(), n, w_dcount.as<uint32_t>(), out_off, src, src + rcap, w_akey.as<uint64_t>(),
                            w_alarge.as<uint32_t>(), counts, to, target, cap, st));
        rw_release(st);
    }

    void finish_batch(hipStream_t st, uint32_t n) {
        (void)st;
        last_stats = tm_batch_stats{};
        last_stats.topics = n;
    }
    void collect_stats() {
        const DevBuf& ws = slots[last_slot].stats;
        if (!stats_enabled || !ws.p) return;
        unsigned long long h[6] = {0, 0, 0, 0, 0, 0};
        HIPCHK(hipMemcpy(h, ws.p, sizeof(h), hipMemcpyDeviceToHost));
        last_stats.levels = h[0];
        last_stats.visits = h[1];
        last_stats.edge_reads = h[2];
        last_stats.matches = h[3];
        last_stats.leaf_visits = h[4];
        last_stats.probe_loads = h[5];
    }
};

// ---------------------------------------------------------------------------
namespace {

template <class F>
int guarded(tm_engine* e, F&& f) {
    if (!e) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    try {
        return f();
    } catch (const ArgError& x) {
        e->last_error = x.what();
        return TM_EINVAL;
    } catch (const RangeError& x) {
        e->last_error = x.what();
        return TM_ERANGE;
    } catch (const DevError& x) {
        e->last_error = x.what();
        return TM_EDEVICE;
    } catch (const std::bad_alloc&) {
        e->last_error = "out of host memory";
        return TM_ENOMEM;
    } catch (const std::exception& x) {
        e->last_error = x.what();
        return TM_EDEVICE;
    } catch (...) {
        e->last_error = "unknown failure";
        return TM_EDEVICE;
    }
}

// emqx_topic:words/1 over a byte string, into (start, len) pairs
inline void split_levels(const uint8_t* p, uint32_t len, std::vector<std::pair<uint32_t, uint32_t>>& out) {
    out.clear();
    uint32_t s = 0;
    for (uint32_t i = 0; i <= len; ++i)
        if (i == len || p[i] == '/') {
            out.emplace_back(s, i - s);
            s = i + 1;
        }
}

}  // namespace

extern "C" {

const char* tm_build_info(void) { return "libtopicmatch gfx950 (CDNA4) HIP; image v4 (inner/leaf 16 B halves, Bloom-masked edge16, dict with 16 B word prefixes), routes + aggre"; }

const char* tm_strerror(int code) {
    switch (code) {
        case TM_OK: return "ok";
        case TM_EINVAL: return "invalid argument";
        case TM_ENOSPC: return "output buffer too small";
        case TM_EDEVICE: return "device unavailable or HIP error";
        case TM_ENOMEM: return "out of memory";
        case TM_ENOENT: return "no such trie node";
        case TM_ERANGE: return "capacity exceeded";
        default: return "unknown status";
    }
}

const char* tm_last_error(tm_engine* e) { return e ? e->last_error.c_str() : "null engine"; }

int tm_open(const tm_config* cfg, tm_engine** out) {
    if (!out) return TM_EINVAL;
    *out = nullptr;
    tm_engine* e = nullptr;
    try {
        e = new tm_engine();
    } catch (...) {
        return TM_ENOMEM;
    }
    int dev = cfg ? cfg->device : -1;
    if (cfg && cfg->filters_hint) {
        size_t nodes_hint = (size_t)cfg->filters_hint * 3;
        e->nodes.reserve(nodes_hint);
        e->aux.reserve(nodes_hint);
        // wide nodes' literal edges and '#' edges use the table (load <= 1/4)
        e->cold.slots.assign(next_pow2(nodes_hint), kEmptySlot);
    }
    if (dev >= 0) {
        int ndev = 0;
        hipError_t err = hipGetDeviceCount(&ndev);
        if (err != hipSuccess || dev >= ndev) {
            delete e;
            return TM_EDEVICE;
        }
        int prev = -1;
        (void)hipGetDevice(&prev);
        if (hipSetDevice(dev) != hipSuccess ||
            hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
            delete e;
            return TM_EDEVICE;
        }
        if (prev >= 0) (void)hipSetDevice(prev);
        e->device = dev;
    }
    *out = e;
    return TM_OK;
}

void tm_close(tm_engine* e) {
    if (!e) return;
    if (e->device >= 0) {
        (void)hipSetDevice(e->device);
        if (e->stream) (void)hipStreamSynchronize(e->stream);
        if (e->rw_done) (void)hipEventDestroy(e->rw_done);
        for (DevBuf* b : {&e->d_ex_rank, &e->d_dt, &e->d_rank_src, &e->d_rank_tg, &e->w_dsrc, &e->w_dcount, &e->w_akey,
                          &e->w_alarge,
             &e->d_fr_meta, &e->d_fr_dest, &e->d_ex_slots, &e->d_ex_arena, &e->d_ex_dest, &e->w_rexact,
                          &e->w_rscan, &e->w_rids, &e->w_rcounts, &e->w_roff})
            b->release();
        for (DevBuf* b : {&e->d_nodes, &e->d_edges, &e->d_hedges, &e->d_dict, &e->d_arena, &e->d_woff, &e->d_inner, &e->d_leaf,
                          &e->w_mpre, &e->w_mscan, &e->w_bytes, &e->w_off, &e->w_counts, &e->w_outoff, &e->w_ids,
                          &e->w_total})
            b->release();
        for (auto& w : e->slots) {
            for (DevBuf* b : {&w.twords, &w.words, &w.path, &w.meta, &w.scan, &w.stage, &w.kstage, &w.ws, &w.stats})
                b->release();
            if (w.done) (void)hipEventDestroy(w.done);
            if (w.maxc_ev) (void)hipEventDestroy(w.maxc_ev);
            if (w.h_maxc) (void)hipHostFree(w.h_maxc);
        }
        for (auto* v : {&e->ev_pool, &e->ev_pending})
            for (auto& k : *v) {
                (void)hipEventDestroy(k.a);
                (void)hipEventDestroy(k.b);
            }
        if (e->stream) (void)hipStreamDestroy(e->stream);
    }
    delete e;
}

int tm_insert(tm_engine* e, const uint8_t* filter, uint32_t len) {
    if (!filter && len) return TM_EINVAL;
    return guarded(e, [&] {
        e->insert(filter, len);
        return TM_OK;
    });
}

int tm_insert_batch(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
    if (n && (!bytes || !off)) return TM_EINVAL;
    return guarded(e, [&] {
        for (uint32_t i = 0; i < n; ++i) {
            if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
            e->insert(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        }
        return TM_OK;
    });
}

uint32_t tm_shard_of(const uint8_t* filter, uint32_t len, uint32_t n_shards) {
    if (n_shards <= 1 || (!filter && len)) return 0;
    // The prefix through the filter's second LITERAL level decides, so every
    // filter under one such prefix lives on one shard.  Root words alone are
    // too coarse (with Zipf root words the heaviest holds ~25 % of the
    // filters), and a fixed two-level prefix puts the whole "+/+/..." subtree,
    // which every topic walks and matches, on one shard; counting only
    // literal levels spreads wildcard-led subtrees by their next literal word
    // (C4 sample: max/mean matches per shard 3.6 -> 1.6).
    uint32_t cut = len, lits = 0, start = 0;
    for (uint32_t i = 0; i <= len; ++i) {
        if (i == len || filter[i] == '/') {
            const bool wild = i - start == 1 && (filter[start] == '+' || filter[start] == '#');
            if (!wild && ++lits == 2) {
                cut = i;
                break;
            }
            start = i + 1;
        }
    }
    uint64_t h = 0xcbf29ce484222325ULL;   // FNV-1a 64
    for (uint32_t i = 0; i < cut; ++i) h = (h ^ filter[i]) * 0x100000001b3ULL;
    return (uint32_t)(fmix64(h) % n_shards);
}

int tm_shard_of_batch(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t n_shards, uint32_t* out) {
    if ((n && (!bytes || !off || !out)) || n_shards == 0) return TM_EINVAL;
    for (uint32_t i = 0; i < n; ++i) {
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) return TM_EINVAL;
        out[i] = tm_shard_of(bytes + off[i], (uint32_t)(off[i + 1] - off[i]), n_shards);
    }
    return TM_OK;
}

int tm_insert_batch_shard(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t n_shards,
                          uint32_t shard) {
    if ((n && (!bytes || !off)) || n_shards == 0 || shard >= n_shards) return TM_EINVAL;
    return guarded(e, [&] {
        for (uint32_t i = 0; i < n; ++i) {
            if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
            const uint32_t len = (uint32_t)(off[i + 1] - off[i]);
            if (tm_shard_of(bytes + off[i], len, n_shards) == shard) e->insert(bytes + off[i], len);
        }
        return TM_OK;
    });
}

int tm_delete_batch(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
    if (n && (!bytes || !off)) return TM_EINVAL;
    return guarded(e, [&] {
        for (uint32_t i = 0; i < n; ++i) {
            if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
            e->remove(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        }
        return TM_OK;
    });
}

int tm_delete(tm_engine* e, const uint8_t* filter, uint32_t len) {
    if (!filter && len) return TM_EINVAL;
    return guarded(e, [&] {
        e->remove(filter, len);
        return TM_OK;
    });
}

int tm_lookup(tm_engine* e, const uint8_t* node_id, uint32_t len, tm_node_info* out) {
    if ((!node_id && len) || !out) return TM_EINVAL;
    return guarded(e, [&] {
        if (!e->split_words(node_id, len, false)) return TM_ENOENT;
        uint32_t v = e->walk(e->tmp_words);
        if (v == NODE_NONE) return TM_ENOENT;
        out->edge_count = e->aux[v].edge_count;
        out->filter_id = e->nodes[v].self_filter;
        return TM_OK;
    });
}

int tm_commit(tm_engine* e, uint64_t* epoch_out) {
    return guarded(e, [&] {
        e->commit();
        if (epoch_out) *epoch_out = e->epoch;
        return TM_OK;
    });
}

uint64_t tm_filter_count(tm_engine* e) { return e ? e->live_filters : 0; }
uint64_t tm_node_count(tm_engine* e) { return e ? e->live_nodes : 0; }
int tm_engine_device(tm_engine* e) { return e ? e->device : -1; }

uint64_t tm_image_bytes(tm_engine* e) {
    if (!e) return 0;
    return e->nodes.size() * sizeof(Node) + (e->cold.slots.size() + e->hot.slots.size()) * sizeof(EdgeSlot) +
           e->dict.size() * sizeof(DictSlot) +
           e->word_arena.size() + e->word_off.size() * 4;
}

const uint8_t* tm_filter_bytes(tm_engine* e, uint32_t fid, uint32_t* len) {
    if (!e) return nullptr;
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    if (fid >= e->filters.size() || e->filters[fid].node == NODE_NONE) {
        if (len) *len = 0;
        return nullptr;
    }
    if (len) *len = e->filters[fid].len;
    return e->filter_arena.data() + e->filters[fid].off;
}

// bytes of many filters (or dests) copied under the engine lock: safe
// against a concurrent insert that grows the arena / dest table
int tm_filters_gather(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, uint64_t cap, uint64_t* off) {
    if (!off || (n && !ids) || (cap && !buf)) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        uint64_t o = 0;
        off[0] = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t f = ids[i];
            if (f >= e->filters.size() || e->filters[f].node == NODE_NONE) throw ArgError("unknown filter id");
            const FilterRec& r = e->filters[f];
            if (o + r.len <= cap) std::memcpy(buf + o, e->filter_arena.data() + r.off, r.len);
            o += r.len;
            off[i + 1] = o;
        }
        return o > cap ? TM_ENOSPC : TM_OK;
    });
}

int tm_dests_gather(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, uint64_t cap, uint64_t* off) {
    if (!off || (n && !ids) || (cap && !buf)) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        uint64_t o = 0;
        off[0] = 0;
        for (uint32_t i = 0; i < n; ++i) {
            if (ids[i] >= e->dest_names.size()) throw ArgError("unknown dest id");
            const std::string& d = e->dest_names[ids[i]];
            if (o + d.size() <= cap) std::memcpy(buf + o, d.data(), d.size());
            o += d.size();
            off[i + 1] = o;
        }
        return o > cap ? TM_ENOSPC : TM_OK;
    });
}

int tm_match_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                   uint32_t* out_count, uint64_t* out_off, uint32_t* out_ids, uint64_t out_cap,
                   uint64_t* out_needed) {
    if (!topic_off || !out_off || (n && (!out_count)) || (out_cap && !out_ids)) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): the match path runs on the GPU only";
            return TM_EDEVICE;
        }
        for (uint32_t i = 0; i < n; ++i)
            if (topic_off[i + 1] < topic_off[i]) throw ArgError("topic offsets not monotone");
        uint64_t base = topic_off[0], nbytes = topic_off[n] - base;
        if (n && nbytes && !topic_bytes) throw ArgError("null topic bytes");
        if (n == 0) {
            out_off[0] = 0;
            if (out_needed) *out_needed = 0;
            return TM_OK;
        }
        e->commit();
        tm_engine::Guard g(e->device);
        hipStream_t st = e->stream;
        e->w_bytes.ensure(nbytes + 16);
        e->w_off.ensure((size_t)(n + 1) * 8);
        e->w_counts.ensure((size_t)n * 4 + 4);
        e->w_outoff.ensure((size_t)(n + 1) * 8);
        std::vector<uint64_t> rel(topic_off, topic_off + n + 1);
        for (auto& x : rel) x -= base;
        if (nbytes)
            HIPCHK(hipMemcpyAsync(e->w_bytes.p, topic_bytes + base, nbytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->w_off.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        e->ensure_workspace(n, nbytes);
        uint64_t* d_total = e->w_total.as<uint64_t>();
        // ids go to an engine buffer sized from the previous batch; grow and
        // rerun only when a batch needs more (the total is always exact)
        uint64_t want = std::max<uint64_t>(e->w_ids.bytes / 4, std::min<uint64_t>(out_cap, (uint64_t)n * 16 + 1024));
        e->w_ids.ensure(want * 4, 1.0);
        uint64_t icap = e->w_ids.bytes / 4;
        uint64_t total = 0;
        for (int pass = 0; pass < 2; ++pass) {
            e->run_batch(e->w_bytes.as<uint8_t>(), e->w_off.as<uint64_t>(), n, nbytes, e->w_counts.as<uint32_t>(),
                         e->w_outoff.as<uint64_t>(), e->w_ids.as<uint32_t>(), icap, d_total, st);
            HIPCHK(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (total <= icap || total > out_cap) break;
            e->w_ids.ensure(total * 4, 1.25);
            icap = e->w_ids.bytes / 4;
        }
        // the workspace holds min(total, icap) ids; with total > out_cap the
        // call reports TM_ENOSPC and copies what fits both
        uint64_t cap = std::min(std::min(total, out_cap), icap);
        e->finish_batch(st, n);
        HIPCHK(hipMemcpyAsync(out_count, e->w_counts.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(out_off, e->w_outoff.p, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, st));
        if (cap) HIPCHK(hipMemcpyAsync(out_ids, e->w_ids.p, cap * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        e->collect_stats();
        if (out_needed) *out_needed = total;
        return total > out_cap ? TM_ENOSPC : TM_OK;
    });
}

static int match_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                        uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                        uint64_t* d_keys, uint32_t key_words, uint64_t out_cap, uint64_t* d_total, void* hip_stream);

// ---- routes (emqx_router) ---------------------------------------------------
int tm_route_add(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen) {
    if ((!topic && tlen) || (!dest && dlen)) return TM_EINVAL;
    return guarded(e, [&] {
        e->route_add(topic, tlen, dest, dlen);
        return TM_OK;
    });
}

int tm_route_add_batch(tm_engine* e, const uint8_t* topics, const uint64_t* topic_off, const uint8_t* dests,
                       const uint64_t* dest_off, uint32_t n) {
    if (n && (!topics || !topic_off || !dests || !dest_off)) return TM_EINVAL;
    return guarded(e, [&] {
        for (uint32_t i = 0; i < n; ++i) {
            if (topic_off[i + 1] < topic_off[i] || topic_off[i + 1] - topic_off[i] > 0xFFFFFFFFull ||
                dest_off[i + 1] < dest_off[i] || dest_off[i + 1] - dest_off[i] > 0xFFFFFFFFull)
                throw ArgError("bad offsets");
            e->route_add(topics + topic_off[i], (uint32_t)(topic_off[i + 1] - topic_off[i]), dests + dest_off[i],
                         (uint32_t)(dest_off[i + 1] - dest_off[i]));
        }
        return TM_OK;
    });
}

int tm_route_del(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen) {
    if ((!topic && tlen) || (!dest && dlen)) return TM_EINVAL;
    return guarded(e, [&] {
        e->route_del(topic, tlen, dest, dlen);
        return TM_OK;
    });
}

int tm_get_routes(tm_engine* e, const uint8_t* topic, uint32_t tlen, uint32_t* out_dest, uint32_t cap,
                  uint32_t* out_n) {
    if ((!topic && tlen) || !out_n || (cap && !out_dest)) return TM_EINVAL;
    return guarded(e, [&] {
        const std::vector<uint32_t>* b = e->get_routes(topic, tlen);
        const uint32_t k = b ? (uint32_t)b->size() : 0u;
        *out_n = k;
        for (uint32_t i = 0; i < k && i < cap; ++i) out_dest[i] = (*b)[i];
        return k > cap ? TM_ENOSPC : TM_OK;
    });
}

uint64_t tm_route_count(tm_engine* e) {
    if (!e) return 0;
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    return e->route_total;
}

const uint8_t* tm_dest_bytes(tm_engine* e, uint32_t dest_id, uint32_t* len) {
    if (!e) return nullptr;
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    if (dest_id >= e->dest_names.size()) return nullptr;
    if (len) *len = (uint32_t)e->dest_names[dest_id].size();
    return reinterpret_cast<const uint8_t*>(e->dest_names[dest_id].data());
}

int tm_match_routes_batch_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                                 uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_src,
                                 uint32_t* d_dest, uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (!d_off || !d_out_off || !d_total || (n && !d_count) || (out_cap && (!d_src || !d_dest))) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): match_routes runs on the GPU only";
            return TM_EDEVICE;
        }
        e->commit();
        tm_engine::Guard g(e->device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : e->stream;
        if (n == 0) {
            HIPCHK(hipMemsetAsync(d_out_off, 0, 8, st));
            HIPCHK(hipMemsetAsync(d_total, 0, 8, st));
            return TM_OK;
        }
        e->run_routes(d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_src, d_dest, out_cap, d_total, st);
        e->finish_batch(st, n);
        return TM_OK;
    });
}

int tm_match_routes_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                          uint32_t* out_count, uint64_t* out_off, uint32_t* out_src, uint32_t* out_dest,
                          uint64_t out_cap, uint64_t* out_needed) {
    if (!topic_off || !out_off || (n && !out_count) || (out_cap && (!out_src || !out_dest))) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): match_routes runs on the GPU only";
            return TM_EDEVICE;
        }
        for (uint32_t i = 0; i < n; ++i)
            if (topic_off[i + 1] < topic_off[i]) throw ArgError("topic offsets not monotone");
        const uint64_t base = topic_off[0], nbytes = topic_off[n] - base;
        if (n && nbytes && !topic_bytes) throw ArgError("null topic bytes");
        if (n == 0) {
            out_off[0] = 0;
            if (out_needed) *out_needed = 0;
            return TM_OK;
        }
        e->commit();
        tm_engine::Guard g(e->device);
        hipStream_t st = e->stream;
        e->w_bytes.ensure(nbytes + 16);
        e->w_off.ensure((size_t)(n + 1) * 8);
        e->w_counts.ensure((size_t)n * 4 + 4);
        e->w_outoff.ensure((size_t)(n + 1) * 8);
        std::vector<uint64_t> rel(topic_off, topic_off + n + 1);
        for (auto& x : rel) x -= base;
        if (nbytes) HIPCHK(hipMemcpyAsync(e->w_bytes.p, topic_bytes + base, nbytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->w_off.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        e->ensure_workspace(n, nbytes);
        uint64_t* d_total = e->w_total.as<uint64_t>() + 1;
        // routes into engine buffers sized from the previous batch; grow and
        // rerun only when a batch needs more
        uint64_t want = std::max<uint64_t>(e->w_ids.bytes / 8, std::min<uint64_t>(out_cap, (uint64_t)n * 16 + 1024));
        e->w_ids.ensure(want * 8, 1.0);
        uint64_t rcap = e->w_ids.bytes / 8, total = 0;
        for (int pass = 0; pass < 2; ++pass) {
            uint32_t* src = e->w_ids.as<uint32_t>();
            e->run_routes(e->w_bytes.as<uint8_t>(), e->w_off.as<uint64_t>(), n, nbytes, e->w_counts.as<uint32_t>(),
                          e->w_outoff.as<uint64_t>(), src, src + rcap, rcap, d_total, st);
            HIPCHK(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (total <= rcap || total > out_cap) break;
            e->w_ids.ensure(total * 8, 1.25);
            rcap = e->w_ids.bytes / 8;
        }
        const uint64_t cap = std::min(std::min(total, out_cap), rcap);   // see tm_match_batch
        e->finish_batch(st, n);
        HIPCHK(hipMemcpyAsync(out_count, e->w_counts.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(out_off, e->w_outoff.p, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, st));
        if (cap) {
            HIPCHK(hipMemcpyAsync(out_src, e->w_ids.p, cap * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(out_dest, e->w_ids.as<uint32_t>() + rcap, cap * 4, hipMemcpyDeviceToHost, st));
        }
        HIPCHK(hipStreamSynchronize(st));
        if (out_needed) *out_needed = total;
        return total > out_cap ? TM_ENOSPC : TM_OK;
    });
}

int tm_dest_target(tm_engine* e, const uint8_t* dest, uint32_t dlen, uint32_t kind, const uint8_t* key,
                   uint32_t klen, uint32_t* target_out) {
    if ((dlen && !dest) || (klen && !key) || kind > TM_TARGET_GROUP) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        const uint32_t d = e->intern_dest(dest, dlen);
        if (e->dest_target.size() <= d) e->dest_target.resize(d + 1, tm_engine::TARGET_DEFAULT);
        const uint32_t t = e->intern_target(kind, key, klen);
        if (e->dest_target[d] != t) {
            e->dest_target[d] = t;
            e->aggre_dirty = true;
        }
        if (target_out) *target_out = t;
        return TM_OK;
    });
}

const uint8_t* tm_target_bytes(tm_engine* e, uint32_t target_id, uint32_t* kind, uint32_t* len) {
    if (!e) return nullptr;
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    if (target_id >= e->target_names.size()) return nullptr;
    const std::string& t = e->target_names[target_id];
    if (kind) *kind = (uint8_t)t[0];
    if (len) *len = (uint32_t)t.size() - 1;
    return reinterpret_cast<const uint8_t*>(t.data()) + 1;
}

int tm_match_deliveries_batch_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                                     uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_to,
                                     uint32_t* d_target, uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (!d_off || !d_out_off || !d_total || (n && !d_count) || (out_cap && (!d_to || !d_target))) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): aggre runs on the GPU only";
            return TM_EDEVICE;
        }
        e->commit();
        tm_engine::Guard g(e->device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : e->stream;
        if (n == 0) {
            HIPCHK(hipMemsetAsync(d_out_off, 0, 8, st));
            HIPCHK(hipMemsetAsync(d_total, 0, 8, st));
            return TM_OK;
        }
        e->run_deliveries(d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_to, d_target, out_cap, d_total, st);
        e->finish_batch(st, n);
        return TM_OK;
    });
}

int tm_match_deliveries_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                              uint32_t* out_count, uint64_t* out_off, uint32_t* out_to, uint32_t* out_target,
                              uint64_t out_cap, uint64_t* out_needed) {
    if (!topic_off || !out_off || (n && !out_count) || (out_cap && (!out_to || !out_target))) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): aggre runs on the GPU only";
            return TM_EDEVICE;
        }
        for (uint32_t i = 0; i < n; ++i)
            if (topic_off[i + 1] < topic_off[i]) throw ArgError("topic offsets not monotone");
        const uint64_t base = topic_off[0], nbytes = topic_off[n] - base;
        if (n && nbytes && !topic_bytes) throw ArgError("null topic bytes");
        if (n == 0) {
            out_off[0] = 0;
            if (out_needed) *out_needed = 0;
            return TM_OK;
        }
        e->commit();
        tm_engine::Guard g(e->device);
        hipStream_t st = e->stream;
        e->w_bytes.ensure(nbytes + 16);
        e->w_off.ensure((size_t)(n + 1) * 8);
        e->w_counts.ensure((size_t)n * 4 + 4);
        e->w_outoff.ensure((size_t)(n + 1) * 8);
        std::vector<uint64_t> rel(topic_off, topic_off + n + 1);
        for (auto& x : rel) x -= base;
        if (nbytes) HIPCHK(hipMemcpyAsync(e->w_bytes.p, topic_bytes + base, nbytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->w_off.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
        e->ensure_workspace(n, nbytes);
        uint64_t* d_total = e->w_total.as<uint64_t>() + 1;
        // lists sit at their route offsets: the route total sizes the output
        uint64_t want = std::max<uint64_t>(e->w_ids.bytes / 8, std::min<uint64_t>(out_cap, (uint64_t)n * 16 + 1024));
        e->w_ids.ensure(want * 8, 1.0);
        uint64_t rcap = e->w_ids.bytes / 8, total = 0;
        for (int pass = 0; pass < 2; ++pass) {
            uint32_t* to = e->w_ids.as<uint32_t>();
            e->run_deliveries(e->w_bytes.as<uint8_t>(), e->w_off.as<uint64_t>(), n, nbytes,
                              e->w_counts.as<uint32_t>(), e->w_outoff.as<uint64_t>(), to, to + rcap, rcap, d_total,
                              st);
            HIPCHK(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (total <= rcap || total > out_cap) break;
            e->w_ids.ensure(total * 8, 1.25);
            rcap = e->w_ids.bytes / 8;
        }
        const uint64_t cap = std::min(std::min(total, out_cap), rcap);   // see tm_match_batch
        e->finish_batch(st, n);
        HIPCHK(hipMemcpyAsync(out_count, e->w_counts.p, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(out_off, e->w_outoff.p, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, st));
        if (cap) {
            HIPCHK(hipMemcpyAsync(out_to, e->w_ids.p, cap * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(out_target, e->w_ids.as<uint32_t>() + rcap, cap * 4, hipMemcpyDeviceToHost, st));
        }
        HIPCHK(hipStreamSynchronize(st));
        if (out_needed) *out_needed = total;
        return total > out_cap ? TM_ENOSPC : TM_OK;
    });
}

int tm_match_batch_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                          uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                          uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    return match_device(e, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_ids, nullptr, 1, out_cap, d_total,
                        hip_stream);
}

int tm_match_batch_device_keys(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                               uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                               uint64_t* d_keys, uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (out_cap && !d_keys) return TM_EINVAL;
    return match_device(e, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_ids, d_keys, 1, out_cap, d_total,
                        hip_stream);
}

int tm_match_batch_device_keys_w(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                                 uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                                 uint64_t* d_keys, uint32_t key_words, uint64_t out_cap, uint64_t* d_total,
                                 void* hip_stream) {
    if ((out_cap && !d_keys) || key_words == 0 || key_words > TM_MAX_KEY_WORDS) return TM_EINVAL;
    return match_device(e, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_ids, d_keys, key_words, out_cap,
                        d_total, hip_stream);
}

int tm_key_levels(tm_engine* e, uint32_t* max_levels) {
    if (!max_levels) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        *max_levels = 0;
        if (e->device < 0) return TM_OK;
        tm_engine::Guard g(e->device);
        for (auto& w : e->slots) {
            if (!w.used || !w.keyed) continue;
            HIPCHK(hipEventSynchronize(w.done));
            uint64_t x = 0;
            HIPCHK(hipMemcpy(&x, w.ws.as<uint64_t>() + QWS_MAXL, 8, hipMemcpyDeviceToHost));
            *max_levels = std::max<uint32_t>(*max_levels, (uint32_t)x);
        }
        return TM_OK;
    });
}

int tm_shard_merge(tm_engine* e, uint32_t n_shards, uint32_t m, const uint32_t* d_counts,
                   const uint64_t* d_src_base, const uint32_t* d_ids, const uint64_t* d_keys, uint32_t* d_out_count,
                   uint64_t* d_out_off, uint32_t* d_out_gid, uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    return tm_shard_merge_w(e, n_shards, m, d_counts, d_src_base, d_ids, d_keys, 1, 0, d_out_count, d_out_off,
                            d_out_gid, out_cap, d_total, hip_stream);
}

int tm_shard_merge_w(tm_engine* e, uint32_t n_shards, uint32_t m, const uint32_t* d_counts,
                     const uint64_t* d_src_base, const uint32_t* d_ids, const uint64_t* d_keys, uint32_t key_words,
                     uint64_t key_stride, uint32_t* d_out_count, uint64_t* d_out_off, uint32_t* d_out_gid,
                     uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (n_shards == 0 || n_shards > MAX_SHARDS || !d_out_off || !d_total) return TM_EINVAL;
    if (key_words == 0 || key_words > TM_MAX_KEY_WORDS) return TM_EINVAL;
    if (m && (!d_counts || !d_src_base || !d_out_count)) return TM_EINVAL;
    if (out_cap && (!d_ids || !d_keys || !d_out_gid)) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): the merge runs on the GPU only";
            return TM_EDEVICE;
        }
        tm_engine::Guard g(e->device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : e->stream;
        e->w_mpre.ensure(((size_t)n_shards * (m + 1) + 1) * 8);
        if ((uint64_t)n_shards * m > 0xFFFFFFFFull) throw ArgError("n_shards x m exceeds 2^32");
        e->w_mscan.ensure(scan_tmp_elems(std::max<uint32_t>(n_shards * m, m)) * 8 + 8);
        HIPCHK(launch_shard_merge(n_shards, m, d_counts, d_src_base, d_ids, d_keys, d_out_count, d_out_off, d_out_gid,
                                  out_cap, d_total, e->w_mpre.as<uint64_t>(), e->w_mscan.as<uint64_t>(), st,
                                  key_words, key_stride));
        return TM_OK;
    });
}

static int match_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                        uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                        uint64_t* d_keys, uint32_t key_words, uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (!d_off || !d_out_off || !d_total || (n && !d_count) || (out_cap && !d_ids)) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (e->device < 0) {
            e->last_error = "engine is host-only (device = -1): the match path runs on the GPU only";
            return TM_EDEVICE;
        }
        e->commit();
        tm_engine::Guard g(e->device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : e->stream;
        if (n == 0) {
            HIPCHK(hipMemsetAsync(d_out_off, 0, 8, st));
            HIPCHK(hipMemsetAsync(d_total, 0, 8, st));
            return TM_OK;
        }
        e->run_batch(d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_ids, out_cap, d_total, st, d_keys,
                     key_words);
        e->finish_batch(st, n);
        if (e->stats_enabled) {
            HIPCHK(hipStreamSynchronize(st));
                e->collect_stats();
        }
        return TM_OK;
    });
}

// diagnostics (not part of include/topicmatch.h): the last stats-mode
// batch's per-level histogram [visits, probe loads, failed probes] x 16
extern "C" int tm_debug_hist(tm_engine* e, uint64_t* out, int n) {
    if (!e || !out || n > 56) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        const DevBuf& ws = e->slots[e->last_slot].stats;
        if (!ws.p) return TM_EINVAL;
        HIPCHK(hipMemcpy(out, ws.as<uint64_t>() + 8, (size_t)n * 8, hipMemcpyDeviceToHost));
        return TM_OK;
    });
}

int tm_set_option(tm_engine* e, const char* name, int64_t value) {
    if (!name) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        if (!std::strcmp(name, "hist")) {
            e->hist_enabled = value != 0;
            return TM_OK;
        }
        if (!std::strcmp(name, "walk_bpc")) {
            if (value < 0 || value > 64) return TM_EINVAL;
            e->walk_bpc = (uint32_t)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "group")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->group = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "xcdq")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->xcdq = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "layout")) {
            if (value < 0 || value > 2) return TM_EINVAL;
            e->layout_mode = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "split")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->split_halves = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "hot_edges")) {
            if (value < 0 || value > 16) return TM_EINVAL;
            if ((uint32_t)value != e->hot_edge_depth) {
                e->hot_edge_depth = (uint32_t)value;
                e->force_relayout = true;
                e->dev_dirty = true;
            }
            return TM_OK;
        }
        if (!std::strcmp(name, "edge_load")) {
            if (value < 2 || value > 16) return TM_EINVAL;
            if ((uint32_t)value != e->edge_div) {
                e->edge_div = (uint32_t)value;
                e->force_relayout = true;
                e->dev_dirty = true;
            }
            return TM_OK;
        }
        if (!std::strcmp(name, "order")) {
            if (value < 0 || value > 15) return TM_EINVAL;
            if ((uint32_t)value != e->layout_order) {
                e->layout_order = (uint32_t)value;
                e->force_relayout = true;
                e->dev_dirty = true;
            }
            return TM_OK;
        }
        if (!std::strcmp(name, "hot_levels")) {
            if (value < 0 || value > 16) return TM_EINVAL;
            if ((uint32_t)value != e->hot_levels) {
                e->hot_levels = (uint32_t)value;
                e->force_relayout = true;
                e->dev_dirty = true;
            }
            return TM_OK;
        }
        if (!std::strcmp(name, "stage_k")) {
            if (value < 4 || value > 4096 || (value & 3)) return TM_EINVAL;
            e->stage_k = e->stage_k_min = (uint32_t)value;
            e->stage_auto = 0;   // an explicit K is kept (set "stage_auto" after it to grow from it)
            return TM_OK;
        }
        if (!std::strcmp(name, "slots")) {
            if (value < 1 || value > tm_engine::MAX_SLOTS) return TM_EINVAL;
            e->nslots = (int)value;
            e->next_slot = 0;
            return TM_OK;
        }
        if (!std::strcmp(name, "stage_auto")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->stage_auto = (int)value;
            return TM_OK;
        }
        return TM_EINVAL;
    });
}

int tm_set_stats(tm_engine* e, int enable) {
    return guarded(e, [&] {
        e->stats_enabled = enable != 0;
        return TM_OK;
    });
}

int tm_last_stats(tm_engine* e, tm_batch_stats* out) {
    if (!out) return TM_EINVAL;
    return guarded(e, [&] {
        *out = e->last_stats;
        return TM_OK;
    });
}

int tm_set_timing(tm_engine* e, int enable) {
    return guarded(e, [&] {
        e->timing_enabled = enable != 0;
        return TM_OK;
    });
}

int tm_last_kernel_times(tm_engine* e, const char** names, float* ms, int cap) {
    return guarded(e, [&]() -> int {
        if (e->ev_pending.empty()) return 0;
        tm_engine::Guard g(e->device);
        // average per batch of each kernel stage over every batch recorded
        // since the previous call
        std::vector<const char*> order;
        std::vector<double> sum;
        std::vector<int> cnt;
        for (auto& t : e->ev_pending) {
            HIPCHK(hipEventSynchronize(t.b));
            float v = 0.f;
            HIPCHK(hipEventElapsedTime(&v, t.a, t.b));
            size_t i = 0;
            while (i < order.size() && std::strcmp(order[i], t.name) != 0) ++i;
            if (i == order.size()) {
                order.push_back(t.name);
                sum.push_back(0.0);
                cnt.push_back(0);
            }
            sum[i] += v;
            cnt[i] += 1;
            e->ev_pool.push_back(t);
        }
        e->ev_pending.clear();
        int k = 0;
        for (size_t i = 0; i < order.size() && k < cap; ++i, ++k) {
            if (names) names[k] = order[i];
            if (ms) ms[k] = (float)(sum[i] / cnt[i]);
        }
        return k;
    });
}

// ---- pure topic algebra ----------------------------------------------------

// emqx_topic:match/2, binary/binary clause (src/emqx_topic.erl:56-61) then the
// word-list clauses (:62-75)
int tm_topic_match(const uint8_t* name, uint32_t nlen, const uint8_t* filt, uint32_t flen) {
    if ((!name && nlen) || (!filt && flen)) return 0;
    if (nlen > 0 && name[0] == '$' && flen > 0 && (filt[0] == '+' || filt[0] == '#')) return 0;
    std::vector<std::pair<uint32_t, uint32_t>> nw, fw;
    split_levels(name, nlen, nw);
    split_levels(filt, flen, fw);
    auto is = [](const uint8_t* p, std::pair<uint32_t, uint32_t> w, char c) {
        return w.second == 1 && p[w.first] == (uint8_t)c;
    };
    size_t i = 0, j = 0;
    for (;;) {
        if (i == nw.size() && j == fw.size()) return 1;          // match([], [])
        if (j < fw.size() && i < nw.size()) {
            auto a = nw[i], b = fw[j];
            // match([H|T1], [H|T2]) — equal words (atoms compare equal too)
            if (a.second == b.second && std::memcmp(name + a.first, filt + b.first, a.second) == 0) {
                ++i, ++j;
                continue;
            }
            if (is(filt, b, '+')) {                              // match([_|T1], ['+'|T2])
                ++i, ++j;
                continue;
            }
        }
        if (j + 1 == fw.size() && is(filt, fw[j], '#')) return 1;  // match(_, ['#'])
        return 0;
    }
}

int tm_topic_wildcard(const uint8_t* topic, uint32_t len) {
    if (!topic && len) return 0;
    std::vector<std::pair<uint32_t, uint32_t>> w;
    split_levels(topic, len, w);
    for (auto x : w)
        if (x.second == 1 && (topic[x.first] == '+' || topic[x.first] == '#')) return 1;
    return 0;
}

// emqx_topic:parse/1,2 (src/emqx_topic.erl:180-200)
int tm_topic_parse(const uint8_t* t, uint32_t len, const uint8_t** inner, uint32_t* inner_len,
                   const uint8_t** group, uint32_t* group_len) {
    if ((!t && len) || !inner || !inner_len || !group || !group_len) return TM_EINVAL;
    static const uint8_t kQueue[] = "$queue";
    auto starts = [&](const uint8_t* p, uint32_t n, const char* pre) {
        size_t k = std::strlen(pre);
        return n >= k && std::memcmp(p, pre, k) == 0;
    };
    const uint8_t* p = t;
    uint32_t n = len;
    bool shared = false;
    *group = nullptr;
    *group_len = 0;
    if (starts(p, n, "$queue/")) {
        p += 7, n -= 7;
        *group = kQueue;
        *group_len = 6;
        shared = true;
        if (starts(p, n, "$queue/") || starts(p, n, "$share/")) return TM_EINVAL;  // nested share
    } else if (starts(p, n, "$share/")) {
        const uint8_t* q = p + 7;
        uint32_t m = n - 7;
        const uint8_t* slash = (const uint8_t*)std::memchr(q, '/', m);
        if (!slash) return TM_EINVAL;  // [<<>>] or [_]
        uint32_t glen = (uint32_t)(slash - q);
        for (uint32_t i = 0; i < glen; ++i)
            if (q[i] == '+' || q[i] == '#') return TM_EINVAL;
        *group = q;
        *group_len = glen;
        p = slash + 1;
        n = m - glen - 1;
        shared = true;
    }
    (void)shared;
    *inner = p;
    *inner_len = n;
    return TM_OK;
}

}  // extern "C"
