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
#ifndef TM_CHUNK_ROWS
#define TM_CHUNK_ROWS 1
#endif
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <thread>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/topicmatch.h"
#include "image.h"
#include "kernels.h"

using namespace tmx;

extern "C" int tm_topic_wildcard(const uint8_t* topic, uint32_t len);

namespace {


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

// the elements of a host table written since the last commit: a log of
// indices (repeats allowed: the commit uploads each one's current value), or
// "all" once the log passes `limit` (a sixteenth of the table, set at every
// commit) -- then a plain copy of the whole table is cheaper than a scatter
struct Dirty {
    std::vector<uint32_t> idx;
    bool all = true;            // whole table must be (re)uploaded
    size_t limit = 1u << 16;
    void mark(size_t i) {
        if (all) return;
        if (idx.size() >= limit) {
            all = true;
            std::vector<uint32_t>().swap(idx);
            return;
        }
        idx.push_back((uint32_t)i);
    }
    void clear() {
        idx.clear();
        all = false;
    }
};

// a host table's dirty log since the last commit, and the previous commit's
// (which the other image epoch missed)
struct Track {
    Dirty cur, prev;
    void rotate(size_t table_elems) {
        prev = cur;
        cur.clear();
        cur.limit = std::max<size_t>(4096, table_elems / 16);
    }
    void mark_range(size_t from, size_t to) {   // elements [from, to)
        for (size_t i = from; i < to && !cur.all; ++i) cur.mark(i);
    }
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool pooled = false;   // from the device's stream-ordered pool (ensure_async)
    void release() {
        if (p) {
            if (pooled) {
                (void)hipFreeAsync(p, nullptr);
                (void)hipStreamSynchronize(nullptr);
            } else {
                (void)hipFree(p);
            }
        }
        p = nullptr;
        bytes = 0;
    }
    // ensure() through the stream-ordered pool on st: neither the free nor the
    // allocation synchronises the device (hipFree waits for every stream, so
    // an image commit would wait for the walks in flight on the other image).
    // The caller guarantees the old contents have no readers left, and orders
    // every use of the new buffer after st.
    bool ensure_async(size_t need, hipStream_t st, double slack = 1.25) {
        if (need <= bytes && p) return false;
        if (p) {
            if (pooled) HIPCHK(hipFreeAsync(p, st));
            else (void)hipFree(p);
        }
        p = nullptr;
        bytes = 0;
        size_t want = std::max<size_t>(256, (size_t)(need * slack));
        hipError_t e = hipMallocAsync(&p, want, st);
        if (e != hipSuccess) {
            p = nullptr;
            throw DevError(std::string("hipMallocAsync(") + std::to_string(want) + "): " + hipGetErrorString(e));
        }
        bytes = want;
        pooled = true;
        return true;
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
    uint16_t sum;         // S(v), the subtree summary (image.h): a superset between relayouts
    uint16_t lsum;        // union of S over v's literal children
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

// per-batch device workspace: consecutive batches rotate over the slots, so
// batches issued on different streams overlap on the GPU (the walk of one
// beside the tokenizer / copy-out of its neighbours); a slot's next user
// waits for its previous batch (hipStreamWaitEvent)
struct Slot {
    DevBuf twords, words, path, meta, scan, stage, kstage, ws, stats, perm, skeys, svals, scount, soff, sscan,
        twords_s, meta_s, spill, spill_head;
    DevBuf sctl;                    // tm_match_small's placement / completion counters (left zeroed by it)
    uint32_t spill_chunks = 0;      // spill capacity of the slot's last batch (0: none)
    bool sorted = false;            // the slot's last batch walked in presort order (perm valid)
    uint64_t* h_maxc = nullptr;     // pinned copy of the slot's ws after its last walk (largest match count,
                                    // spill chunks taken per XCD)
    hipEvent_t maxc_ev = nullptr, done = nullptr;
    bool maxc_pending = false, used = false, keyed = false, shaped = false;
    // the slot's last batch, for a re-copy into a larger output (no re-walk)
    uint32_t n = 0, K = 0, kw = 1;
    const uint8_t* bytes = nullptr;
    const uint64_t* off = nullptr;
    const uint32_t* counts = nullptr;
    const uint64_t* out_off = nullptr;
};
constexpr int MAX_SLOTS = 4;

// One committed trie image (nodes, edge tables, dictionary, word arena) in a
// GPU's HBM.  A replica keeps two (epochs): a commit writes the one no batch
// is reading and then flips, so tm_commit never waits for running walks;
// `uses` holds an event per batch launched on the image since it was last
// written, and only the next write to it waits for them (by then they are
// long done).
struct Image {
    DevBuf d_nodes, d_edges, d_hedges, d_dict, d_arena, d_woff, d_inner, d_leaf;
    // route image (routes.hip) and aggre tables (aggre.hip), same epoch as the
    // trie: a batch's filter ids and the route lists it expands them with
    // always come from one commit
    DevBuf d_rslots, d_rarena, d_rdest, d_fr_meta, d_rank_src, d_dt, d_rank_tg;
    DevBuf d_fshape;   // option "shape_keys": filter id -> order key
    DevBuf d_wheat;    // word id -> heat (option "presort" 2: the tail order's cost estimate)
    size_t arena_uploaded = 0, woff_uploaded = 0;
    uint64_t heat_uploaded = ~0ull;   // word_heat version in d_wheat
    uint32_t heat_words = 0;          // words in d_wheat (the host table may have grown since)
    bool split_stale = true, written = false;
    uint64_t epoch = 0;
    std::vector<hipEvent_t> uses;
    int pins = 0;   // batches between pin and unpin on it (their launches not all recorded in uses yet)
    // the views kernels get, captured when the image was written: a batch
    // reads these, never the host tables, which change under it
    ImageView iv{};
    RouteView rv{};
    AggreView av{};
    void release() {
        for (DevBuf* b : {&d_nodes, &d_edges, &d_hedges, &d_dict, &d_arena, &d_woff, &d_inner, &d_leaf, &d_rslots,
                          &d_rarena, &d_rdest, &d_fr_meta, &d_rank_src, &d_dt, &d_rank_tg, &d_fshape, &d_wheat})
            b->release();
        for (hipEvent_t ev : uses) (void)hipEventDestroy(ev);
        uses.clear();
    }
};

// One device replica: the committed images (trie, dictionary, route and aggre
// tables) in that GPU's HBM, its stream and its workspaces.  An engine has
// one replica per GPU it was opened on (tm_open_devices); they all mirror the
// one host trie, so a batch can be cut across them with no collective.
struct DevState {
    int device = -1;
    hipStream_t stream = nullptr;
    hipStream_t ustream = nullptr;   // commits: image uploads and scatters (never behind a batch on `stream`)
    // the pipelined host-buffer match (host_batch_pipelined): two chunk
    // workspaces, the read-back stream and the events between them
    hipStream_t hstream = nullptr;
    DevBuf hp_bytes[2], hp_off[2], hp_ids[2], hp_outoff[2], hp_total[2];
    hipEvent_t hp_comp[2] = {nullptr, nullptr}, hp_copy[2] = {nullptr, nullptr};
    uint64_t* hp_htot = nullptr;     // pinned: the chunk totals
    // trie image + dictionary, two epochs (Image)
    Image img[2];
    int cur = 0;                          // the image new batches pin (switched by commit, under the engine lock)
    int bimg = 0;                         // the image the running batch pinned
    std::vector<hipEvent_t> ev_spare;     // recycled use events
    // Locks: bmu = one batch at a time on this replica's workspaces, held for
    // the whole call; the engine lock is taken inside it only to commit and
    // pin (so host deltas run while the GPU works); umu guards pins, uses and
    // ev_spare (a leaf lock)
    std::mutex bmu, umu;
    std::condition_variable ucv;
    Image& live() { return img[cur]; }
    void pin() {
        std::lock_guard<std::mutex> lk(umu);
        bimg = cur;
        ++img[bimg].pins;
    }
    void unpin() {
        std::lock_guard<std::mutex> lk(umu);
        --img[bimg].pins;
        ucv.notify_all();
    }
    // one use of the pinned image by a batch on st (pruned as uses complete)
    void note_use(hipStream_t st) {
        std::lock_guard<std::mutex> lk(umu);
        Image& im = img[bimg];
        if (im.uses.size() >= 64) {   // drop the completed ones
            size_t k = 0;
            for (hipEvent_t ev : im.uses)
                if (hipEventQuery(ev) == hipSuccess) ev_spare.push_back(ev);
                else im.uses[k++] = ev;
            im.uses.resize(k);
        }
        hipEvent_t ev = nullptr;
        if (!ev_spare.empty()) {
            ev = ev_spare.back();
            ev_spare.pop_back();
        } else {
            HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        }
        HIPCHK(hipEventRecord(ev, st));
        im.uses.push_back(ev);
    }
    // host: every batch that read image i has finished (none still pinned,
    // every recorded use complete)
    void drain_image(int i) {
        std::vector<hipEvent_t> evs;
        {
            std::unique_lock<std::mutex> lk(umu);
            ucv.wait(lk, [&] { return img[i].pins == 0; });
            evs.swap(img[i].uses);
        }
        for (hipEvent_t ev : evs) HIPCHK(hipEventSynchronize(ev));
        std::lock_guard<std::mutex> lk(umu);
        ev_spare.insert(ev_spare.end(), evs.begin(), evs.end());
    }
    // commit packets: the changed elements of every table, one H2D copy,
    // then a scatter per table into the back image
    struct ScatterOp {
        void* table;
        uint64_t off, n;
        uint32_t words;
    };
    std::vector<uint8_t> stage_host;
    std::vector<ScatterOp> stage_ops;
    DevBuf stage_dev;
    // workspaces: route / aggre (w_r*, w_d*, w_a*), host-buffer batches, merge
    DevBuf w_rexact, w_rscan, w_rids, w_rcounts, w_roff;
    DevBuf w_dsrc, w_dcount, w_akey, w_alarge;
    DevBuf w_mpre, w_mscan, w_bytes, w_off, w_counts, w_outoff, w_ids, w_total;
    // the route / aggre workspaces are shared by every stream:
    // rw_done is recorded after the last route or aggre kernel of a batch;
    // the host waits on it before the next batch reuses (or reallocates) the
    // workspaces and before it rewrites an image
    hipEvent_t rw_done = nullptr;
    bool rw_used = false;
    Slot slots[MAX_SLOTS];
    int next_slot = 0, last_slot = 0;
    uint32_t stage_k = 128;   // ids staged per topic (stage footprint n x K x 4 B: a wide row costs walk
                              // time in address translation, profiles/r02_ab/ab_stage_k.jsonl)
    uint32_t keyed_k = 0;     // K of keyed walks (grown by stage_auto)
    uint32_t unkeyed_k = 0;   // K of unkeyed walks once their lists mostly spilled (grown by stage_auto)
    uint64_t spill_chunks = 0;   // spill area of unkeyed walks (adapted per batch)
    uint32_t light_max = 31;     // presort 6: the light-tail cost-class bound (adapted per batch; 31 = none yet)
    // per-batch event records, accumulated until tm_last_kernel_times()
    std::vector<KTimes> ev_pool;          // recycled events
    std::vector<KTimes> ev_pending;       // recorded, not yet read
    KTimes ev_cur[N_KERNEL_SLOTS];
    tm_batch_stats stats{};               // counters of this replica's last stats-mode batch

    void rw_release(hipStream_t st) {
        if (!rw_done) HIPCHK(hipEventCreateWithFlags(&rw_done, hipEventDisableTiming));
        HIPCHK(hipEventRecord(rw_done, st));
        rw_used = true;
    }
    void rw_drain() {   // host: every route / aggre kernel issued so far has finished
        if (rw_used) HIPCHK(hipEventSynchronize(rw_done));
    }
    void release() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (ustream) (void)hipStreamSynchronize(ustream);
        if (rw_done) (void)hipEventDestroy(rw_done);
        img[0].release();
        img[1].release();
        for (hipEvent_t ev : ev_spare) (void)hipEventDestroy(ev);
        ev_spare.clear();
        for (DevBuf* b : {&stage_dev, &w_rexact, &w_rscan, &w_rids, &w_rcounts, &w_roff, &w_dsrc, &w_dcount, &w_akey,
                          &w_alarge, &w_mpre, &w_mscan, &w_bytes, &w_off, &w_counts, &w_outoff, &w_ids, &w_total,
                          &hp_bytes[0], &hp_bytes[1], &hp_off[0], &hp_off[1], &hp_ids[0], &hp_ids[1], &hp_outoff[0],
                          &hp_outoff[1], &hp_total[0], &hp_total[1]})
            b->release();
        for (auto& w : slots) {
            for (DevBuf* b : {&w.twords, &w.words, &w.path, &w.meta, &w.scan, &w.stage, &w.kstage, &w.ws, &w.stats,
                              &w.perm, &w.skeys, &w.svals, &w.scount, &w.soff, &w.sscan, &w.twords_s, &w.meta_s,
                              &w.spill, &w.spill_head, &w.sctl})
                b->release();
            if (w.done) (void)hipEventDestroy(w.done);
            if (w.maxc_ev) (void)hipEventDestroy(w.maxc_ev);
            if (w.h_maxc) (void)hipHostFree(w.h_maxc);
        }
        for (auto* v : {&ev_pool, &ev_pending})
            for (auto& k : *v) {
                (void)hipEventDestroy(k.a);
                (void)hipEventDestroy(k.b);
            }
        if (stream) (void)hipStreamDestroy(stream);
        if (ustream) (void)hipStreamDestroy(ustream);
        if (hstream) {
            (void)hipStreamSynchronize(hstream);
            (void)hipStreamDestroy(hstream);
        }
        for (int j = 0; j < 2; ++j) {
            if (hp_comp[j]) (void)hipEventDestroy(hp_comp[j]);
            if (hp_copy[j]) (void)hipEventDestroy(hp_copy[j]);
            hp_comp[j] = hp_copy[j] = nullptr;
        }
        if (hp_htot) (void)hipHostFree(hp_htot);
        hp_htot = nullptr;
        hstream = nullptr;
        stream = ustream = nullptr;
    }
};

}  // namespace

struct tm_engine {
    std::recursive_mutex mu;
    std::atomic<int> lock_waiters{0};   // API calls blocked on mu (a chunked delta batch yields to them)
    int device = -1;                  // first replica's HIP ordinal (-1: host-only engine)
    std::vector<std::unique_ptr<DevState>> devs;   // one replica per GPU (tm_open_devices)
    std::string last_error;
    std::atomic<uint64_t> epoch{0};   // commits published so far (the live image's epoch)

    // ---- word dictionary (host copy of dict/word_arena/word_off) ----
    std::vector<DictSlot> dict;
    size_t dict_used = 0;
    std::vector<uint8_t> word_arena;   // 8-aligned, zero-padded words
    std::vector<uint32_t> word_off;
    // word heat: floor(log2(1 + trie nodes a word labels)), the tail order's
    // per-level cost estimate (a word on many edges leads into many filters)
    std::vector<uint32_t> word_nodes;
    std::vector<uint8_t> word_heat;
    uint64_t heat_version = 0;
    void heat_bump(uint32_t w, int d) {
        if (w >= word_nodes.size()) return;
        word_nodes[w] = (uint32_t)((int64_t)word_nodes[w] + d);
        const uint32_t x = word_nodes[w] + 1;
        const uint8_t h = (uint8_t)(31 - __builtin_clz(x));
        if (h != word_heat[w]) {
            word_heat[w] = h;
            ++heat_version;
        }
    }
    Dirty dict_dirty;

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
    // the dirty maps of the previous commit (the other image missed them)
    Dirty prev_node_dirty, prev_cold_dirty, prev_hot_dirty, prev_dict_dirty;
    EdgeTable& tab(uint32_t parent) { return parent < hot_limit ? hot : cold; }
    const EdgeTable& tab(uint32_t parent) const { return parent < hot_limit ? hot : cold; }
    // ---- filter registry ----
    std::vector<uint8_t> filter_arena;
    std::vector<FilterRec> filters;
    std::vector<uint32_t> free_filters;
    // Deferred filter id reuse.  A batch's ids name filters of the image it
    // pinned, and its caller turns them into bytes afterwards (the NIF's
    // callbacks, tm_filters_gather): a deleted filter's id is reusable only
    // once no image holds it (two commits after the delete: both epochs
    // rewritten) and no lease (tm_lease_begin: a reader between its match
    // and its last gather) predates the commit that dropped it.  Until then
    // the id keeps its bytes, and the gather keeps serving them.
    std::deque<std::pair<uint64_t, uint32_t>> quarantine;   // (epoch from which images lack the id, id)
    // id -> the epoch of its live quarantine entry: a forced (caller-chosen)
    // re-insert takes an id out of quarantine in O(1) and leaves its deque
    // entry stale (skipped on release), as free_listed does for free_filters
    std::unordered_map<uint32_t, uint64_t> quarantined;
    std::vector<uint8_t> free_listed;                        // id has a live entry in free_filters
    std::mutex lease_mu;                                     // leaf lock
    std::multiset<uint64_t> leases;                          // epochs of the open leases
    uint64_t lease_begin() {
        std::lock_guard<std::mutex> lk(lease_mu);
        const uint64_t x = epoch.load();
        leases.insert(x);
        return x;
    }
    void lease_end(uint64_t x) {
        std::lock_guard<std::mutex> lk(lease_mu);
        auto it = leases.find(x);
        if (it != leases.end()) leases.erase(it);
    }
    // an id that left the images at epoch `vis` names nothing any more once
    // both epochs are rewritten (now >= vis + 1) and no lease predates vis
    bool quarantine_over(uint64_t vis, uint64_t now, uint64_t oldest) const { return now >= vis + 1 && oldest >= vis; }
    uint64_t oldest_lease() {   // under lease_mu
        return leases.empty() ? UINT64_MAX : *leases.begin();
    }
    void release_quarantine() {
        if (quarantine.empty()) return;
        std::lock_guard<std::mutex> lk(lease_mu);
        const uint64_t now = epoch.load();
        const uint64_t oldest = oldest_lease();
        while (!quarantine.empty()) {
            const uint64_t vis = quarantine.front().first;
            const uint32_t id = quarantine.front().second;
            auto it = quarantined.find(id);
            if (it == quarantined.end() || it->second != vis) {   // stale: re-inserted under its id meanwhile
                quarantine.pop_front();
                continue;
            }
            if (!quarantine_over(vis, now, oldest)) break;
            quarantined.erase(it);
            free_filters.push_back(id);
            free_listed[id] = 1;
            quarantine.pop_front();
        }
    }
    size_t live_filters = 0;

    // ---- device image (per replica: DevState) ----
    bool dev_dirty = true;
    int hist_enabled = 0;             // option "hist": per-level histogram in stats mode (diagnostic, slow)
    uint32_t walk_bpc = 0;            // option "walk_bpc": walk blocks per CU (0 = full occupancy)
    int xcdq = 1;                     // option "xcdq": per-XCD dequeue ranges in the queue walk (default on)
    int presort = 3;                  // option "presort": walk the batch in the order of a key of its first
                                      // eight words (presort.hip; 0 = arrival order, 1 the word-hash key,
                                      // 2 the tail order, 5 the word-hash key within each XCD range, 3 by
                                      // batch size: 5 from sort_min topics, else 2)
    uint32_t sort_min = 1500000;      // option "sort_min": presort 3's smallest batch in range-local word-hash order
                                      // (with the lanes' drains hidden: 2M 2.806-2.809 ms vs 2.861-2.868 in the
                                      // tail order, 1M 1.525 vs 1.514-1.515; profiles/r05_orders)
    uint32_t light_tail = 60;         // option "light_tail": presort 6 walks the lightest ~light_tail per mille of
                                      // each XCD range last (the cost classes that cover it in the previous batch)
    std::atomic<int> last_order{-1};  // the walk order (presort mode) of the last device batch (tm_debug_last_order)
    int host_pipeline = 1;            // option "host_pipeline": host-buffer match/1 batches of >= 2M topics on
                                      // one replica go up, walk and come back in 1M-topic chunks, overlapped
    uint32_t sort_bits = 24;          // option "sort_bits": key bits sorted (8..32, % 8; one radix pass per
                                      // 8): presort 1 sorts the word-hash key's top bits (16 walk as fast as
                                      // 32, profiles/r04_p), presort 5 the range's 3 bits over the key's top
                                      // sort_bits - 3 (24: 8M +0.6 % over 16, profiles/r04_t)
    int layout_mode = 1;              // option "layout": 0 off, 1 auto, 2 every commit (tests)
    size_t created_since_layout = 0;  // nodes created since the last relayout
    uint32_t hot_levels = 4;          // option "hot_levels": relayout puts depths <= H level by level (BFS)
                                      // (an in-process relayout to 2 / 3 / 6 walks 8M topics 5 % faster, but
                                      // the first layout at 3 does not: DESIGN 5.2b, profiles/r04_x, r04_final8)
                                      // first, then DFS-preorder subtrees (0 = DFS throughout)
    uint32_t edge_div = 4;            // option "edge_load": edge tables kept at load <= 1/edge_div
    uint32_t layout_order = 15;       // option "order" (default 15; A/B at C3, walk ms: 0 3.90, 1 3.84, 7 3.51-3.66, 15 3.44): bit 0 = a node's '+' child directly follows it
                                      // (the walk's most frequent step, 67 of 101 visits per topic at
                                      // C3, then lands in the line the parent's load fetched); bit 1 =
                                      // '#' nodes (never visited with words left) moved to the end;
                                      // bit 2 = heat order (heat_sort); bit 3 = heat from filter counts
    bool force_relayout = false;
    int split_halves = 1;             // option "split": walk reads separate inner / leaf half arrays
    int double_buffer = 1;            // option "double_buffer": two image epochs per replica (commit never waits
                                      // on running walks); 0: one image, commit waits for the walks on it
    int summaries = 1;                // option "summaries": subtree summaries in the inner half prune dead
                                      // '+' / literal subtrees (0: field 1 is FILTER_NONE, nothing pruned)

    // ---- route table: the emqx_route bag (src/emqx_router.erl:52-59) ----
    std::unordered_map<std::string, uint32_t> dest_index;   // dest bytes -> dest id
    std::vector<std::string> dest_names;
    static constexpr uint32_t SLOT_NONE = 0xFFFFFFFFu;
    // to_rank labels: an order-maintenance labelling of the topics (list
    // labelling with density thresholds per window), so a new topic costs
    // O(log^2 n) amortised relabels, not a re-rank of every topic.  The
    // ordered index keeps each topic's first 32 bytes (big-endian u64s, zero
    // padded: their numeric order is the bytes' order whenever they differ)
    // and its label in the tree node, so a search reads a full topic only on
    // a 32-byte tie (16 bytes tied ~6 topics each at C3, 32 almost none).
    struct RouteRec;
    struct OrdKey {
        uint64_t p[4];
        RouteRec* r;
        mutable uint32_t label;   // == r->label
    };
    struct OrdLess {
        bool operator()(const OrdKey& a, const OrdKey& b) const {
            for (int i = 0; i < 4; ++i)
                if (a.p[i] != b.p[i]) return a.p[i] < b.p[i];
            return a.r != b.r && *a.r->key < *b.r->key;
        }
    };
    using OrdSet = std::set<OrdKey, OrdLess>;
    // one topic with routes, and where the route image holds it
    struct RouteRec {
        std::vector<uint32_t> dests;          // the bag, insertion order
        // membership index once the bag passes BAG_INDEX_MIN dests (scanned
        // linearly below that): add/del of a route stay O(1) probes for
        // topics with tens of thousands of dests
        std::unique_ptr<std::unordered_set<uint32_t>> index;
        const std::string* key = nullptr;     // the route_bag key (node-stable)
        uint32_t slot = SLOT_NONE;            // exact-table slot (rt_slots)
        uint32_t fid = FILTER_NONE;           // trie filter of a wildcard topic, while both exist
        uint32_t label = 0;                   // to_rank: order label, Erlang binary order of the topics
        uint32_t off = 0, cap = 0;            // dest segment in rt_dest
        uint64_t arena = 0, words = 0;        // topic bytes in rt_arena (u64 words)
        OrdSet::iterator ord;                 // its entry in rt_order
        bool has(uint32_t d) const {
            return index ? index->count(d) != 0 : std::find(dests.begin(), dests.end(), d) != dests.end();
        }
    };
    static constexpr size_t BAG_INDEX_MIN = 32;
    std::unordered_map<std::string, RouteRec> route_bag;   // topic -> its routes
    size_t route_total = 0;
    // The route image, maintained in place by every add / del (no rebuild):
    // commit uploads the dirty pages into the back image epoch.
    //   rt_slots  exact-topic table (open addressing, load <= 1/2, backward-
    //             shift deletion): get_routes(Topic) of a publish topic
    //   rt_arena  topic bytes of the slots (u64 words, zero padded)
    //   rt_dest   dest segments, one per topic (capacity doubles; a moved
    //             segment leaves garbage, compacted past half the pool)
    //   fr_meta   filter id -> {segment, count, label}: the routes of a
    //             matched wildcard filter (the same segment as its slot)
    //   rank_src  label -> that topic as a route source (aggre's large lists)
    std::vector<ExactSlot> rt_slots = std::vector<ExactSlot>(16, ExactSlot{0, 0, 0, 0, 0, 0});
    std::vector<RouteRec*> rt_slot_rec = std::vector<RouteRec*>(16, nullptr);
    size_t rt_used = 0;
    std::vector<uint64_t> rt_arena;
    size_t rt_arena_garbage = 0;
    std::vector<uint32_t> rt_dest;
    size_t rt_dest_garbage = 0;
    size_t route_gc_min = 1u << 20;   // option "route_gc": garbage entries before a compaction is considered
    std::vector<uint4> fr_meta;
    std::vector<RouteRec*> fr_rec;   // filter id -> linked topic
    OrdSet rt_order;
    uint32_t label_bits = 16;        // label universe 2^label_bits
    std::vector<uint32_t> rank_src = std::vector<uint32_t>(1u << 16, TM_ROUTE_TOPIC_ID);
    Track t_slots, t_rarena, t_rdest, t_fr_meta, t_rank_src, t_dt, t_rank_tg;
    // ---- emqx_broker:aggre/1 targets (aggre.hip) ----
    // a dest aggregates to a target: a node (atom) or a $share group; targets
    // are interned as kind byte + key bytes, so string order is the Erlang
    // term order of the X in {To, X} (atom < binary, then bytewise)
    std::unordered_map<std::string, uint32_t> target_index;
    std::vector<std::string> target_names;
    std::vector<uint32_t> dest_target;      // dest id -> target id (TARGET_DEFAULT: node named by the dest bytes)
    static constexpr uint32_t TARGET_DEFAULT = 0xFFFFFFFFu;
    std::vector<uint2> dt;                  // dest id -> {target rank, target id | group << 31}
    std::vector<uint32_t> rank_tg;          // target rank -> target id
    bool targets_dirty = true;              // a dest or a dest's target was added: re-rank the targets

    // ---- batch pipeline knobs ----
    int nslots = 2;                     // option "slots"
    uint32_t stage_k_min = 128;         // option "stage_k" (TM_STAGE_K)
    int stage_auto = 1;                 // option "stage_auto": keyed walks grow K to the largest list seen
                                        // (no re-walks); unkeyed walks keep K and spill (kernels.h)
    int spill_on = 1;                   // option "spill": ids past K to spill chunks (0: re-walk, as keyed)
    int chunk_rows = TM_CHUNK_ROWS;     // option "chunk_rows" (kernels.h QueueBufs)
    int tok_wave = 1;                   // option "tok_wave" (kernels.h QueueBufs)
    uint32_t wave_walk_max = 32768;     // option "wave_walk_max": batches of at most this many topics take the
                                        // wave-per-topic walk (tm_walk_wave: ~2 dependent loads per level);
                                        // faster up to 16K topics, slower from 64K (profiles/r03_d)
    int shape_keys = 0;                 // option "shape_keys": keyed batches of <= 31 levels walk unkeyed and
                                        // take each id's order key from fshape (image.h filter_shape)
    std::vector<uint64_t> fshape;       // filter id -> filter_shape (kept always; uploaded with shape_keys)
    Track t_fshape;
    static constexpr size_t SPILL_BUDGET = 8ull << 30;   // spill-area cap per slot (bytes)
    static constexpr size_t STAGE_BUDGET = 16ull << 30;  // stage-row footprint cap (bytes, of 288 GB HBM)
    bool stats_enabled = false, timing_enabled = false;
    tm_batch_stats last_stats{};

    // scratch for words of one filter, and its path of nodes
    std::vector<uint32_t> tmp_words, tmp_path;

    tm_engine() {
        if (const char* v = std::getenv("TM_XCDQ")) xcdq = std::atoi(v) ? 1 : 0;
        if (const char* v = std::getenv("TM_STAGE_K")) {
            long k = std::atol(v);
            if (k >= 4 && k <= 4096 && !(k & 3)) {
                stage_k_min = (uint32_t)k;
                stage_auto = 0;
            }
        }
        dict.assign(1024, DictSlot{0, WORD_NONE, 0, 0, 0, 0});
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
            if (d.tag == dict_tag(h, len) && d.len == len && std::memcmp(&word_arena[word_off[d.word]], p, len) == 0)
                return d.word;
        }
    }
    void dict_place(uint64_t h, uint32_t id, uint32_t len) {
        size_t mask = dict.size() - 1;
        size_t s = h & mask;
        while (dict[s].word != WORD_NONE) s = (s + 1) & mask;
        DictSlot d{dict_tag(h, len), id, 0, 0, len, 0};
        uint8_t head[16] = {0};
        std::memcpy(head, &word_arena[word_off[id]], std::min<size_t>(16, len));
        std::memcpy(&d.head0, head, 8);
        std::memcpy(&d.head1, head + 8, 8);
        dict[s] = d;
        dict_dirty.mark(s);
    }
    void dict_grow() {
        std::vector<DictSlot> old;
        old.swap(dict);
        dict.assign(old.size() * 2, DictSlot{0, WORD_NONE, 0, 0, 0, 0});
        for (const DictSlot& d : old)
            if (d.word != WORD_NONE)
                dict_place(word_hash(&word_arena[word_off[d.word]], d.len), d.word, d.len);
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
        word_nodes.push_back(0);
        word_heat.push_back(0);
        ++heat_version;
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
        e.plus = SLOT_RECORD ? c.plus : child_sum(child);
#if TM_SLOT_RECORD
        e.hash_filter = c.hash_filter;
        e.lw = c.lw;
        e.lc = c.lc;
        e.self_filter = c.self_filter;
#endif
        return e;
    }
    // the summary a child's edge slot carries (image.h EdgeSlot): its own
    // S(c), so the walk drops a table child whose subtree cannot match
    uint32_t child_sum(uint32_t x) const { return summaries ? aux[x].sum : SUM_ALL; }
    void refresh_slot_sum(uint32_t x) {
        if (SLOT_RECORD) return;   // such slots carry the child's record instead
        const uint32_t p = aux[x].parent, w = aux[x].word;
        if (p == NODE_NONE || w == WORD_PLUS) return;
        if (w != WORD_HASH && !(nodes[p].plus & WIDE)) return;
        const size_t s = edge_find_slot(p, w);
        if (s == SIZE_MAX) return;
        EdgeSlot& e = tab(p).slots[s];
        const uint32_t v = child_sum(x);
        if (e.plus != v) {
            e.plus = v;
            tab(p).dirty.mark(s);
        }
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
        aux[id] = NodeAux{parent, word, 0, 0, (uint16_t)SUM_NONE, (uint16_t)SUM_NONE};
        if (word < WORD_MAX) heat_bump(word, +1);
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
        if (w < WORD_MAX) heat_bump(w, -1);
        nodes[c] = empty_node();
        aux[c] = NodeAux{NODE_NONE, 0, 0, 0, (uint16_t)SUM_NONE, (uint16_t)SUM_NONE};
        node_dirty.mark(c);
        free_nodes.push_back(c);
        --live_nodes;
        refresh_hf(v);   // a removed '#' child gives the field back to the summaries
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
            nodes[aux[c].parent].hash_filter2 = fid;
            touched(aux[c].parent);
            refresh_hf(aux[c].parent);
        }
    }
    // the inner half's field 1 (image.h): the '#' child's filter, else the
    // summaries of the '+' child and of the literal children
    uint32_t hf_value(uint32_t v) const {
        const Node& x = nodes[v];
        if (x.hash != NODE_NONE && nodes[x.hash].self_filter != FILTER_NONE) return nodes[x.hash].self_filter;
        const uint32_t pc = x.plus & NODE_MASK;
        const uint32_t sp = pc == NODE_NONE ? SUM_NONE : aux[pc].sum;
        const uint32_t sl = aux[v].lit_count ? aux[v].lsum : SUM_NONE;
        return summaries ? (SUM_TAG | sp | (sl << 15)) : FILTER_NONE;
    }
    void refresh_hf(uint32_t v) {
        const uint32_t x = hf_value(v);
        if (nodes[v].hash_filter != x) {
            nodes[v].hash_filter = x;
            touched(v);
        }
    }
    // a new filter at the end of tmp_path: OR it into the summaries of its
    // path (emqx_trie's insert only adds; deletes leave supersets)
    void add_summaries(bool hash_filter) {
        const uint32_t D = (uint32_t)tmp_path.size() - 1;
        for (uint32_t i = D + 1; i-- > 0;) {
            const uint32_t rel = D - i;
            uint32_t s = (rel < 10 ? (1u << rel) : 0x400u) | SUM_NONE;   // ends rel levels below path[i]
            if (hash_filter && i < D)   // the '#' filter fires at path[D-1], D-1-i levels below path[i]
                s = sum_union(s, std::min<uint32_t>(D - 1 - i, 15u) << 11);
            NodeAux& a = aux[tmp_path[i]];
            a.sum = (uint16_t)sum_union(a.sum, s);
            if (i > 0 && tmp_words[i - 1] < WORD_MAX)
                aux[tmp_path[i - 1]].lsum = (uint16_t)sum_union(aux[tmp_path[i - 1]].lsum, a.sum);
            if (i > 0) refresh_slot_sum(tmp_path[i]);
        }
        for (uint32_t i = 0; i < D; ++i) refresh_hf(tmp_path[i]);
    }

    // ------------------------------------------------------------------
    // filters
    // the id the next new filter takes (tm_insert_batch_ids), FILTER_NONE: allocate one
    uint32_t forced_fid = FILTER_NONE;
    bool forced_dup_first = false;   // a filter already present keeps its id (tm_insert_batch_routed)
    uint32_t new_filter(const uint8_t* p, uint32_t len, uint32_t node) {
        uint32_t id = FILTER_NONE;
        if (forced_fid != FILTER_NONE) {   // a caller-chosen (global) id: holes below it stay unused
            id = forced_fid;
            if (id >= 0x7FFFFFF0u) throw RangeError("filter id past 2^31 - 16");
            if (id >= filters.size()) {
                filters.resize((size_t)id + 1, FilterRec{0, 0, NODE_NONE});
                free_listed.resize(filters.size(), 0);
            } else if (filters[id].node != NODE_NONE) {
                throw ArgError("filter id " + std::to_string(id) + " in use");
            }
            auto q = quarantined.find(id);
            if (q != quarantined.end()) {
                // a deleted id batches in flight may still emit: taken again
                // at once only for the same filter (whatever those batches
                // name, it is still this filter) or once its quarantine is over
                const FilterRec& old = filters[id];
                const bool same = old.len == len && (len == 0 || std::memcmp(&filter_arena[old.off], p, len) == 0);
                if (!same) {
                    std::lock_guard<std::mutex> lk(lease_mu);
                    if (!quarantine_over(q->second, epoch.load(), oldest_lease()))
                        throw ArgError("filter id " + std::to_string(id) + " was deleted and may still be named by "
                                       "batches in flight: reusable for another filter after two commits and the "
                                       "leases open at its delete");
                }
                quarantined.erase(q);   // its deque entry goes stale
            }
            free_listed[id] = 0;        // a free_filters entry of it goes stale
        } else {
            if (free_filters.empty()) release_quarantine();
            while (!free_filters.empty()) {
                const uint32_t f = free_filters.back();
                free_filters.pop_back();
                if (free_listed[f]) {   // else stale: taken by a forced insert
                    free_listed[f] = 0;
                    id = f;
                    break;
                }
            }
            if (id == FILTER_NONE) {
                if (filters.size() >= 0x7FFFFFF0ull) throw RangeError("filter ids exhausted (2^31: the image tags summaries with bit 31)");
                id = (uint32_t)filters.size();
                filters.push_back(FilterRec{});
                free_listed.push_back(0);
            }
        }
        uint64_t off = filter_arena.size();
        filter_arena.insert(filter_arena.end(), p, p + len);
        filters[id] = FilterRec{off, len, node};
        if (fshape.size() < filters.size()) {
            const size_t old = fshape.size();
            fshape.resize(filters.size(), 0);
            t_fshape.mark_range(old, fshape.size());
        }
        fshape[id] = filter_shape(tmp_words.data(), (uint32_t)tmp_words.size());   // insert's split_words
        t_fshape.cur.mark(id);
        ++live_filters;
        on_filter_new(p, len, id);
        return id;
    }
    void free_filter(uint32_t id) {
        on_filter_free(id);
        filters[id].node = NODE_NONE;   // off / len stay: the gather serves the id until it is reused
        quarantine.emplace_back(epoch.load() + 1, id);   // the next commit drops it from the images
        quarantined[id] = epoch.load() + 1;
        --live_filters;
    }

    // emqx_trie:insert/1 (src/emqx_trie.erl:62-73)
    void insert(const uint8_t* p, uint32_t len) {
        split_words(p, len, true);
        uint32_t v = ROOT;
        tmp_path.assign(1, ROOT);
        for (uint32_t w : tmp_words) {
            v = child_or_create(v, w);
            tmp_path.push_back(v);
        }
        if (nodes[v].self_filter == FILTER_NONE) {
            set_topic(v, new_filter(p, len, v));
            add_summaries(!tmp_words.empty() && tmp_words.back() == WORD_HASH);
        } else if (forced_fid != FILTER_NONE && nodes[v].self_filter != forced_fid && !forced_dup_first) {
            // the filter is in the trie under another id: a caller that
            // believes it now has forced_fid would mis-name its matches
            // (tm_insert_batch_routed instead keeps the first occurrence's id)
            throw ArgError("filter already present under id " + std::to_string(nodes[v].self_filter) +
                           ", not " + std::to_string(forced_fid));
        }
        dev_dirty = true;
    }

    // tm_insert_batch_ids' pre-pass: the error insert() under
    // forced id `id` would throw for filter p, without changing anything, so
    // a batch that fails is refused whole instead of partly applied
    void check_forced(const uint8_t* p, uint32_t len, uint32_t id) {
        if (id == FILTER_NONE) throw ArgError("filter id FILTER_NONE");
        if (id >= 0x7FFFFFF0u) throw RangeError("filter id past 2^31 - 16");
        const uint32_t v = split_words(p, len, false) ? walk(tmp_words) : NODE_NONE;
        const uint32_t f = v != NODE_NONE ? nodes[v].self_filter : FILTER_NONE;
        if (f != FILTER_NONE) {
            if (f != id)
                throw ArgError("filter already present under id " + std::to_string(f) + ", not " + std::to_string(id));
            return;   // present under this id: insert is a no-op
        }
        if (id < filters.size() && filters[id].node != NODE_NONE)
            throw ArgError("filter id " + std::to_string(id) + " in use");
        auto q = quarantined.find(id);
        if (q != quarantined.end()) {
            const FilterRec& old = filters[id];
            const bool same = old.len == len && (len == 0 || std::memcmp(&filter_arena[old.off], p, len) == 0);
            std::lock_guard<std::mutex> lk(lease_mu);
            if (!same && !quarantine_over(q->second, epoch.load(), oldest_lease()))
                throw ArgError("filter id " + std::to_string(id) + " was deleted and may still be named by "
                               "batches in flight");
        }
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
        targets_dirty = true;   // dt must cover the new dest
        dev_dirty = true;
        return id;
    }
    // handle_cast({add_route, Route}) (:153-163) + add_trie_route/1 (:226-231);
    // trie = false: the bare mnesia:write of #route{} to emqx_route (a table
    // event of the delta feed): the route bag only, the trie is driven by
    // its own emqx_trie_node events
    void route_add(const uint8_t* t, uint32_t tlen, const uint8_t* d, uint32_t dlen, bool trie = true) {
        const uint32_t dest = intern_dest(d, dlen);
        std::string key(reinterpret_cast<const char*>(t), tlen);
        auto it = route_bag.find(key);
        if (it != route_bag.end() && it->second.has(dest)) return;   // lists:member(Route, get_routes(Topic)) -> ok
        const bool wild = tm_topic_wildcard(t, tlen);
        if (it == route_bag.end()) {
            if (wild && trie) insert(t, tlen);   // mnesia:wread -> [] -> emqx_trie:insert
            it = route_bag.emplace(std::move(key), RouteRec{}).first;
            RouteRec& r = it->second;
            r.key = &it->first;
            rt_arena_put(r);
            rt_slot_put(&r);
            order_insert(&r);
            if (wild) fr_link(&r, filter_of(t, tlen));
        }
        RouteRec& r = it->second;
        r.dests.push_back(dest);
        if (r.dests.size() == BAG_INDEX_MIN)
            r.index.reset(new std::unordered_set<uint32_t>(r.dests.begin(), r.dests.end()));
        else if (r.index)
            r.index->insert(dest);
        seg_write(r, r.dests.size() - 1);
        ++route_total;
        dev_dirty = true;
    }
    // handle_cast({del_route, Route}) (:165-187) + del_trie_route/1 (:252-260)
    // or del_direct_route/1 (:240-241); the emqx_subscriber check (:179) is
    // the broker's and stays in the caller.  trie = false: the bare
    // mnesia:delete_object of #route{} (emqx_router_helper:cleanup_routes/1,
    // src/emqx_router_helper.erl:156-160, deletes routes only: the filter
    // stays in the trie and match/1 keeps returning it)
    void route_del(const uint8_t* t, uint32_t tlen, const uint8_t* d, uint32_t dlen, bool trie = true) {
        auto di = dest_index.find(std::string(reinterpret_cast<const char*>(d), dlen));
        if (di == dest_index.end()) return;
        auto it = route_bag.find(std::string(reinterpret_cast<const char*>(t), tlen));
        if (it == route_bag.end()) return;   // [] -> ok
        RouteRec& r = it->second;
        if (!r.has(di->second)) return;      // delete_object of an absent route: no-op
        const size_t at = std::find(r.dests.begin(), r.dests.end(), di->second) - r.dests.begin();
        r.dests.erase(r.dests.begin() + at);
        if (r.index) {
            if (r.dests.size() < BAG_INDEX_MIN) r.index.reset();
            else r.index->erase(di->second);
        }
        --route_total;
        dev_dirty = true;
        if (!r.dests.empty()) {
            seg_write(r, at);
            return;
        }
        // the last route of the topic: out of the image, then [Route] -> emqx_trie:delete(Topic)
        fr_unlink(&r);
        rt_slot_del(&r);
        order_erase(&r);
        rt_dest_garbage += r.cap;
        rt_arena_garbage += r.words;
        route_bag.erase(it);
        if (trie && tm_topic_wildcard(t, tlen)) remove(t, tlen);
        maybe_compact_routes();
    }
    const std::vector<uint32_t>* get_routes(const uint8_t* t, uint32_t tlen) const {
        auto it = route_bag.find(std::string(reinterpret_cast<const char*>(t), tlen));
        return it == route_bag.end() ? nullptr : &it->second.dests;
    }
    // filter id of a trie filter (or FILTER_NONE)
    uint32_t filter_of(const uint8_t* p, uint32_t len) {
        if (!split_words(p, len, false)) return FILTER_NONE;
        const uint32_t v = walk(tmp_words);
        return v == NODE_NONE ? FILTER_NONE : nodes[v].self_filter;
    }

    // ---- route image maintenance ----
    // the slot, filter entry and label entry of topic r, from its record
    void rt_sync(const RouteRec& r) {
        const uint32_t count = (uint32_t)r.dests.size();
        if (r.slot != SLOT_NONE) {
            ExactSlot& s = rt_slots[r.slot];
            s.count = count;
            s.dest_off = r.off;
            s.rank = r.label;
            s.arena = r.arena * 8;
            t_slots.cur.mark(r.slot);
        }
        if (r.fid != FILTER_NONE) {
            fr_meta[r.fid] = make_uint4(r.off, count, r.label, 0u);
            t_fr_meta.cur.mark(r.fid);
        }
        rank_src[r.label] = r.fid != FILTER_NONE ? r.fid : TM_ROUTE_TOPIC_ID;
        t_rank_src.cur.mark(r.label);
    }
    // dests [from, end) of r into its segment (a new, doubled segment at the
    // pool's end when they no longer fit; the old one becomes garbage)
    void seg_write(RouteRec& r, size_t from) {
        const size_t n = r.dests.size();
        if (n > r.cap) {
            rt_dest_garbage += r.cap;
            uint32_t cap = std::max<uint32_t>(r.cap * 2, 2);
            while (cap < n) cap *= 2;
            if (rt_dest.size() + cap >= 0xFFFFFFF0ull) throw RangeError("route dest pool past 2^32 entries");
            r.off = (uint32_t)rt_dest.size();
            r.cap = cap;
            rt_dest.resize(rt_dest.size() + cap, 0);
            from = 0;
        }
        if (n > from) {
            std::copy(r.dests.begin() + from, r.dests.end(), rt_dest.begin() + r.off + from);
            t_rdest.mark_range(r.off + from, r.off + n);
        }
        rt_sync(r);
    }
    void rt_arena_put(RouteRec& r) {
        const uint32_t len = (uint32_t)r.key->size();
        r.words = std::max<uint64_t>(1, (len + 7) / 8);
        r.arena = rt_arena.size();
        rt_arena.resize(rt_arena.size() + r.words, 0);
        if (len) std::memcpy(&rt_arena[r.arena], r.key->data(), len);
        t_rarena.mark_range(r.arena, r.arena + r.words);
    }
    void rt_slot_put(RouteRec* r) {
        if ((rt_used + 1) * 2 > rt_slots.size()) rt_regrow(rt_slots.size() * 2);
        const uint8_t* t = reinterpret_cast<const uint8_t*>(r->key->data());
        const uint64_t h = word_hash(t, (uint32_t)r->key->size());
        const size_t mask = rt_slots.size() - 1;
        size_t s = h & mask;
        while (rt_slots[s].hash) s = (s + 1) & mask;
        rt_slots[s] = ExactSlot{h, (uint32_t)r->key->size(), 0, r->arena * 8, 0, 0};
        rt_slot_rec[s] = r;
        r->slot = (uint32_t)s;
        ++rt_used;
        t_slots.cur.mark(s);
    }
    // backward-shift deletion: later members of the probe run move up, so
    // lookups never need tombstones
    void rt_slot_del(RouteRec* r) {
        const size_t mask = rt_slots.size() - 1;
        size_t i = r->slot;
        for (size_t j = (i + 1) & mask; rt_slots[j].hash; j = (j + 1) & mask) {
            const size_t home = rt_slots[j].hash & mask;
            // move j into the hole at i unless its home lies cyclically in (i, j]
            const bool stays = i <= j ? (home > i && home <= j) : (home > i || home <= j);
            if (stays) continue;
            rt_slots[i] = rt_slots[j];
            rt_slot_rec[i] = rt_slot_rec[j];
            rt_slot_rec[i]->slot = (uint32_t)i;
            t_slots.cur.mark(i);
            i = j;
        }
        rt_slots[i] = ExactSlot{0, 0, 0, 0, 0, 0};
        rt_slot_rec[i] = nullptr;
        t_slots.cur.mark(i);
        r->slot = SLOT_NONE;
        --rt_used;
    }
    void rt_regrow(size_t cap) {
        std::vector<RouteRec*> recs;
        recs.reserve(rt_used);
        for (RouteRec* r : rt_slot_rec)
            if (r) recs.push_back(r);
        rt_slots.assign(cap, ExactSlot{0, 0, 0, 0, 0, 0});
        rt_slot_rec.assign(cap, nullptr);
        rt_used = 0;
        for (RouteRec* r : recs) {
            rt_slot_put(r);
            rt_sync(*r);
        }
        t_slots.cur.all = true;
    }
    // the pool and the arena rewritten without garbage (all pages re-uploaded)
    void maybe_compact_routes() {
        const bool dest_gc = rt_dest_garbage > route_gc_min && rt_dest_garbage * 2 > rt_dest.size();
        const bool arena_gc = rt_arena_garbage > route_gc_min / 4 && rt_arena_garbage * 2 > rt_arena.size();
        if (!dest_gc && !arena_gc) return;
        std::vector<uint32_t> nd;
        std::vector<uint64_t> na;
        if (dest_gc) nd.reserve(rt_dest.size() - rt_dest_garbage);
        if (arena_gc) na.reserve(rt_arena.size() - rt_arena_garbage);
        for (auto& kv : route_bag) {
            RouteRec& r = kv.second;
            if (dest_gc) {
                const uint32_t off = (uint32_t)nd.size();
                nd.insert(nd.end(), rt_dest.begin() + r.off, rt_dest.begin() + r.off + r.cap);
                r.off = off;
            }
            if (arena_gc) {
                const uint64_t a = na.size();
                na.insert(na.end(), rt_arena.begin() + r.arena, rt_arena.begin() + r.arena + r.words);
                r.arena = a;
            }
            rt_sync(r);
        }
        if (dest_gc) {
            rt_dest.swap(nd);
            rt_dest_garbage = 0;
            t_rdest.cur.all = true;
        }
        if (arena_gc) {
            rt_arena.swap(na);
            rt_arena_garbage = 0;
            t_rarena.cur.all = true;
        }
    }
    // a wildcard topic's filter id <-> its routes
    void fr_link(RouteRec* r, uint32_t fid) {
        if (fid == FILTER_NONE) return;
        if (fid >= fr_meta.size()) {
            const size_t old = fr_meta.size(), n = std::max<size_t>(fid + 1, filters.size());
            fr_meta.resize(n, make_uint4(0, 0, 0, 0));
            fr_rec.resize(n, nullptr);
            t_fr_meta.mark_range(old, n);
        }
        r->fid = fid;
        fr_rec[fid] = r;
        rt_sync(*r);
    }
    void fr_unlink(RouteRec* r) {
        if (r->fid == FILTER_NONE) return;
        fr_meta[r->fid] = make_uint4(0, 0, 0, 0);
        fr_rec[r->fid] = nullptr;
        t_fr_meta.cur.mark(r->fid);
        r->fid = FILTER_NONE;
        rt_sync(*r);
    }
    // trie hooks (new_filter / free_filter): a filter created or deleted
    // outside add_route / del_route (tm_insert / tm_delete of a topic that
    // has routes) keeps the link right
    void on_filter_new(const uint8_t* p, uint32_t len, uint32_t fid) {
        if (route_bag.empty() || !tm_topic_wildcard(p, len)) return;
        auto it = route_bag.find(std::string(reinterpret_cast<const char*>(p), len));
        if (it != route_bag.end() && it->second.fid == FILTER_NONE) fr_link(&it->second, fid);
    }
    void on_filter_free(uint32_t fid) {
        if (fid < fr_rec.size() && fr_rec[fid]) fr_unlink(fr_rec[fid]);
    }

    // ---- to_rank labels (order maintenance) ----
    static OrdKey ord_key(RouteRec* r) {
        uint8_t b[32] = {0};
        std::memcpy(b, r->key->data(), std::min<size_t>(32, r->key->size()));
        OrdKey k{{0, 0, 0, 0}, r, 0};
        for (int w = 0; w < 4; ++w)
            for (int i = 0; i < 8; ++i) k.p[w] = k.p[w] << 8 | b[8 * w + i];
        return k;
    }
    void set_label(const OrdKey& k, uint32_t label) {
        k.label = label;
        k.r->label = label;
        rt_sync(*k.r);
    }
    void order_insert(RouteRec* r) {
        auto it = rt_order.insert(ord_key(r)).first;
        r->ord = it;
        if ((uint64_t)rt_order.size() * 4 > (1ull << label_bits)) {   // keep the universe >= 4n
            relabel_all(label_bits + 1);
            return;
        }
        const int64_t U = int64_t(1) << label_bits;
        const int64_t lo = it == rt_order.begin() ? -1 : (int64_t)std::prev(it)->label;
        const int64_t hi = std::next(it) == rt_order.end() ? U : (int64_t)std::next(it)->label;
        if (hi - lo >= 2) {
            set_label(*it, (uint32_t)(lo + (hi - lo) / 2));
            return;
        }
        // no gap: the smallest aligned window around the neighbours whose
        // density is under its threshold (1 at width 2, falling to 1/2 at the
        // whole universe) is spread evenly, the new topic included
        const int64_t anchor = lo >= 0 ? lo : 0;
        auto left = it, right = std::next(it);   // [left, right) = the window's members
        int64_t count = 1;
        for (uint32_t k = 1; k <= label_bits; ++k) {
            const int64_t L = (anchor >> k) << k, R = L + (int64_t(1) << k);
            while (left != rt_order.begin() && (int64_t)std::prev(left)->label >= L) {
                --left;
                ++count;
            }
            while (right != rt_order.end() && (int64_t)right->label < R) {
                ++right;
                ++count;
            }
            const double tau = 1.0 - 0.5 * (double)k / (double)label_bits;
            if ((double)count <= tau * (double)(R - L)) {
                spread(left, right, count, L, R);
                return;
            }
        }
        relabel_all(label_bits + 1);
    }
    // members [a, b) (count of them) get labels evenly spaced in [L, R)
    void spread(OrdSet::iterator a, OrdSet::iterator b, int64_t count, int64_t L, int64_t R) {
        const double step = (double)(R - L) / (double)count;
        int64_t i = 0;
        for (auto x = a; x != b; ++x, ++i) set_label(*x, (uint32_t)(L + (int64_t)(step * (double)i + step / 2)));
    }
    void relabel_all(uint32_t bits) {
        while ((uint64_t)rt_order.size() * 4 > (1ull << bits)) ++bits;
        if (bits > 31) throw RangeError("route topics past 2^29: to_rank labels exhausted");
        label_bits = bits;
        rank_src.assign(size_t(1) << bits, TM_ROUTE_TOPIC_ID);
        t_rank_src.cur.all = true;
        if (!rt_order.empty()) spread(rt_order.begin(), rt_order.end(), (int64_t)rt_order.size(), 0, int64_t(1) << bits);
    }
    void order_erase(RouteRec* r) { rt_order.erase(r->ord); }   // its label is simply free again

    // ------------------------------------------------------------------
    // emqx_broker:aggre/1 (src/emqx_broker.erl:194-206) targets: per dest its
    // target's rank and id, the targets in Erlang term order.  Small tables
    // (nodes and $share groups), re-ranked when a dest or a target is added.
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
    void rank_targets() {
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
        rank_tg.assign(tord.begin(), tord.end());
        dt.resize(nd);
        for (size_t d = 0; d < nd; ++d) {
            const uint32_t tid = dest_target[d];
            dt[d] = make_uint2(trank[tid], tid | (target_names[tid][0] ? 0x80000000u : 0u));
        }
        t_dt.cur.all = true;
        t_rank_tg.cur.all = true;
        targets_dirty = false;
    }
    AggreView make_aggre_view(const Image& g) const {
        AggreView av;
        av.dt = g.d_dt.as<const uint2>();
        av.rank_src = g.d_rank_src.as<const uint32_t>();
        av.rank_tg = g.d_rank_tg.as<const uint32_t>();
        return av;
    }
    RouteView make_route_view(const Image& g) const {
        RouteView rv;
        rv.fr_meta = g.d_fr_meta.as<const uint4>();
        rv.n_filters = (uint32_t)fr_meta.size();
        rv.ex_slots = g.d_rslots.as<const ExactSlot>();
        rv.ex_slot_mask = rt_slots.size() - 1;
        rv.ex_arena = g.d_rarena.as<const uint8_t>();
        rv.dest = g.d_rdest.as<const uint32_t>();
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
    // f(parent, word, child) for every literal edge of a WIDE node (in the
    // edge tables)
    template <class F>
    void table_literals(F&& f) const {
        for (const EdgeTable* t : {&cold, &hot})
            for (const EdgeSlot& e : t->slots)
                if (e.parent != EDGE_EMPTY && e.word != WORD_HASH) f(e.parent, e.word, e.child);
    }
    void relayout() {
        const size_t N = nodes.size();
        // literal children per node (inline or table edges), CSR
        std::vector<uint32_t> start(N + 1, 0);
        for (size_t v = 0; v < N; ++v) {
            if (aux[v].parent == NODE_NONE && v != ROOT) continue;  // free slot
            if (!(nodes[v].plus & WIDE) && nodes[v].lw != WORD_NONE) start[v + 1]++;
        }
        table_literals([&](uint32_t p, uint32_t, uint32_t) { start[p + 1]++; });
        for (size_t v = 0; v < N; ++v) start[v + 1] += start[v];
        std::vector<uint32_t> kids(start[N]);
        {
            std::vector<uint32_t> fill(start.begin(), start.end() - 1);
            for (size_t v = 0; v < N; ++v) {
                if (aux[v].parent == NODE_NONE && v != ROOT) continue;
                if (!(nodes[v].plus & WIDE) && nodes[v].lw != WORD_NONE) kids[fill[v]++] = nodes[v].lc;
            }
            table_literals([&](uint32_t p, uint32_t, uint32_t c) { kids[fill[p]++] = c; });
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
        // exact subtree summaries: `order` lists parents before children, so
        // in reverse every subtree is complete before its root
        for (uint32_t v : order) aux[v].sum = aux[v].lsum = (uint16_t)SUM_NONE;
        for (size_t i = order.size(); i-- > 0;) {
            const uint32_t v = order[i];
            NodeAux& a = aux[v];
            if (nodes[v].self_filter != FILTER_NONE) a.sum = (uint16_t)sum_union(a.sum, sum_end0());
            if (v == ROOT || a.parent == NODE_NONE) continue;
            NodeAux& pa = aux[a.parent];
            pa.sum = (uint16_t)sum_union(pa.sum, sum_shift(a.sum));
            if (a.word < WORD_MAX) pa.lsum = (uint16_t)sum_union(pa.lsum, a.sum);
            if (a.word == WORD_HASH && nodes[v].self_filter != FILTER_NONE)
                pa.sum = (uint16_t)sum_union(pa.sum, sum_hash0(SUM_NONE));
        }
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
        table_literals([&](uint32_t p, uint32_t w, uint32_t c) {
            EdgeSlot e{};
            e.parent = p;
            e.word = w;
            e.child = c;
            old.push_back(e);
        });
        for (EdgeTable* t : {&cold, &hot}) {
            for (const EdgeSlot& e : t->slots)
                if (e.parent != EDGE_EMPTY && e.word == WORD_HASH) old.push_back(e);
            std::vector<EdgeSlot>().swap(t->slots);
            t->used = 0;
        }
        for (const EdgeSlot& e : old)
            if (e.word != WORD_HASH) bloom_add(nn[newid[e.parent]], e.word);
        nodes.swap(nn);
        aux.swap(na);   // before the edges are placed: slot_for reads the children's new summaries
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
        for (uint32_t v = 0; v < nodes.size(); ++v) nodes[v].hash_filter = hf_value(v);
        if (SLOT_RECORD)   // the slots carry their children's records: those of the final hash_filter values
            for (EdgeTable* t : {&cold, &hot})
                for (EdgeSlot& e : t->slots)
                    if (e.parent != EDGE_EMPTY) e = slot_for(e.parent, e.word, e.child);
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

    // what a batch's kernels read: the views of the image it pinned
    static const ImageView& view(const DevState& d) { return d.img[d.bimg].iv; }
    static const RouteView& route_view(const DevState& d) { return d.img[d.bimg].rv; }
    static const AggreView& aggre_view(const DevState& d) { return d.img[d.bimg].av; }
    void capture_views(Image& g) const {
        g.iv = make_view(g);
        g.rv = make_route_view(g);
        g.av = make_aggre_view(g);
    }
    // the views of image g, from the host tables it was just written from
    ImageView make_view(const Image& g) const {
        ImageView im;
        if (split_halves && g.d_inner.p && !g.split_stale) {
            im.inner = g.d_inner.as<const uint8_t>();
            im.leaf = g.d_leaf.as<const uint8_t>();
            im.node_shift = 4;
        } else {
            im.inner = g.d_nodes.as<const uint8_t>();
            im.leaf = g.d_nodes.as<const uint8_t>() + 16;
            im.node_shift = 5;
        }
        im.edges = g.d_edges.as<const EdgeSlot>();
        im.edge_slot_mask = cold.slots.size() - 1;
        im.hot_edges = g.d_hedges.as<const EdgeSlot>();
        im.hot_slot_mask = hot.slots.size() - 1;
        im.hot_limit = hot_limit;
        im.dict = g.d_dict.as<const DictSlot>();
        im.dict_slot_mask = dict.size() - 1;
        im.word_arena = g.d_arena.as<const uint8_t>();
        im.word_off = g.d_woff.as<const uint32_t>();
        im.fshape = shape_keys ? g.d_fshape.as<const uint64_t>() : nullptr;
        im.word_heat = g.d_wheat.as<const uint8_t>();
        im.n_words = g.heat_words;
        return im;
    }

    // upload a host table to one replica: the whole table after a resize (or
    // when the replica is new), else the dirty pages; the caller clears the
    // dirty map once every replica has its copy
    // the elements changed since image g was last written (this commit's log
    // and, when g missed the previous commit (two epochs), that one's too):
    // packed for one scatter, or the whole table copied when that is cheaper
    template <class T>
    void upload_table(DevState& d, Image& g, DevBuf& buf, const std::vector<T>& host, const Dirty& dirty,
                      const Dirty& prev) {
        static_assert(sizeof(T) % 4 == 0, "tables are scattered in 32-bit words");
        const bool re = buf.ensure_async(std::max<size_t>(host.size(), 1) * sizeof(T), d.ustream);
        // g holds commit g.epoch; this one makes epoch + 1
        const bool two = g.written && g.epoch + 1 == epoch;        // g missed exactly the previous commit
        const bool stale = !g.written || g.epoch + 1 < epoch;      // missed more (double_buffer switched on)
        const size_t n = dirty.idx.size() + (two ? prev.idx.size() : 0);
        if (re || stale || dirty.all || (two && prev.all) || n * (4 + sizeof(T)) * 4 > host.size() * sizeof(T)) {
            if (!host.empty())
                HIPCHK(hipMemcpyAsync(buf.p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice, d.ustream));
            return;
        }
        if (n == 0) return;
        const uint64_t off = (d.stage_host.size() + 15) & ~uint64_t(15);
        d.stage_host.resize(off + n * (4 + sizeof(T)));
        uint32_t* ix = reinterpret_cast<uint32_t*>(d.stage_host.data() + off);
        // values as bytes: ix + n need not meet T's alignment (ExactSlot is
        // alignas(32)), so no T* may point there
        uint8_t* val = reinterpret_cast<uint8_t*>(ix + n);
        size_t k = 0;
        for (const Dirty* dl : {&dirty, &prev}) {
            if (dl == &prev && !two) break;
            for (uint32_t i : dl->idx) {
                if (i >= host.size())
                    throw DevError("commit: dirty index " + std::to_string(i) + " past a table of " +
                                   std::to_string(host.size()) + " elements of " + std::to_string(sizeof(T)) + " B");
                ix[k] = i;
                std::memcpy(val + k * sizeof(T), &host[i], sizeof(T));
                ++k;
            }
        }
        d.stage_ops.push_back(DevState::ScatterOp{buf.p, off, n, (uint32_t)(sizeof(T) / 4)});
    }
    // the packed changes of every table: one copy, a scatter per table
    void flush_stage(DevState& d) {
        if (d.stage_ops.empty()) return;
        d.stage_dev.ensure_async(d.stage_host.size(), d.ustream);
        HIPCHK(hipMemcpyAsync(d.stage_dev.p, d.stage_host.data(), d.stage_host.size(), hipMemcpyHostToDevice, d.ustream));
        for (const auto& op : d.stage_ops)
            HIPCHK(launch_scatter(op.table, reinterpret_cast<const uint32_t*>(d.stage_dev.as<uint8_t>() + op.off), op.n,
                                  op.words, d.ustream));
        d.stage_ops.clear();
        d.stage_host.clear();
    }

    void maybe_relayout() {
        if (force_relayout || layout_mode == 2 ||
            (layout_mode == 1 && live_nodes >= 4096 && created_since_layout * 4 >= live_nodes))
            relayout();
    }

    // Publish the host trie to every replica: the changes go to the image no
    // batch reads (after the batches that read it before the previous flip
    // have finished: normally long ago), then that image becomes live for the
    // batches launched from now on.  Batches in flight keep the image they
    // were launched on, consistent and untouched.
    void commit() {
        if (dev_dirty || devs.empty() || !devs[0]->img[devs[0]->cur].written) maybe_relayout();
        if (targets_dirty && !devs.empty()) rank_targets();
        if (devs.empty()) {
            ++epoch;
            dev_dirty = false;
            release_quarantine();
            return;
        }
        if (!dev_dirty && devs[0]->img[devs[0]->cur].written) {
            for (auto& dp : devs) {
                Image& g = dp->live();
                if (split_halves && g.split_stale) {   // option "split" turned on: derive the halves
                    Guard gd(dp->device);
                    dp->drain_image(dp->cur);
                    split_image(*dp, g);
                    HIPCHK(hipStreamSynchronize(dp->ustream));
                    capture_views(g);
                }
            }
            return;
        }
        for (auto& dp : devs) {
            DevState& d = *dp;
            Guard gd(d.device);
            const int back = double_buffer ? 1 - d.cur : d.cur;
            Image& g = d.img[back];
            d.drain_image(back);   // the batches launched on it before the last flip
            upload_table(d, g, g.d_nodes, nodes, node_dirty, prev_node_dirty);
            upload_table(d, g, g.d_edges, cold.slots, cold.dirty, prev_cold_dirty);
            upload_table(d, g, g.d_hedges, hot.slots, hot.dirty, prev_hot_dirty);
            upload_table(d, g, g.d_dict, dict, dict_dirty, prev_dict_dirty);
            upload_table(d, g, g.d_rslots, rt_slots, t_slots.cur, t_slots.prev);
            upload_table(d, g, g.d_rarena, rt_arena, t_rarena.cur, t_rarena.prev);
            upload_table(d, g, g.d_rdest, rt_dest, t_rdest.cur, t_rdest.prev);
            upload_table(d, g, g.d_fr_meta, fr_meta, t_fr_meta.cur, t_fr_meta.prev);
            upload_table(d, g, g.d_rank_src, rank_src, t_rank_src.cur, t_rank_src.prev);
            upload_table(d, g, g.d_dt, dt, t_dt.cur, t_dt.prev);
            upload_table(d, g, g.d_rank_tg, rank_tg, t_rank_tg.cur, t_rank_tg.prev);
            if (shape_keys) upload_table(d, g, g.d_fshape, fshape, t_fshape.cur, t_fshape.prev);
            flush_stage(d);
            // append-only arrays: upload the new tail (or all after a realloc)
            {
                const bool re = g.d_arena.ensure_async(std::max<size_t>(word_arena.size(), 8) + 16, d.ustream);
                const size_t from = re ? 0 : g.arena_uploaded;
                if (word_arena.size() > from)
                    HIPCHK(hipMemcpyAsync(g.d_arena.as<uint8_t>() + from, word_arena.data() + from,
                                          word_arena.size() - from, hipMemcpyHostToDevice, d.ustream));
                g.arena_uploaded = word_arena.size();
            }
            {
                const bool re = g.d_woff.ensure_async(std::max<size_t>(word_off.size(), 1) * 4, d.ustream);
                const size_t from = re ? 0 : g.woff_uploaded;
                if (word_off.size() > from)
                    HIPCHK(hipMemcpyAsync(g.d_woff.as<uint32_t>() + from, word_off.data() + from,
                                          (word_off.size() - from) * 4, hipMemcpyHostToDevice, d.ustream));
                g.woff_uploaded = word_off.size();
            }
            if (g.heat_uploaded != heat_version) {   // small: the whole table
                g.d_wheat.ensure_async(std::max<size_t>(word_heat.size(), 1) + 16, d.ustream);
                if (!word_heat.empty())
                    HIPCHK(hipMemcpyAsync(g.d_wheat.p, word_heat.data(), word_heat.size(), hipMemcpyHostToDevice,
                                          d.ustream));
                g.heat_uploaded = heat_version;
                g.heat_words = (uint32_t)word_heat.size();
            }
            g.split_stale = true;
            if (split_halves) split_image(d, g);
            HIPCHK(hipStreamSynchronize(d.ustream));   // host tables may change once this returns
            g.written = true;
            g.epoch = epoch + 1;
            capture_views(g);
            d.cur = back;   // live from the next batch on
        }
        // this commit's dirty pages become the "previous" set the other image
        // still needs at the next commit
        struct Rot {
            Dirty *cur, *prev;
            size_t elems;
        };
        for (const Rot& r : {Rot{&node_dirty, &prev_node_dirty, nodes.size()},
                             Rot{&cold.dirty, &prev_cold_dirty, cold.slots.size()},
                             Rot{&hot.dirty, &prev_hot_dirty, hot.slots.size()},
                             Rot{&dict_dirty, &prev_dict_dirty, dict.size()}}) {
            *r.prev = *r.cur;
            r.cur->clear();
            r.cur->limit = std::max<size_t>(4096, r.elems / 16);
        }
        t_slots.rotate(rt_slots.size());
        t_rarena.rotate(rt_arena.size());
        t_rdest.rotate(rt_dest.size());
        t_fr_meta.rotate(fr_meta.size());
        t_rank_src.rotate(rank_src.size());
        t_dt.rotate(dt.size());
        t_rank_tg.rotate(rank_tg.size());
        t_fshape.rotate(fshape.size());
        dev_dirty = false;
        ++epoch;
        release_quarantine();   // also for engines that only take forced ids (never reach new_filter's release)
    }

    // option "split": de-interleave the uploaded records into inner / leaf arrays
    void split_image(DevState& d, Image& g) {
        g.d_inner.ensure_async(nodes.size() * 16, d.ustream);
        g.d_leaf.ensure_async(nodes.size() * 16, d.ustream);
        HIPCHK(launch_split_nodes(g.d_nodes.p, nodes.size(), g.d_inner.p, g.d_leaf.p, d.ustream));
        g.split_stale = false;
    }

    // ------------------------------------------------------------------
    // the match pipeline on device buffers (all stream-ordered on st)
    static KTimes take_event(DevState& d, const char* name) {
        KTimes k{name, nullptr, nullptr};
        if (!d.ev_pool.empty()) {
            k = d.ev_pool.back();
            d.ev_pool.pop_back();
            k.name = name;
        } else {
            HIPCHK(hipEventCreate(&k.a));
            HIPCHK(hipEventCreate(&k.b));
        }
        return k;
    }
    // the walk order of an n-topic batch (option "presort" 3; C3, topics/s,
    // profiles/r04_o, r04_s): the word-hash order shares the trie's lines
    // between neighbouring lanes; sorted within each XCD range (5: every
    // prefix spread over all XCDs, each XCD's lanes grouped by prefix) it
    // beats the global sort (1: a key slice per XCD, so the hot prefixes
    // crowd one XCD): 8M 795-797M vs 767M (1) vs 741M (2), 4M 744-748M vs
    // 730M vs 711M; the tail order (2: heaviest topics first in each range,
    // one radix pass) shortens the walk's fixed ~0.4 ms tail and wins below
    // ~3M: 1M 622-624M vs 597-603M (5)
    // Heavy batches (lists mostly past the stage row, so the rows were
    // widened: C5, ~880 ids per topic) walk thousands of nodes per topic,
    // where lanes sharing prefixes matter more than the drain: the
    // range-local word-hash order with the light tail (6) at any size (C5
    // 1M topics: step 35.7 vs 38.9 ms in the tail order, profiles/r05_e)
    int presort_of(uint32_t n, const DevState& d) const {
        if (presort != 3) return presort;
        if (d.unkeyed_k > stage_k_min) return 6;
        return n >= sort_min ? 5 : 2;
    }
    // (presort 4: the tail order, then the word-hash key within each heat
    // class; 5: the word-hash key within each XCD range -- A/B orders)
    void ensure_slot(DevState& d, Slot& w, uint32_t n, uint64_t nbytes, uint32_t key_words, int presort) {
        w.twords.ensure((size_t)(n + 1) * WREG * 4);
        w.words.ensure((nbytes + n + 1) * 4);
        w.path.ensure((nbytes + 2ull * n + 2) * 4);
        w.stats.ensure(STATS_BYTES);
        w.meta.ensure((size_t)(n + 1) * 4);
        w.scan.ensure(scan_tmp_elems(n) * 8 + 8);
        w.stage.ensure(((size_t)n * d.stage_k + 4) * 4);
        if (key_words) w.kstage.ensure(((size_t)n * d.stage_k * key_words + 4) * 8);
        w.spill_chunks = 0;
        if (!key_words && spill_on && (!presort || chunk_rows) && d.spill_chunks >= 8) {
            w.spill.ensure((size_t)d.spill_chunks * SPILL_CHUNK * 4);
            w.spill_head.ensure((size_t)n * 4 + 4);
            w.spill_chunks = (uint32_t)d.spill_chunks;
        }
        w.ws.ensure(QWS_BYTES);
        if (presort) {
            w.perm.ensure((size_t)n * 4 + 4);
            if (key_words || !chunk_rows || stats_enabled) {   // the rows gathered into walk order (by_pos)
                w.twords_s.ensure((size_t)(n + 1) * WREG * 4);
                w.meta_s.ensure((size_t)n * 4 + 4);
            }
            const uint32_t nc = presort_counts(n);
            w.skeys.ensure((size_t)n * 8 + 8);
            w.svals.ensure((size_t)n * 4 + 4);
            w.scount.ensure((size_t)nc * 4 + 4);
            w.soff.ensure(((size_t)nc + 1) * 8);
            w.sscan.ensure(scan_tmp_elems(nc) * 8 + 8);
        }
        if (!w.done) HIPCHK(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    }

    // stage rows sized to the largest list of the previous walk (read back
    // asynchronously), within STAGE_BUDGET: fan-out beyond K costs a re-walk
    void adapt_stage_k(DevState& d, uint32_t n, uint32_t key_words) {
        uint64_t mc = 0, sp = 0, spt = 0;
        for (Slot& w : d.slots) {
            if (!w.maxc_pending || hipEventQuery(w.maxc_ev) != hipSuccess) continue;
            w.maxc_pending = false;
            uint64_t ht = 0;   // presort 6: the cost classes that hold the lightest light_tail per mille
            for (int c = 0; c < 32; ++c) ht += w.h_maxc[QWS_CHIST + c];
            if (ht) {
                uint64_t run = 0;
                uint32_t T = 0;
                for (; T < 31; ++T) {
                    run += w.h_maxc[QWS_CHIST + T];
                    if (run * 1000 >= ht * light_tail) break;
                }
                d.light_max = T;
            }
            mc = std::max<uint64_t>(mc, w.h_maxc[QWS_MAXC]);
            uint64_t t = 0;
            for (uint32_t x = 0; x < 8; ++x) {
                sp = std::max<uint64_t>(sp, w.h_maxc[QWS_SPILL + 16 * x]);
                t += w.h_maxc[QWS_SPILL + 16 * x];
            }
            spt = std::max(spt, t);
        }
        // spill area: n/16 chunks, or twice the most any XCD took last time
        // (an area that ran out re-walked its topics)
        const uint64_t want = std::max<uint64_t>((uint64_t)n / 16, 2 * 8 * sp);
        d.spill_chunks = std::min<uint64_t>(std::max<uint64_t>(d.spill_chunks, (want + 7) & ~7ull),
                                            SPILL_BUDGET / (SPILL_CHUNK * 4));
        if (!key_words && spill_on) {
            // unkeyed: a narrow row, the rare long list spills.  Batches whose
            // lists mostly pass K (more than one spill chunk per 8 topics: an
            // atomic per chunk, e.g. C5 at ~900 ids per topic) widen the rows
            // as keyed walks do (stage_auto), once: the spill stays the tail.
            if (stage_auto && mc && spt * 8 > n) {
                uint64_t wk = std::max<uint64_t>(stage_k_min, d.unkeyed_k);
                while (wk < mc && wk < 4096) wk <<= 1;
                while (wk > stage_k_min && (uint64_t)n * 4 * wk > STAGE_BUDGET) wk >>= 1;
                d.unkeyed_k = std::max<uint32_t>(d.unkeyed_k, (uint32_t)wk);
            }
            d.stage_k = std::max<uint32_t>(stage_k_min, d.unkeyed_k);
            return;
        }
        if (!stage_auto) {
            d.stage_k = stage_k_min;
            return;
        }
        if (d.stage_k < stage_k_min) d.stage_k = stage_k_min;
        d.keyed_k = std::max(d.keyed_k, d.stage_k);
        if (mc) {
            uint64_t wk = stage_k_min;
            while (wk < mc && wk < 4096) wk <<= 1;
            uint64_t k = d.keyed_k;
            const uint64_t per = (uint64_t)n * (4 + 8 * key_words);
            while (k < wk && per * (k << 1) <= STAGE_BUDGET) k <<= 1;
            d.keyed_k = (uint32_t)k;
        }
        d.stage_k = d.keyed_k;
    }
    // tm_reserve: every slot sized for batches of up to n topics (nbytes of
    // topic bytes), the spill area for n / 16 chunks
    void reserve(DevState& d, uint32_t n, uint64_t nbytes) {
        const uint64_t sp = std::min<uint64_t>(((uint64_t)n / 16 + 7) & ~7ull, SPILL_BUDGET / (SPILL_CHUNK * 4));
        d.spill_chunks = std::max<uint64_t>(d.spill_chunks, sp);
        const int presort = presort_of(n, d);
        bool cleared = false;
        for (int k = 0; k < nslots; ++k) {
            Slot& w = d.slots[k];
            ensure_slot(d, w, n, nbytes, 0, presort);
            if (!w.sctl.p) {
                w.sctl.ensure(64);
                HIPCHK(hipMemset(w.sctl.p, 0, 64));
                cleared = true;
            }
        }
        // only the memsets on the null stream are waited for (the engine's
        // streams are non-blocking): walks in flight on other streams go on
        // (a device-wide sync stalled every batcher's lanes)
        if (cleared) HIPCHK(hipStreamSynchronize(nullptr));
    }
    void record_maxc(Slot& w, hipStream_t st) {
        if (!w.h_maxc) HIPCHK(hipHostMalloc((void**)&w.h_maxc, QWS_BYTES, hipHostMallocDefault));
        if (!w.maxc_ev) HIPCHK(hipEventCreateWithFlags(&w.maxc_ev, hipEventDisableTiming));
        HIPCHK(hipMemcpyAsync(w.h_maxc, w.ws.p, QWS_BYTES, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(w.maxc_ev, st));
        w.maxc_pending = true;
    }

    // the whole hot path of one batch on replica d, stream-ordered on st:
    // CSR of ordered filter ids (ids past cap are dropped; *total always exact)
    void run_batch(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes,
                   uint32_t* counts, uint64_t* out_off, uint32_t* ids, uint64_t cap, uint64_t* total, hipStream_t st,
                   uint64_t* keys = nullptr, uint32_t key_words = 1) {
        // shape keys: a keyed batch of one key word walks unkeyed (narrow
        // rows, spill) and its copy-out takes each id's key from fshape; a
        // topic with a literal '+' / '#' level re-walks keyed there
        const bool shaped = keys && key_words == 1 && shape_keys;
        const uint32_t kw = keys && !shaped ? key_words : 0u;
        adapt_stage_k(d, n, kw);
        const int presort = presort_of(n, d);
        last_order = presort;
        // small batches walk one wave per topic (a wave-walk batch has no perm)
        const bool wave = n <= wave_walk_max && !kw && presort != 1;
        const int si = d.next_slot;
        d.next_slot = (d.next_slot + 1) % nslots;
        Slot& w = d.slots[si];
        if (w.used) HIPCHK(hipStreamWaitEvent(st, w.done, 0));   // its previous batch, maybe on another stream
        // every slot sized for this batch now: a slot first used later would
        // allocate (hipMalloc of GBs of stage rows) in the middle of a stream
        // of batches
        for (int k = 0; k < nslots; ++k) ensure_slot(d, d.slots[(si + k) % nslots], n, nbytes, kw, presort);
        d.last_slot = si;
        ImageView im = view(d);
        unsigned long long* sp = w.stats.as<unsigned long long>();
        if (stats_enabled) HIPCHK(hipMemsetAsync(w.stats.p, 0, STATS_BYTES, st));
        static const char* kStage[4] = {"tokenize", "walk", "scan", "copy_out"};
        hipEvent_t marks[8];
        if (timing_enabled)
            for (int i = 0; i < 4; ++i) {
                d.ev_cur[i] = take_event(d, kStage[i]);
                marks[2 * i] = d.ev_cur[i].a;
                marks[2 * i + 1] = d.ev_cur[i].b;
            }
        QueueBufs qb;
        qb.twords = w.twords.as<uint32_t>();
        qb.words = w.words.as<uint32_t>();
        qb.meta = w.meta.as<uint32_t>();
        qb.path = w.path.as<uint32_t>();
        qb.stage = w.stage.as<uint32_t>();
        qb.kstage = kw ? w.kstage.as<uint64_t>() : nullptr;
        qb.shaped = shaped;
        // the tail order (presort 2) leaves small batches to the wave walk
        qb.wave_walk = wave;   // (the range-keyed orders: 2, 4, 5, 6)
        qb.chunk_rows = chunk_rows;
        qb.tok_wave = tok_wave != 0;
        qb.scan_tmp = w.scan.as<uint64_t>();
        qb.ws = w.ws.as<unsigned long long>();
        qb.perm = presort && !shaped && !(qb.wave_walk && presort >= 2) ? w.perm.as<uint32_t>() : nullptr;
        qb.presort_mode = presort >= 2 ? (uint32_t)presort : 1u;
        qb.sort_passes = sort_bits / 8;
        qb.light_max = light_tail ? d.light_max : 31u;
        if (presort) {
            qb.sort_keys = w.skeys.as<uint32_t>();
            qb.sort_vals = w.svals.as<uint32_t>();
            qb.sort_counts = w.scount.as<uint32_t>();
            qb.sort_off = w.soff.as<uint64_t>();
            qb.sort_scan = w.sscan.as<uint64_t>();
            qb.twords_s = w.twords_s.as<uint32_t>();
            qb.meta_s = w.meta_s.as<uint32_t>();
        }
        if (w.spill_chunks) {
            qb.spill = w.spill.as<uint32_t>();
            qb.spill_head = w.spill_head.as<uint32_t>();
            qb.spill_chunks = w.spill_chunks;
        }
        w.sorted = queue_rows_by_position(qb, stats_enabled);   // the copy-out moves rows by perm
        HIPCHK(launch_queue(stats_enabled, xcdq != 0, im, bytes, off, n, qb, d.stage_k, counts, out_off, ids, keys,
                            cap, total, sp, st, timing_enabled ? marks : nullptr, walk_bpc, hist_enabled != 0,
                            keys ? key_words : 1u));
        d.note_use(st);   // the live image is read until this point of st
        w.keyed = kw != 0;
        w.shaped = shaped;
        w.n = n;
        w.K = d.stage_k;
        w.kw = keys ? key_words : 1u;
        w.bytes = bytes;
        w.off = off;
        w.counts = counts;
        w.out_off = out_off;
        record_maxc(w, st);
        HIPCHK(hipEventRecord(w.done, st));
        w.used = true;
        if (timing_enabled)
            for (int i = 0; i < 4; ++i) d.ev_pending.push_back(d.ev_cur[i]);
    }
    // a small batch in one launch (tm_match_small_device): tokenize, walk a
    // wave per topic, place each list with one atomic -- no stage rows, no
    // scan, no copy-out kernel.  Uses the next slot's row / word / path
    // buffers like run_batch; the slot's last CSR batch is not re-copied
    // after this (re-copies happen inside one call, under the batch lock).
    void run_small(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes,
                   uint32_t* counts, uint64_t* out_off, uint32_t* ids, uint64_t cap, uint64_t* total, hipStream_t st) {
        const int si = d.next_slot;
        d.next_slot = (d.next_slot + 1) % nslots;
        Slot& w = d.slots[si];
        if (w.used) HIPCHK(hipStreamWaitEvent(st, w.done, 0));   // its previous batch, maybe on another stream
        w.twords.ensure((size_t)(n + 1) * WREG * 4);
        w.words.ensure((nbytes + n + 1) * 4);
        w.path.ensure((nbytes + 2ull * n + 2) * 4);
        w.meta.ensure((size_t)(n + 1) * 4);
        if (!w.sctl.p) {
            w.sctl.ensure(64);
            HIPCHK(hipMemsetAsync(w.sctl.p, 0, 64, st));
        }
        if (!w.done) HIPCHK(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
        HIPCHK(launch_small(view(d), bytes, off, n, w.twords.as<uint32_t>(), w.words.as<uint32_t>(),
                            w.meta.as<uint32_t>(), w.path.as<uint32_t>(), counts, out_off, ids, cap, total,
                            w.sctl.as<unsigned long long>(), st));
        d.note_use(st);
        HIPCHK(hipEventRecord(w.done, st));
        w.used = true;
    }
    // emqx_router:match_routes/1 over a device batch (stream-ordered except
    // for one read of the match total that sizes the ids workspace)
    // the ids of replica d's last batch again, into a larger output: only
    // tm_copy_out runs (stage rows, counts and offsets are still in its slot)
    void recopy(DevState& d, uint32_t* ids, uint64_t* keys, uint64_t cap, hipStream_t st) {
        Slot& w = d.slots[d.last_slot];
        QueueBufs qb;
        qb.twords = w.twords.as<uint32_t>();
        qb.words = w.words.as<uint32_t>();
        qb.meta = w.meta.as<uint32_t>();
        qb.path = w.path.as<uint32_t>();
        qb.stage = w.stage.as<uint32_t>();
        qb.kstage = keys && w.keyed ? w.kstage.as<uint64_t>() : nullptr;
        qb.shaped = keys && w.shaped;
        qb.scan_tmp = w.scan.as<uint64_t>();
        qb.ws = w.ws.as<unsigned long long>();
        qb.perm = w.sorted ? w.perm.as<uint32_t>() : nullptr;   // the rows of a presorted walk
        if (w.spill_chunks && !w.keyed) {   // the spill chunks of the same walk
            qb.spill = w.spill.as<uint32_t>();
            qb.spill_head = w.spill_head.as<uint32_t>();
            qb.spill_chunks = w.spill_chunks;
        }
        HIPCHK(launch_copy(view(d), w.bytes, w.off, w.n, qb, w.K, w.kw, w.counts, w.out_off, ids, keys, cap, st));
        HIPCHK(hipEventRecord(w.done, st));
        d.note_use(st);
    }

    // match ids of a batch into d.w_rcounts / w_roff / w_rids with ONE walk
    // (an overflowing id workspace is grown and re-copied, not re-walked)
    void walk_ids(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes,
                  uint64_t* total, hipStream_t st) {
        d.w_rcounts.ensure((size_t)n * 4 + 4);
        d.w_roff.ensure((size_t)(n + 1) * 8);
        const uint64_t want = std::max<uint64_t>(d.w_rids.bytes / 4, (uint64_t)n * 16 + 1024);
        d.w_rids.ensure(want * 4, 1.0);
        const uint64_t icap = d.w_rids.bytes / 4;
        uint64_t ids_total = 0;
        run_batch(d, bytes, off, n, nbytes, d.w_rcounts.as<uint32_t>(), d.w_roff.as<uint64_t>(),
                  d.w_rids.as<uint32_t>(), icap, total, st);
        HIPCHK(hipMemcpyAsync(&ids_total, total, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (ids_total > icap) {
            d.w_rids.ensure(ids_total * 4, 1.25);   // contents not kept: the re-copy writes them all
            recopy(d, d.w_rids.as<uint32_t>(), nullptr, d.w_rids.bytes / 4, st);
        }
    }
    // match_routes/1 expansion of the ids walk_ids left in the workspace
    void emit_routes(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t* counts,
                     uint64_t* out_off, uint32_t* src, uint32_t* dest, uint64_t cap, uint64_t* total, hipStream_t st,
                     uint64_t* out_key = nullptr) {
        d.w_rexact.ensure((size_t)n * 16 + 16);
        d.w_rscan.ensure(scan_tmp_elems(n) * 8 + 8);
        const AggreView av_tmp = aggre_view(d);
        HIPCHK(launch_routes(route_view(d), bytes, off, n, d.w_rcounts.as<uint32_t>(), d.w_roff.as<uint64_t>(),
                             d.w_rids.as<uint32_t>(), d.w_rexact.as<uint4>(), counts, out_off, src, dest, cap, total,
                             d.w_rscan.as<uint64_t>(), st, out_key ? &av_tmp : nullptr, out_key));
    }
    void run_routes(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes,
                    uint32_t* counts, uint64_t* out_off, uint32_t* src, uint32_t* dest, uint64_t cap,
                    uint64_t* total, hipStream_t st) {
        // this path reads the match total back anyway (host sync per batch):
        // wait for the previous route / aggre batch of any stream, so its
        // workspaces can be reused or reallocated
        d.rw_drain();
        walk_ids(d, bytes, off, n, nbytes, total, st);
        emit_routes(d, bytes, off, n, counts, out_off, src, dest, cap, total, st);
        d.rw_release(st);
    }

    // aggre(match_routes(T)) over a device batch: the route lists and their
    // sort keys go to replica workspace (sized by the route total read back;
    // an overflow re-emits the routes, never re-walks), aggre.hip writes each
    // topic's list at its route offset; *total = route total
    void deliveries_routes(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes,
                           uint64_t* out_off, uint64_t* total, hipStream_t st, uint64_t& rcap) {
        d.rw_drain();   // w_d* / w_a* may be reallocated below
        d.w_dcount.ensure((size_t)n * 4 + 4);
        const uint64_t want = std::max<uint64_t>(d.w_dsrc.bytes / 8, (uint64_t)n * 16 + 1024);
        d.w_dsrc.ensure(want * 8, 1.0);
        d.w_akey.ensure(want * 8, 1.0);
        rcap = std::min(d.w_dsrc.bytes / 8, d.w_akey.bytes / 8);
        walk_ids(d, bytes, off, n, nbytes, total, st);
        uint64_t rtotal = 0;
        for (int pass = 0; pass < 2; ++pass) {
            uint32_t* src = d.w_dsrc.as<uint32_t>();
            emit_routes(d, bytes, off, n, d.w_dcount.as<uint32_t>(), out_off, src, src + rcap, rcap, total, st,
                        d.w_akey.as<uint64_t>());
            HIPCHK(hipMemcpyAsync(&rtotal, total, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (rtotal <= rcap) break;
            d.w_dsrc.ensure(rtotal * 8, 1.25);
            d.w_akey.ensure(rtotal * 8, 1.25);
            rcap = std::min(d.w_dsrc.bytes / 8, d.w_akey.bytes / 8);
        }
        d.w_alarge.ensure((size_t)n * 4 + 16);
    }
    void aggre_out(DevState& d, uint32_t n, const uint64_t* out_off, uint64_t rcap, uint32_t* counts, uint32_t* to,
                   uint32_t* target, uint64_t cap, hipStream_t st) {
        const uint32_t* src = d.w_dsrc.as<uint32_t>();
        HIPCHK(launch_aggre(aggre_view(d), n, d.w_dcount.as<uint32_t>(), out_off, src, src + rcap,
                            d.w_akey.as<uint64_t>(), d.w_alarge.as<uint32_t>(), counts, to, target, cap, st));
    }
    void run_deliveries(DevState& d, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint64_t nbytes,
                        uint32_t* counts, uint64_t* out_off, uint32_t* to, uint32_t* target, uint64_t cap,
                        uint64_t* total, hipStream_t st) {
        uint64_t rcap = 0;
        deliveries_routes(d, bytes, off, n, nbytes, out_off, total, st, rcap);
        aggre_out(d, n, out_off, rcap, counts, to, target, cap, st);
        d.rw_release(st);
    }

    void finish_batch(uint32_t n) {
        last_stats = tm_batch_stats{};
        last_stats.topics = n;
    }
    // counters of replica d's last stats-mode batch (synchronous read)
    tm_batch_stats read_stats(DevState& d, uint32_t n) {
        tm_batch_stats s{};
        s.topics = n;
        const DevBuf& ws = d.slots[d.last_slot].stats;
        if (!stats_enabled || !ws.p) return s;
        unsigned long long h[7] = {0, 0, 0, 0, 0, 0, 0};
        HIPCHK(hipMemcpy(h, ws.p, sizeof(h), hipMemcpyDeviceToHost));
        s.prunable_visits = h[6];
        s.levels = h[0];
        s.visits = h[1];
        s.edge_reads = h[2];
        s.matches = h[3];
        s.leaf_visits = h[4];
        s.probe_loads = h[5];
        return s;
    }

    // ------------------------------------------------------------------
    // replicas: which one a device-buffer call runs on, and a worker per
    // replica for host-buffer batches cut across them
    DevState* replica_for(const void* dptr) {
        if (devs.size() == 1 || !dptr) return devs[0].get();
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, dptr) == hipSuccess)
            for (auto& d : devs)
                if (d->device == at.device) return d.get();
        return devs[0].get();
    }
    struct Pool {
        std::vector<std::thread> th;
        std::mutex m;
        std::condition_variable cv, done_cv;
        std::vector<std::function<void()>> jobs;   // one slot per replica
        std::vector<char> busy;
        bool stop = false;
        void start(size_t k) {
            jobs.resize(k);
            busy.assign(k, 0);
            for (size_t i = 0; i < k; ++i)
                th.emplace_back([this, i] {
                    for (;;) {
                        std::function<void()> f;
                        {
                            std::unique_lock<std::mutex> lk(m);
                            cv.wait(lk, [&] { return stop || busy[i] == 1; });
                            if (stop) return;
                            f.swap(jobs[i]);
                        }
                        f();
                        {
                            std::lock_guard<std::mutex> lk(m);
                            busy[i] = 2;
                        }
                        done_cv.notify_all();
                    }
                });
        }
        // run f(i) for i < k, replica i's call on worker i (i = 0 on the caller)
        void run(size_t k, const std::function<void(size_t)>& f) {
            {
                std::lock_guard<std::mutex> lk(m);
                for (size_t i = 1; i < k; ++i) {
                    jobs[i] = [&f, i] { f(i); };
                    busy[i] = 1;
                }
            }
            cv.notify_all();
            f(0);
            std::unique_lock<std::mutex> lk(m);
            done_cv.wait(lk, [&] {
                for (size_t i = 1; i < k; ++i)
                    if (busy[i] != 2) return false;
                return true;
            });
            for (size_t i = 1; i < k; ++i) busy[i] = 0;
        }
        ~Pool() {
            {
                std::lock_guard<std::mutex> lk(m);
                stop = true;
            }
            cv.notify_all();
            for (auto& t : th) t.join();
        }
    };
    std::unique_ptr<Pool> pool;
    // run f(replica index) on every replica in parallel; exceptions are
    // carried back to the caller (the first one wins)
    void for_replicas(size_t k, const std::function<void(size_t)>& f) {
        if (k <= 1) {
            f(0);
            return;
        }
        if (!pool) {
            pool.reset(new Pool());
            pool->start(devs.size());
        }
        std::vector<std::exception_ptr> err(k);
        pool->run(k, [&](size_t i) {
            try {
                Guard g(devs[i]->device);
                f(i);
            } catch (...) {
                err[i] = std::current_exception();
            }
        });
        for (auto& x : err)
            if (x) std::rethrow_exception(x);
    }
};

// ---------------------------------------------------------------------------
namespace {

// Pinned host memory for library-sized outputs (tm_match_batch_owned): the
// lists come back over PCIe by DMA straight into them, and tm_free returns a
// block to a small pool for the next batch instead of unpinning it.
struct PinnedPool {
    std::mutex mu;
    std::unordered_map<void*, size_t> live;   // handed out: pointer -> bytes
    std::multimap<size_t, void*> spare;       // returned, kept pinned
    size_t spare_bytes = 0;
    static constexpr size_t SPARE_MAX = 8ull << 30;
    void* get(size_t need) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = spare.lower_bound(need);
        if (it != spare.end() && it->first <= need * 2) {
            void* p = it->second;
            live[p] = it->first;
            spare_bytes -= it->first;
            spare.erase(it);
            return p;
        }
        void* p = nullptr;
        const size_t want = std::max<size_t>(need + need / 4, 4096);
        if (hipHostMalloc(&p, want, hipHostMallocPortable) != hipSuccess) return nullptr;
        live[p] = want;
        return p;
    }
    bool put(void* p) {
        std::lock_guard<std::mutex> lk(mu);
        auto it = live.find(p);
        if (it == live.end()) return false;
        const size_t b = it->second;
        live.erase(it);
        spare.emplace(b, p);
        spare_bytes += b;
        while (spare_bytes > SPARE_MAX && !spare.empty()) {   // drop the largest spare blocks
            auto last = std::prev(spare.end());
            spare_bytes -= last->first;
            (void)hipHostFree(last->second);
            spare.erase(last);
        }
        return true;
    }
};
PinnedPool g_pinned;

// the C-ABI's error mapping: exception -> status code and message
template <class F>
int catching(std::string& err, F&& f) {
    try {
        return f();
    } catch (const ArgError& x) {
        err = x.what();
        return TM_EINVAL;
    } catch (const RangeError& x) {
        err = x.what();
        return TM_ERANGE;
    } catch (const DevError& x) {
        err = x.what();
        return TM_EDEVICE;
    } catch (const std::bad_alloc&) {
        err = "out of host memory";
        return TM_ENOMEM;
    } catch (const std::exception& x) {
        err = x.what();
        return TM_EDEVICE;
    } catch (...) {
        err = "unknown failure";
        return TM_EDEVICE;
    }
}

template <class F>
int guarded(tm_engine* e, F&& f, bool counted = true) {
    if (!e) return TM_EINVAL;
    if (counted) e->lock_waiters.fetch_add(1, std::memory_order_relaxed);
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    if (counted) e->lock_waiters.fetch_sub(1, std::memory_order_relaxed);
    std::string err;
    const int rc = catching(err, f);
    if (!err.empty()) e->last_error = err;
    return rc;
}

// A batch on replicas `reps` (ascending): their batch locks for the whole
// call; the engine lock only to commit and pin each replica's live image
// (its captured views), so deltas and commits proceed on the host while the
// batch runs and waits on the GPU; then, after the pins are released, the
// engine lock again for `post` (stats) or the error text.
template <class W, class P>
int batch_call(tm_engine* e, const std::vector<DevState*>& reps, W&& work, P&& post) {
    if (!e) return TM_EINVAL;
    std::vector<std::unique_lock<std::mutex>> held;
    held.reserve(reps.size());
    for (DevState* d : reps) held.emplace_back(d->bmu);
    int rc = guarded(e, [&] {
        e->commit();
        for (DevState* d : reps) d->pin();
        return TM_OK;
    });
    if (rc != TM_OK) return rc;
    std::string err;
    rc = catching(err, work);
    for (DevState* d : reps) d->unpin();
    return guarded(e, [&] {
        if (rc != TM_OK) {
            e->last_error = err;
            return rc;
        }
        post();
        return rc;
    });
}
int no_device(tm_engine* e, const char* what) {
    return guarded(e, [&] {
        e->last_error = std::string("engine is host-only (no device): ") + what + " runs on the GPU only";
        return TM_EDEVICE;
    });
}
std::vector<DevState*> all_replicas(tm_engine* e) {
    std::vector<DevState*> v;
    for (auto& d : e->devs) v.push_back(d.get());
    return v;
}
// the batch locks of every replica (in order): for the calls that read what
// batches write (slots, kernel-time events) outside the engine lock
std::vector<std::unique_lock<std::mutex>> lock_batches(tm_engine* e) {
    std::vector<std::unique_lock<std::mutex>> held;
    if (e)
        for (auto& d : e->devs) held.emplace_back(d->bmu);
    return held;
}

// a batch of deltas applied in chunks, the engine lock taken per chunk: each
// delta is its own transaction in the reference (mnesia, per route), so a
// batch need not be atomic, and a match launched meanwhile waits for one
// chunk at most instead of the whole batch.  Between chunks the batch lets
// every call already waiting for the lock go first (a plain mutex would
// hand it straight back to the thread that just released it).
// A chunk ends after 1024 deltas or 0.5 ms, whichever comes first.
constexpr uint32_t DELTA_CHUNK = 1024;
template <class F>
int chunked(tm_engine* e, uint32_t n, F&& one) {
    for (uint32_t c = 0; c < n;) {
        if (e && c)
            for (int spin = 0; e->lock_waiters.load(std::memory_order_relaxed) > 0 && spin < 100000; ++spin)
                std::this_thread::yield();
        const int rc = guarded(e, [&] {
            const auto t0 = std::chrono::steady_clock::now();
            const uint32_t end = std::min(n, c + DELTA_CHUNK);
            while (c < end) {
                one(c++);
                if ((c & 31) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(500)) break;
            }
            return TM_OK;
        }, false);
        if (rc != TM_OK) return rc;
    }
    return guarded(e, [] { return TM_OK; });
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
    const int32_t dev = cfg ? cfg->device : -1;
    return tm_open_devices(cfg, dev >= 0 ? &dev : nullptr, dev >= 0 ? 1u : 0u, out);
}

int tm_open_devices(const tm_config* cfg, const int32_t* devices, uint32_t n_devices, tm_engine** out) {
    if (!out || (n_devices && !devices) || n_devices > TM_MAX_REPLICAS) return TM_EINVAL;
    *out = nullptr;
    tm_engine* e = nullptr;
    try {
        e = new tm_engine();
    } catch (...) {
        return TM_ENOMEM;
    }
    if (cfg && cfg->filters_hint) {
        size_t nodes_hint = (size_t)cfg->filters_hint * 3;
        e->nodes.reserve(nodes_hint);
        e->aux.reserve(nodes_hint);
        // wide nodes' literal edges and '#' edges use the table (load <= 1/4)
        e->cold.slots.assign(next_pow2(nodes_hint), kEmptySlot);
    }
    int ndev = 0;
    if (n_devices && (hipGetDeviceCount(&ndev) != hipSuccess)) {
        delete e;
        return TM_EDEVICE;
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    for (uint32_t i = 0; i < n_devices; ++i) {
        std::unique_ptr<DevState> d(new (std::nothrow) DevState());
        if (!d || devices[i] < 0 || devices[i] >= ndev || hipSetDevice(devices[i]) != hipSuccess ||
            hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&d->ustream, hipStreamNonBlocking) != hipSuccess) {
            for (auto& x : e->devs) x->release();
            delete e;
            if (prev >= 0) (void)hipSetDevice(prev);
            return d ? TM_EDEVICE : TM_ENOMEM;
        }
        d->device = devices[i];
        d->stage_k = e->stage_k_min;
        {   // image buffers come from the stream-ordered pool (DevBuf::ensure_async);
            // keep what they free cached there, so trimming never waits on the device
            hipMemPool_t pool = nullptr;
            uint64_t keep = UINT64_MAX;
            if (hipDeviceGetDefaultMemPool(&pool, devices[i]) == hipSuccess)
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        }
        e->devs.push_back(std::move(d));
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    e->device = n_devices ? devices[0] : -1;
    *out = e;
    return TM_OK;
}

void tm_close(tm_engine* e) {
    if (!e) return;
    e->pool.reset();
    for (auto& d : e->devs) d->release();
    delete e;
}

int tm_engine_replicas(tm_engine* e) { return e ? (int)e->devs.size() : 0; }

int tm_engine_devices(tm_engine* e, int32_t* out, uint32_t cap) {
    if (!e || (cap && !out)) return TM_EINVAL;
    for (uint32_t i = 0; i < cap && i < e->devs.size(); ++i) out[i] = e->devs[i]->device;
    return (int)e->devs.size();
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
    return chunked(e, n, [&](uint32_t i) {
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
        e->insert(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
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

// routed sharded mode (topicmatch.h): the key is the first min(depth, levels)
// levels' bytes, hashed as the device hashes words (route.hip does the same)
uint32_t tm_route_of(const uint8_t* topic, uint32_t len, uint32_t n_shards, uint32_t depth, int is_filter) {
    if ((!topic && len) || n_shards == 0) return 0;
    uint32_t lev = 0, start = 0, cut = len;
    for (uint32_t i = 0; i <= len; ++i) {
        if (i == len || topic[i] == '/') {
            if (lev < depth && is_filter && i - start == 1 && (topic[start] == '+' || topic[start] == '#'))
                return TM_ROUTE_ALL;
            if (++lev == depth) {
                cut = i;
                break;
            }
            start = i + 1;
        }
    }
    if (n_shards == 1) return 0;
    return route_shard(word_hash(topic, cut), n_shards);
}

int tm_insert_batch_ids(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n, const uint32_t* ids) {
    if (n && (!bytes || !off || !ids)) return TM_EINVAL;
    return guarded(e, [&] {
        struct Reset {
            tm_engine* e;
            ~Reset() { e->forced_fid = FILTER_NONE; }
        } reset{e};
        // validate the whole batch first (each id free or this filter's, not
        // quarantined for another filter; no id or filter twice with
        // different partners), then insert: a refused batch changes nothing
        std::unordered_map<uint32_t, std::string_view> by_id;
        std::unordered_map<std::string_view, uint32_t> by_filter;
        for (uint32_t i = 0; i < n; ++i) {
            if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
            const std::string_view f(reinterpret_cast<const char*>(bytes + off[i]), (size_t)(off[i + 1] - off[i]));
            e->check_forced(bytes + off[i], (uint32_t)f.size(), ids[i]);
            auto a = by_id.emplace(ids[i], f);
            auto b = by_filter.emplace(f, ids[i]);
            if (a.first->second != f || b.first->second != ids[i])
                throw ArgError("batch names filter id " + std::to_string(ids[i]) + " or its filter twice");
        }
        for (uint32_t i = 0; i < n; ++i) {
            e->forced_fid = ids[i];
            e->insert(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        }
        return TM_OK;
    });
}

int tm_insert_batch_routed(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t n_shards,
                           uint32_t shard, uint32_t depth, uint32_t gid_base) {
    if ((n && (!bytes || !off)) || n_shards == 0 || shard >= n_shards || depth == 0) return TM_EINVAL;
    return guarded(e, [&] {
        struct Reset {
            tm_engine* e;
            ~Reset() {
                e->forced_fid = FILTER_NONE;
                e->forced_dup_first = false;
            }
        } reset{e};
        e->forced_dup_first = true;
        for (uint32_t i = 0; i < n; ++i) {
            if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
            const uint32_t len = (uint32_t)(off[i + 1] - off[i]);
            const uint32_t r = tm_route_of(bytes + off[i], len, n_shards, depth, 1);
            if (r != TM_ROUTE_ALL && r != shard) continue;
            e->forced_fid = gid_base + i;
            e->insert(bytes + off[i], len);
        }
        return TM_OK;
    });
}

int tm_delete_batch(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
    if (n && (!bytes || !off)) return TM_EINVAL;
    return chunked(e, n, [&](uint32_t i) {
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > 0xFFFFFFFFull) throw ArgError("bad offsets");
        e->remove(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
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

int tm_lease_begin(tm_engine* e, uint64_t* lease) {
    if (!e || !lease) return TM_EINVAL;
    *lease = e->lease_begin();
    return TM_OK;
}

void tm_lease_end(tm_engine* e, uint64_t lease) {
    if (e) e->lease_end(lease);
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
            if (f >= e->filters.size()) throw ArgError("unknown filter id");   // deleted ids: their bytes until reuse
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

namespace {
enum BatchKind { K_MATCH = 0, K_ROUTES = 1, K_DELIVERIES = 2 };

// A host-buffer batch cut into one contiguous slice per replica, run on all
// replicas at once (one worker per GPU): each uploads its slice, runs the
// pipeline into its workspace (grown and re-run only when a slice needs
// more), and reports its total; then each copies its lists to the caller's
// buffers at the prefix of the totals before it.  Results are identical to
// one replica running the whole batch.
// the body of a host-buffer batch, inside batch_call over every replica
// (the batch is cut across them); *stats_out gets the merged counters
// match/1 of a host batch on ONE replica, pipelined: chunks of HP_CHUNK
// topics go up, walk and come back on two streams, so the read-back of a
// chunk's ids (PCIe: 4 B per match, most of a host batch's time) overlaps the
// upload and walk of the next.  A chunk's ids land at the running total in
// the output (offsets rebased on the host at the end); an owned output is
// sized from the first chunk's fan-out and grown (host copy of what is there)
// if a later chunk outruns it.  Same results and errors as the one-shot path.
constexpr uint32_t HP_CHUNK = 1u << 20;
int host_batch_pipelined_body(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                              uint32_t* out_count, uint64_t* out_off, uint32_t* out_a, uint64_t out_cap,
                              uint64_t* out_needed, uint32_t** out_alloc);
// an owned output: pinned (DMA target) when the pool has it, else pageable
// (as the one-shot path); freed by tm_free either way
uint32_t* owned_ids(uint64_t n) {
    void* p = g_pinned.get(n * 4);
    if (!p) p = std::malloc(n * 4);
    if (!p) throw std::bad_alloc();
    return (uint32_t*)p;
}
int host_batch_pipelined(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                         uint32_t* out_count, uint64_t* out_off, uint32_t* out_a, uint64_t out_cap,
                         uint64_t* out_needed, uint32_t** out_alloc) {
    try {
        return host_batch_pipelined_body(e, topic_bytes, topic_off, n, out_count, out_off, out_a, out_cap, out_needed,
                                         out_alloc);
    } catch (...) {
        // an owned output handed out before a later chunk failed: no DMA may
        // still target it, and the caller gets no pointer (nothing to free)
        if (out_alloc && *out_alloc) {
            DevState& d = *e->devs[0];
            (void)hipStreamSynchronize(d.stream);
            if (d.hstream) (void)hipStreamSynchronize(d.hstream);
            tm_free(*out_alloc);
            *out_alloc = nullptr;
        }
        throw;
    }
}
int host_batch_pipelined_body(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                              uint32_t* out_count, uint64_t* out_off, uint32_t* out_a, uint64_t out_cap,
                              uint64_t* out_needed, uint32_t** out_alloc) {
    DevState& d = *e->devs[0];
    tm_engine::Guard g(d.device);
    hipStream_t s = d.stream;
    d.rw_drain();
    if (!d.hstream) HIPCHK(hipStreamCreateWithFlags(&d.hstream, hipStreamNonBlocking));
    for (int j = 0; j < 2; ++j) {
        if (!d.hp_comp[j]) HIPCHK(hipEventCreateWithFlags(&d.hp_comp[j], hipEventDisableTiming));
        if (!d.hp_copy[j]) HIPCHK(hipEventCreateWithFlags(&d.hp_copy[j], hipEventDisableTiming));
    }
    if (!d.hp_htot) HIPCHK(hipHostMalloc((void**)&d.hp_htot, 64, hipHostMallocDefault));
    d.w_counts.ensure((size_t)n * 4 + 4);
    const uint32_t nch = (n + HP_CHUNK - 1) / HP_CHUNK;
    std::vector<uint64_t> place(nch + 1, 0);
    std::vector<uint64_t> rel;
    uint32_t* out = out_alloc ? nullptr : out_a;
    uint64_t ocap = out_alloc ? 0 : out_cap;
    bool used[2] = {false, false};
    for (uint32_t k = 0; k < nch; ++k) {
        const int j = (int)(k & 1u);
        const uint32_t lo = k * HP_CHUNK, hi = std::min<uint32_t>(n, lo + HP_CHUNK), c = hi - lo;
        const uint64_t base = topic_off[lo], nb = topic_off[hi] - base;
        if (used[j]) HIPCHK(hipEventSynchronize(d.hp_copy[j]));   // chunk k-2's read-back left set j
        d.hp_bytes[j].ensure(nb + 16);
        d.hp_off[j].ensure((size_t)(c + 1) * 8);
        d.hp_outoff[j].ensure((size_t)(c + 1) * 8);
        d.hp_total[j].ensure(64);
        const uint64_t per = k ? place[k] / std::max<uint64_t>(lo, 1) + 1 : 16;   // ids per topic so far
        d.hp_ids[j].ensure(((uint64_t)c * per * 5 / 4 + 1024) * 4, 1.0);
        rel.assign(topic_off + lo, topic_off + hi + 1);
        for (auto& x : rel) x -= base;
        if (nb) HIPCHK(hipMemcpyAsync(d.hp_bytes[j].p, topic_bytes + base, nb, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(d.hp_off[j].p, rel.data(), (size_t)(c + 1) * 8, hipMemcpyHostToDevice, s));
        uint64_t cap = d.hp_ids[j].bytes / 4;
        uint64_t* d_total = d.hp_total[j].as<uint64_t>();
        e->run_batch(d, d.hp_bytes[j].as<uint8_t>(), d.hp_off[j].as<uint64_t>(), c, nb, d.w_counts.as<uint32_t>() + lo,
                     d.hp_outoff[j].as<uint64_t>(), d.hp_ids[j].as<uint32_t>(), cap, d_total, s);
        HIPCHK(hipMemcpyAsync(d.hp_htot + j, d_total, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const uint64_t total = d.hp_htot[j];
        if (total > cap) {   // the lists outgrew the chunk workspace: copy-out again, no re-walk
            d.hp_ids[j].ensure(total * 4, 1.25);
            cap = d.hp_ids[j].bytes / 4;
            e->recopy(d, d.hp_ids[j].as<uint32_t>(), nullptr, cap, s);
        }
        place[k + 1] = place[k] + total;
        if (out_alloc && place[k + 1] > ocap) {   // owned output: size it (first chunk) or grow it
            const uint64_t want = std::max<uint64_t>(place[k + 1] * 5 / 4,
                                                     (uint64_t)((double)place[k + 1] / hi * n * 1.15) + 1024);
            uint32_t* grown = owned_ids(want);
            if (out) {
                HIPCHK(hipStreamSynchronize(d.hstream));
                std::memcpy(grown, out, place[k] * 4);
                tm_free(out);
            }
            out = grown;
            ocap = want;
            *out_alloc = out;   // (the old block was freed above: *out_alloc never names a freed block)
        }
        // counts and chunk-local offsets on the walk's stream (small; the
        // caller's arrays may be pageable, which makes a copy wait on the
        // host: behind a previous chunk's ids on the read-back stream it would
        // stall the pipeline), then the ids that fit the output (past out_cap
        // the call reports TM_ENOSPC) on the read-back stream
        HIPCHK(hipMemcpyAsync(out_count + lo, d.w_counts.as<uint32_t>() + lo, (size_t)c * 4, hipMemcpyDeviceToHost,
                              s));
        HIPCHK(hipMemcpyAsync(out_off + lo, d.hp_outoff[j].p, (size_t)c * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventRecord(d.hp_comp[j], s));
        HIPCHK(hipStreamWaitEvent(d.hstream, d.hp_comp[j], 0));
        const uint64_t room = ocap > place[k] ? ocap - place[k] : 0;
        const uint64_t cp = std::min(total, room);
        if (cp) HIPCHK(hipMemcpyAsync(out + place[k], d.hp_ids[j].p, cp * 4, hipMemcpyDeviceToHost, d.hstream));
        HIPCHK(hipEventRecord(d.hp_copy[j], d.hstream));
        used[j] = true;
    }
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipStreamSynchronize(d.hstream));
    if (out_alloc && !out) {   // no ids at all: still a valid (empty) allocation for tm_free
        out = owned_ids(1);
        *out_alloc = out;
    }
    for (uint32_t k = 1; k < nch; ++k) {
        const uint32_t lo = k * HP_CHUNK, hi = std::min<uint32_t>(n, lo + HP_CHUNK);
        for (uint32_t t = lo; t < hi; ++t) out_off[t] += place[k];
    }
    const uint64_t total = place[nch];
    out_off[n] = total;
    if (out_needed) *out_needed = total;
    return total > ocap ? TM_ENOSPC : TM_OK;
}

int host_batch_work(tm_engine* e, BatchKind kind, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                    uint32_t* out_count, uint64_t* out_off, uint32_t* out_a, uint32_t* out_b, uint64_t out_cap,
                    uint64_t* out_needed, uint32_t** out_alloc, tm_batch_stats* stats_out) {
    *stats_out = tm_batch_stats{};
    stats_out->topics = n;
    for (uint32_t i = 0; i < n; ++i)
        if (topic_off[i + 1] < topic_off[i]) throw ArgError("topic offsets not monotone");
    if (n && topic_off[n] > topic_off[0] && !topic_bytes) throw ArgError("null topic bytes");
    if (n == 0) {
        out_off[0] = 0;
        if (out_needed) *out_needed = 0;
        if (out_alloc && !(*out_alloc = (uint32_t*)std::malloc(4))) throw std::bad_alloc();
        return TM_OK;
    }
    if (kind == K_MATCH && e->devs.size() == 1 && n >= 2 * HP_CHUNK && !e->stats_enabled && e->host_pipeline)
        return host_batch_pipelined(e, topic_bytes, topic_off, n, out_count, out_off, out_a, out_cap, out_needed,
                                    out_alloc);
    if (out_alloc) out_cap = UINT64_MAX;   // sized below at the exact total
    const size_t R = std::min<size_t>(e->devs.size(), n);
    const uint32_t planes = kind == K_MATCH ? 1u : 2u;
    std::vector<uint64_t> tot(R, 0), icap(R, 0);
    std::vector<tm_batch_stats> st(R);
    auto slice = [&](size_t i, uint32_t& lo, uint32_t& hi) {
        lo = (uint32_t)((uint64_t)n * i / R);
        hi = (uint32_t)((uint64_t)n * (i + 1) / R);
    };
    e->for_replicas(R, [&](size_t i) {
        DevState& d = *e->devs[i];
        uint32_t lo, hi;
        slice(i, lo, hi);
        const uint32_t m = hi - lo;
        const uint64_t base = topic_off[lo], nb = topic_off[hi] - base;
        hipStream_t s = d.stream;
        d.rw_drain();   // the host-buffer workspaces below are shared with route batches' host syncs
        d.w_bytes.ensure(nb + 16);
        d.w_off.ensure((size_t)(m + 1) * 8);
        d.w_counts.ensure((size_t)m * 4 + 4);
        d.w_outoff.ensure((size_t)(m + 1) * 8);
        d.w_total.ensure(64);
        std::vector<uint64_t> rel(topic_off + lo, topic_off + hi + 1);
        for (auto& x : rel) x -= base;
        if (nb) HIPCHK(hipMemcpyAsync(d.w_bytes.p, topic_bytes + base, nb, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(d.w_off.p, rel.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
        uint64_t* d_total = d.w_total.as<uint64_t>();
        const uint64_t elem = 4ull * planes;
        const uint64_t want = std::max<uint64_t>(d.w_ids.bytes / elem, (uint64_t)m * 16 + 1024);
        d.w_ids.ensure(want * elem, 1.0);
        uint64_t cap = d.w_ids.bytes / elem, total = 0, rcap = 0;
        // one walk; when the lists outgrow the workspace, only the last
        // stage (copy-out / route emit / aggre) runs again into a larger one
        uint32_t* a = d.w_ids.as<uint32_t>();
        if (kind == K_MATCH) {
            e->run_batch(d, d.w_bytes.as<uint8_t>(), d.w_off.as<uint64_t>(), m, nb, d.w_counts.as<uint32_t>(),
                         d.w_outoff.as<uint64_t>(), a, cap, d_total, s);
        } else if (kind == K_ROUTES) {
            d.rw_drain();
            e->walk_ids(d, d.w_bytes.as<uint8_t>(), d.w_off.as<uint64_t>(), m, nb, d_total, s);
            e->emit_routes(d, d.w_bytes.as<uint8_t>(), d.w_off.as<uint64_t>(), m, d.w_counts.as<uint32_t>(),
                           d.w_outoff.as<uint64_t>(), a, a + cap, cap, d_total, s);
        } else {
            e->deliveries_routes(d, d.w_bytes.as<uint8_t>(), d.w_off.as<uint64_t>(), m, nb,
                                 d.w_outoff.as<uint64_t>(), d_total, s, rcap);
            e->aggre_out(d, m, d.w_outoff.as<uint64_t>(), rcap, d.w_counts.as<uint32_t>(), a, a + cap, cap, s);
        }
        HIPCHK(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (total > cap && (out_alloc || total <= out_cap)) {
            d.w_ids.ensure(total * elem, 1.25);
            cap = d.w_ids.bytes / elem;
            a = d.w_ids.as<uint32_t>();
            if (kind == K_MATCH)
                e->recopy(d, a, nullptr, cap, s);
            else if (kind == K_ROUTES)
                e->emit_routes(d, d.w_bytes.as<uint8_t>(), d.w_off.as<uint64_t>(), m, d.w_counts.as<uint32_t>(),
                               d.w_outoff.as<uint64_t>(), a, a + cap, cap, d_total, s);
            else
                e->aggre_out(d, m, d.w_outoff.as<uint64_t>(), rcap, d.w_counts.as<uint32_t>(), a, a + cap, cap, s);
        }
        if (kind != K_MATCH) d.rw_release(s);
        tot[i] = total;
        icap[i] = cap;
        // straight into the caller's arrays (DMA when they are pinned): the
        // slice's local offsets, rebased below once every total is known
        HIPCHK(hipMemcpyAsync(out_count + lo, d.w_counts.p, (size_t)m * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(out_off + lo, d.w_outoff.p, (size_t)m * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (e->stats_enabled && kind == K_MATCH) st[i] = e->read_stats(d, m);
    });
    std::vector<uint64_t> pre(R + 1, 0);
    for (size_t i = 0; i < R; ++i) pre[i + 1] = pre[i] + tot[i];
    const uint64_t total = pre[R];
    if (out_alloc) {   // pinned (DMA target), else pageable
        *out_alloc = (uint32_t*)g_pinned.get(std::max<uint64_t>(total, 1) * 4);
        if (!*out_alloc) *out_alloc = (uint32_t*)std::malloc(std::max<uint64_t>(total, 1) * 4);
        if (!*out_alloc) throw std::bad_alloc();
        out_a = *out_alloc;
        out_cap = total;
    }
    e->for_replicas(R, [&](size_t i) {
        DevState& d = *e->devs[i];
        uint32_t lo, hi;
        slice(i, lo, hi);
        if (pre[i])
            for (uint32_t j = lo; j < hi; ++j) out_off[j] += pre[i];
        // the workspace holds min(total, cap) entries; past out_cap the call
        // reports TM_ENOSPC and copies what fits both
        const uint64_t room = out_cap > pre[i] ? out_cap - pre[i] : 0;
        const uint64_t c = std::min(std::min(tot[i], icap[i]), room);
        if (!c) return;
        HIPCHK(hipMemcpyAsync(out_a + pre[i], d.w_ids.p, c * 4, hipMemcpyDeviceToHost, d.stream));
        if (planes == 2)
            HIPCHK(hipMemcpyAsync(out_b + pre[i], d.w_ids.as<uint32_t>() + icap[i], c * 4, hipMemcpyDeviceToHost,
                                  d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
    });
    out_off[n] = total;
    if (e->stats_enabled && kind == K_MATCH)
        for (auto& s : st) {
            stats_out->levels += s.levels;
            stats_out->visits += s.visits;
            stats_out->edge_reads += s.edge_reads;
            stats_out->matches += s.matches;
            stats_out->leaf_visits += s.leaf_visits;
            stats_out->probe_loads += s.probe_loads;
            stats_out->prunable_visits += s.prunable_visits;
        }
    if (out_needed) *out_needed = total;
    return total > out_cap ? TM_ENOSPC : TM_OK;
}
int host_batch(tm_engine* e, BatchKind kind, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
               uint32_t* out_count, uint64_t* out_off, uint32_t* out_a, uint32_t* out_b, uint64_t out_cap,
               uint64_t* out_needed, uint32_t** out_alloc = nullptr) {
    if (!e) return TM_EINVAL;
    if (e->devs.empty()) return no_device(e, "the match path");
    tm_batch_stats stats{};
    return batch_call(e, all_replicas(e), [&] {
        return host_batch_work(e, kind, topic_bytes, topic_off, n, out_count, out_off, out_a, out_b, out_cap,
                               out_needed, out_alloc, &stats);
    }, [&] { e->last_stats = stats; });
}
}  // namespace

int tm_match_batch_owned(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                         uint32_t* out_count, uint64_t* out_off, uint32_t** out_ids, uint64_t* out_total) {
    if (!topic_off || !out_off || !out_ids || (n && !out_count)) return TM_EINVAL;
    *out_ids = nullptr;
    return host_batch(e, K_MATCH, topic_bytes, topic_off, n, out_count, out_off, nullptr, nullptr, 0, out_total,
                          out_ids);
}

void tm_free(void* p) {
    if (p && !g_pinned.put(p)) std::free(p);
}

int tm_match_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                   uint32_t* out_count, uint64_t* out_off, uint32_t* out_ids, uint64_t out_cap,
                   uint64_t* out_needed) {
    if (!topic_off || !out_off || (n && (!out_count)) || (out_cap && !out_ids)) return TM_EINVAL;
    return host_batch(e, K_MATCH, topic_bytes, topic_off, n, out_count, out_off, out_ids, nullptr, out_cap,
                          out_needed);
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
    return chunked(e, n, [&](uint32_t i) {
        if (topic_off[i + 1] < topic_off[i] || topic_off[i + 1] - topic_off[i] > 0xFFFFFFFFull ||
            dest_off[i + 1] < dest_off[i] || dest_off[i + 1] - dest_off[i] > 0xFFFFFFFFull)
            throw ArgError("bad offsets");
        e->route_add(topics + topic_off[i], (uint32_t)(topic_off[i + 1] - topic_off[i]), dests + dest_off[i],
                     (uint32_t)(dest_off[i + 1] - dest_off[i]));
    });
}

int tm_route_del(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen) {
    if ((!topic && tlen) || (!dest && dlen)) return TM_EINVAL;
    return guarded(e, [&] {
        e->route_del(topic, tlen, dest, dlen);
        return TM_OK;
    });
}

int tm_route_del_batch(tm_engine* e, const uint8_t* topics, const uint64_t* topic_off, const uint8_t* dests,
                       const uint64_t* dest_off, uint32_t n) {
    if (n && (!topics || !topic_off || !dests || !dest_off)) return TM_EINVAL;
    return chunked(e, n, [&](uint32_t i) {
        if (topic_off[i + 1] < topic_off[i] || topic_off[i + 1] - topic_off[i] > 0xFFFFFFFFull ||
            dest_off[i + 1] < dest_off[i] || dest_off[i + 1] - dest_off[i] > 0xFFFFFFFFull)
            throw ArgError("bad offsets");
        e->route_del(topics + topic_off[i], (uint32_t)(topic_off[i + 1] - topic_off[i]), dests + dest_off[i],
                     (uint32_t)(dest_off[i + 1] - dest_off[i]));
    });
}

// the emqx_route table events (delta feed): the bag only, never the trie
int tm_route_write(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen) {
    if ((!topic && tlen) || (!dest && dlen)) return TM_EINVAL;
    return guarded(e, [&] {
        e->route_add(topic, tlen, dest, dlen, false);
        return TM_OK;
    });
}

int tm_route_delete_object(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen) {
    if ((!topic && tlen) || (!dest && dlen)) return TM_EINVAL;
    return guarded(e, [&] {
        e->route_del(topic, tlen, dest, dlen, false);
        return TM_OK;
    });
}

int tm_route_write_batch(tm_engine* e, const uint8_t* topics, const uint64_t* topic_off, const uint8_t* dests,
                         const uint64_t* dest_off, uint32_t n) {
    if (n && (!topics || !topic_off || !dests || !dest_off)) return TM_EINVAL;
    return chunked(e, n, [&](uint32_t i) {
        if (topic_off[i + 1] < topic_off[i] || topic_off[i + 1] - topic_off[i] > 0xFFFFFFFFull ||
            dest_off[i + 1] < dest_off[i] || dest_off[i + 1] - dest_off[i] > 0xFFFFFFFFull)
            throw ArgError("bad offsets");
        e->route_add(topics + topic_off[i], (uint32_t)(topic_off[i + 1] - topic_off[i]), dests + dest_off[i],
                     (uint32_t)(dest_off[i + 1] - dest_off[i]), false);
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
    if (!e) return TM_EINVAL;
    if (e->devs.empty()) return no_device(e, "match_routes");
    DevState& d = *e->replica_for(d_off);
    return batch_call(e, {&d}, [&]() -> int {
        tm_engine::Guard g(d.device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : d.stream;
        if (n == 0) {
            HIPCHK(hipMemsetAsync(d_out_off, 0, 8, st));
            HIPCHK(hipMemsetAsync(d_total, 0, 8, st));
            return TM_OK;
        }
        e->run_routes(d, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_src, d_dest, out_cap, d_total, st);
        return TM_OK;
    }, [&] { e->finish_batch(n); });
}

int tm_match_routes_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                          uint32_t* out_count, uint64_t* out_off, uint32_t* out_src, uint32_t* out_dest,
                          uint64_t out_cap, uint64_t* out_needed) {
    if (!topic_off || !out_off || (n && !out_count) || (out_cap && (!out_src || !out_dest))) return TM_EINVAL;
    return host_batch(e, K_ROUTES, topic_bytes, topic_off, n, out_count, out_off, out_src, out_dest, out_cap,
                          out_needed);
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
            e->targets_dirty = true;
            e->dev_dirty = true;
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
    if (!e) return TM_EINVAL;
    if (e->devs.empty()) return no_device(e, "aggre");
    DevState& d = *e->replica_for(d_off);
    return batch_call(e, {&d}, [&]() -> int {
        tm_engine::Guard g(d.device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : d.stream;
        if (n == 0) {
            HIPCHK(hipMemsetAsync(d_out_off, 0, 8, st));
            HIPCHK(hipMemsetAsync(d_total, 0, 8, st));
            return TM_OK;
        }
        e->run_deliveries(d, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_to, d_target, out_cap, d_total,
                          st);
        return TM_OK;
    }, [&] { e->finish_batch(n); });
}

int tm_match_deliveries_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                              uint32_t* out_count, uint64_t* out_off, uint32_t* out_to, uint32_t* out_target,
                              uint64_t out_cap, uint64_t* out_needed) {
    if (!topic_off || !out_off || (n && !out_count) || (out_cap && (!out_to || !out_target))) return TM_EINVAL;
    return host_batch(e, K_DELIVERIES, topic_bytes, topic_off, n, out_count, out_off, out_to, out_target,
                          out_cap, out_needed);
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
    auto held = lock_batches(e);
    return guarded(e, [&]() -> int {
        *max_levels = 0;
        for (auto& dp : e->devs) {
            tm_engine::Guard g(dp->device);
            for (auto& w : dp->slots) {
                if (!w.used || !(w.keyed || w.shaped)) continue;
                HIPCHK(hipEventSynchronize(w.done));
                uint64_t x = 0;
                HIPCHK(hipMemcpy(&x, w.ws.as<uint64_t>() + QWS_MAXL, 8, hipMemcpyDeviceToHost));
                *max_levels = std::max<uint32_t>(*max_levels, (uint32_t)x);
            }
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
        if (e->devs.empty()) {
            e->last_error = "engine is host-only (no device): the merge runs on the GPU only";
            return TM_EDEVICE;
        }
        DevState& d = *e->replica_for(d_out_off);
        tm_engine::Guard g(d.device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : d.stream;
        d.w_mpre.ensure(((size_t)n_shards * (m + 1) + 1) * 8);
        if ((uint64_t)n_shards * m > 0xFFFFFFFFull) throw ArgError("n_shards x m exceeds 2^32");
        d.w_mscan.ensure(scan_tmp_elems(std::max<uint32_t>(n_shards * m, m)) * 8 + 8);
        HIPCHK(launch_shard_merge(n_shards, m, d_counts, d_src_base, d_ids, d_keys, d_out_count, d_out_off, d_out_gid,
                                  out_cap, d_total, d.w_mpre.as<uint64_t>(), d.w_mscan.as<uint64_t>(), st,
                                  key_words, key_stride));
        return TM_OK;
    });
}

static int match_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                        uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                        uint64_t* d_keys, uint32_t key_words, uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (!d_off || !d_out_off || !d_total || (n && !d_count) || (out_cap && !d_ids)) return TM_EINVAL;
    if (!e) return TM_EINVAL;
    if (e->devs.empty()) return no_device(e, "the match path");
    DevState& d = *e->replica_for(d_off);   // the replica on the GPU that holds the batch
    tm_batch_stats stats{};
    stats.topics = n;
    return batch_call(e, {&d}, [&]() -> int {
        tm_engine::Guard g(d.device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : d.stream;
        if (n == 0) {
            HIPCHK(hipMemsetAsync(d_out_off, 0, 8, st));
            HIPCHK(hipMemsetAsync(d_total, 0, 8, st));
            return TM_OK;
        }
        e->run_batch(d, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_ids, out_cap, d_total, st, d_keys,
                     key_words);
        if (e->stats_enabled) {
            HIPCHK(hipStreamSynchronize(st));
            stats = e->read_stats(d, n);
        }
        return TM_OK;
    }, [&] { e->last_stats = stats; });
}

int tm_match_small_device(tm_engine* e, const uint8_t* d_bytes, const uint64_t* d_off, uint32_t n,
                          uint64_t topic_bytes, uint32_t* d_count, uint64_t* d_out_off, uint32_t* d_ids,
                          uint64_t out_cap, uint64_t* d_total, void* hip_stream) {
    if (!d_off || !d_out_off || !d_total || (n && !d_count) || (out_cap && !d_ids)) return TM_EINVAL;
    if (!e) return TM_EINVAL;
    if (e->devs.empty()) return no_device(e, "the match path");
    DevState& d = *e->replica_for(d_off);
    return batch_call(e, {&d}, [&]() -> int {
        tm_engine::Guard g(d.device);
        hipStream_t st = hip_stream ? (hipStream_t)hip_stream : d.stream;
        e->run_small(d, d_bytes, d_off, n, topic_bytes, d_count, d_out_off, d_ids, out_cap, d_total, st);
        return TM_OK;
    }, [&] { e->finish_batch(n); });
}

// diagnostics (not part of include/topicmatch.h): the walk order of the
// last device batch (option "presort" resolved by batch size: 5 the
// range-local word-hash order, 2 the tail order, 0 arrival order ...)
extern "C" int tm_debug_last_order(tm_engine* e) { return e ? e->last_order.load() : TM_EINVAL; }

// diagnostics (not part of include/topicmatch.h): the phases of the last
// per-lane queue walk on replica 0, per XCD x (kernels.h QWS_CLOCK):
// out[4x..4x+3] = ms from the walk's first wave start to XCD x's first wave
// start, to the first exhaustion of its home range, to its last wave's end,
// and the chunks its waves stole (-1 where not recorded)
extern "C" int tm_debug_walk_clocks(tm_engine* e, double* out) {
    if (!e || !out) return TM_EINVAL;
    auto held = lock_batches(e);
    return guarded(e, [&]() -> int {
        if (e->devs.empty()) return TM_EINVAL;
        DevState& d = *e->devs[0];
        tm_engine::Guard g(d.device);
        const DevBuf& ws = d.slots[d.last_slot].ws;
        if (!ws.p) return TM_EINVAL;
        HIPCHK(hipDeviceSynchronize());
        std::vector<uint64_t> h(QWS_BYTES / 8);
        HIPCHK(hipMemcpy(h.data(), ws.p, QWS_BYTES, hipMemcpyDeviceToHost));
        int khz = 0;
        HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d.device));
        uint64_t t0 = UINT64_MAX;
        for (int x = 0; x < 8; ++x)
            if (h[QWS_CLOCK + 16 * x]) t0 = std::min<uint64_t>(t0, ~h[QWS_CLOCK + 16 * x]);
        for (int x = 0; x < 8; ++x) {
            const uint64_t* c = &h[QWS_CLOCK + 16 * x];
            auto ms = [&](uint64_t t) { return khz > 0 ? (double)(t - t0) / (double)khz : -1.0; };
            out[4 * x] = c[0] ? ms(~c[0]) : -1.0;
            out[4 * x + 1] = c[1] ? ms(~c[1]) : -1.0;
            out[4 * x + 2] = c[2] ? ms(c[2]) : -1.0;
            out[4 * x + 3] = (double)c[3];
        }
        return TM_OK;
    });
}

// diagnostics (not part of include/topicmatch.h): the last stats-mode
// batch's per-level histogram [visits, probe loads, failed probes] x 16
extern "C" int tm_debug_hist(tm_engine* e, uint64_t* out, int n) {
    if (!e || !out || n > 56) return TM_EINVAL;
    auto held = lock_batches(e);
    return guarded(e, [&]() -> int {
        if (e->devs.empty()) return TM_EINVAL;
        const DevBuf& ws = e->devs[0]->slots[e->devs[0]->last_slot].stats;
        if (!ws.p) return TM_EINVAL;
        HIPCHK(hipMemcpy(out, ws.as<uint64_t>() + 8, (size_t)n * 8, hipMemcpyDeviceToHost));
        return TM_OK;
    });
}

// diagnostics (not part of include/topicmatch.h): the host mirror of the
// trie image as the last commit laid it out, for the walk simulator
// (tools/sim/walksim.cpp): node records, edge tables, per-node parent and
// word; pointers stay valid until the next delta or commit
struct tm_debug_image_view {
    const void* nodes;       // Node[n_nodes], 32 B each (image.h)
    uint64_t n_nodes;
    const void* cold;        // EdgeSlot[cold_slots]
    uint64_t cold_slots;
    const void* hot;         // EdgeSlot[hot_slots]
    uint64_t hot_slots;
    uint32_t hot_limit;
    uint32_t aux_stride;     // bytes per aux record
    const void* aux;         // per node: {parent u32, word u32, edge_count u32, lit_count u32, ...}
};
extern "C" int tm_debug_image(tm_engine* e, tm_debug_image_view* out) {
    if (!e || !out) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        out->nodes = e->nodes.data();
        out->n_nodes = e->nodes.size();
        out->cold = e->cold.slots.data();
        out->cold_slots = e->cold.slots.size();
        out->hot = e->hot.slots.data();
        out->hot_slots = e->hot.slots.size();
        out->hot_limit = e->hot_limit;
        out->aux_stride = (uint32_t)sizeof(NodeAux);
        out->aux = e->aux.data();
        return TM_OK;
    });
}
// diagnostics: the word ids of n topics as the device tokenizer makes them
// (WORD_NONE for bytes no filter contains, WORD_PLUS / WORD_HASH for the
// atoms), levels[t] per topic, ids packed in topic order (cap ids at most)
extern "C" int tm_debug_words(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t* levels,
                              uint32_t* ids, uint64_t cap) {
    if (!e || (n && (!bytes || !off || !levels || !ids))) return TM_EINVAL;
    return guarded(e, [&]() -> int {
        uint64_t k = 0;
        for (uint32_t t = 0; t < n; ++t) {
            const uint8_t* p = bytes + off[t];
            const uint32_t len = (uint32_t)(off[t + 1] - off[t]);
            uint32_t s = 0, lv = 0;
            for (uint32_t i = 0; i <= len; ++i) {
                if (i == len || p[i] == '/') {
                    if (k >= cap) return TM_ENOSPC;
                    ids[k++] = e->word_id(p + s, i - s, false);
                    ++lv;
                    s = i + 1;
                }
            }
            levels[t] = lv;
        }
        return TM_OK;
    });
}

// diagnostics (not part of include/topicmatch.h): the in-place route image
// against the route bags it mirrors -- every topic found in the exact table
// by the kernel's probe, its segment equal to its bag, its filter entry, the
// labels strictly increasing in topic order, rank_src -- TM_OK or TM_EINVAL
// with the first inconsistency in tm_last_error
extern "C" int tm_debug_check_routes(tm_engine* e) {
    return guarded(e, [&]() -> int {
        auto fail = [&](const std::string& what) -> int { throw ArgError("route image: " + what); };
        size_t used = 0;
        for (size_t s = 0; s < e->rt_slots.size(); ++s)
            if (e->rt_slots[s].hash) {
                ++used;
                if (!e->rt_slot_rec[s] || e->rt_slot_rec[s]->slot != s) return fail("slot owner");
            }
        if (used != e->rt_used || used != e->route_bag.size()) return fail("slot count");
        size_t total = 0;
        for (auto& kv : e->route_bag) {
            const tm_engine::RouteRec& r = kv.second;
            const uint8_t* t = reinterpret_cast<const uint8_t*>(kv.first.data());
            const uint32_t len = (uint32_t)kv.first.size();
            total += r.dests.size();
            if (r.key != &kv.first || r.dests.empty()) return fail("record of " + kv.first);
            // the probe the kernel runs (routes.hip exact_lookup)
            const uint64_t h = word_hash(t, len);
            const size_t mask = e->rt_slots.size() - 1;
            size_t s = h & mask;
            while (e->rt_slots[s].hash && !(e->rt_slots[s].hash == h && e->rt_slots[s].len == len &&
                                             std::memcmp(&e->rt_arena[e->rt_slots[s].arena / 8], t, len) == 0))
                s = (s + 1) & mask;
            if (!e->rt_slots[s].hash || s != r.slot) return fail("probe of " + kv.first);
            const ExactSlot& x = e->rt_slots[s];
            if (x.count != r.dests.size() || x.dest_off != r.off || x.rank != r.label) return fail("slot of " + kv.first);
            if (len % 8 && (e->rt_arena[x.arena / 8 + len / 8] >> (8 * (len % 8))) != 0) return fail("arena padding");
            if (r.cap < r.dests.size() || (uint64_t)r.off + r.cap > e->rt_dest.size() ||
                !std::equal(r.dests.begin(), r.dests.end(), e->rt_dest.begin() + r.off))
                return fail("segment of " + kv.first);
            const bool wild = tm_topic_wildcard(t, len);
            const uint32_t fid = wild ? e->filter_of(t, len) : FILTER_NONE;
            if (r.fid != fid) return fail("filter link of " + kv.first);
            if (fid != FILTER_NONE) {
                const uint4 m = e->fr_meta[fid];
                if (m.x != r.off || m.y != r.dests.size() || m.z != r.label || e->fr_rec[fid] != &r)
                    return fail("fr_meta of " + kv.first);
            }
            if (r.label >= e->rank_src.size() || e->rank_src[r.label] != (fid != FILTER_NONE ? fid : TM_ROUTE_TOPIC_ID))
                return fail("rank_src of " + kv.first);
            if ((r.index != nullptr) != (r.dests.size() >= tm_engine::BAG_INDEX_MIN)) return fail("bag index");
        }
        if (total != e->route_total) return fail("route total");
        for (size_t f = 0; f < e->fr_meta.size(); ++f)
            if (e->fr_meta[f].y && (!e->fr_rec[f] || e->fr_rec[f]->fid != f)) return fail("stale fr_meta");
        if (e->rt_order.size() != e->route_bag.size()) return fail("order size");
        const tm_engine::RouteRec* prev = nullptr;
        for (const tm_engine::OrdKey& k : e->rt_order) {
            const tm_engine::RouteRec* r = k.r;
            if (k.label != r->label || r->ord->r != r) return fail("order entry of " + *r->key);
            if (prev && !(prev->label < r->label && *prev->key < *r->key)) return fail("label order at " + *r->key);
            prev = r;
        }
        return TM_OK;
    });
}

int tm_reserve(tm_engine* e, uint32_t n_topics, uint64_t n_bytes) {
    if (!e) return TM_EINVAL;
    auto held = lock_batches(e);
    return guarded(e, [&]() -> int {
        for (auto& dp : e->devs) {
            tm_engine::Guard g(dp->device);
            e->reserve(*dp, n_topics, n_bytes);
        }
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
        if (!std::strcmp(name, "light_tail")) {   // per mille of each range walked last by presort 6
            if (value < 0 || value > 500) return TM_EINVAL;
            e->light_tail = (uint32_t)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "relayout")) {   // 1: relayout at the next commit (layout A/Bs)
            if (value != 1) return TM_EINVAL;
            e->force_relayout = true;
            e->dev_dirty = true;
            return TM_OK;
        }
        if (!std::strcmp(name, "presort")) {   // 0 arrival order, 1 word-hash key, 2 the tail order, 3 auto
            if (value < 0 || value > 6) return TM_EINVAL;
            e->presort = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "host_pipeline")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->host_pipeline = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "sort_bits")) {
            if (value < 8 || value > 32 || value % 8) return TM_EINVAL;
            e->sort_bits = (uint32_t)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "sort_min")) {
            if (value < 0 || value > 0xffffffffll) return TM_EINVAL;
            e->sort_min = (uint32_t)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "route_gc")) {
            if (value < 0) return TM_EINVAL;
            e->route_gc_min = (size_t)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "double_buffer")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->double_buffer = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "summaries")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            if ((int)value != e->summaries) {
                e->summaries = (int)value;
                for (uint32_t v = 0; v < e->nodes.size(); ++v)
                    if (e->aux[v].parent != NODE_NONE || v == ROOT) {
                        e->refresh_hf(v);
                        e->refresh_slot_sum(v);
                    }
                e->dev_dirty = true;
            }
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
            e->stage_k_min = (uint32_t)value;
            for (auto& d : e->devs) {
                d->stage_k = d->keyed_k = (uint32_t)value;
                d->unkeyed_k = 0;
            }
            e->stage_auto = 0;   // an explicit K is kept (set "stage_auto" after it to grow from it)
            return TM_OK;
        }
        if (!std::strcmp(name, "slots")) {
            if (value < 1 || value > MAX_SLOTS) return TM_EINVAL;
            e->nslots = (int)value;
            for (auto& d : e->devs) d->next_slot = 0;
            return TM_OK;
        }
        if (!std::strcmp(name, "stage_auto")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->stage_auto = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "spill")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->spill_on = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "wave_walk_max")) {
            if (value < 0 || value > 0xFFFFFFFFll) return TM_EINVAL;
            e->wave_walk_max = (uint32_t)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "chunk_rows")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            e->chunk_rows = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "tok_wave")) {   // 1: wave-cooperative tokenizer, 0: one lane per topic
            if (value < 0 || value > 1) return TM_EINVAL;
            e->tok_wave = (int)value;
            return TM_OK;
        }
        if (!std::strcmp(name, "shape_keys")) {
            if (value < 0 || value > 1) return TM_EINVAL;
            if ((int)value != e->shape_keys) {
                e->shape_keys = (int)value;
                e->t_fshape.cur.all = true;   // both images take the whole table
                e->dev_dirty = true;
            }
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
    auto held = lock_batches(e);
    return guarded(e, [&]() -> int {
        // average per batch of each kernel stage over every batch recorded
        // since the previous call, over all replicas
        std::vector<const char*> order;
        std::vector<double> sum;
        std::vector<int> cnt;
        for (auto& dp : e->devs) {
            DevState& d = *dp;
            if (d.ev_pending.empty()) continue;
            tm_engine::Guard g(d.device);
            for (auto& t : d.ev_pending) {
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
                d.ev_pool.push_back(t);
            }
            d.ev_pending.clear();
        }
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
