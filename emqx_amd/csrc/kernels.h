// kernels.h — host-side declarations of the HIP launchers in kernels.hip.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>
#include "image.h"

namespace tmx {

constexpr uint32_t WREG = 16;        // topic levels kept in VGPRs / LDS path slots; longer
                                     // topics keep their path in global scratch
constexpr size_t QWS_BYTES = 3328;   // queue heads: 8 ranges x 128 B, 8 spill counters x 128 B, 8 XCD clocks x 128 B,
                                     // the batch's cost histogram
constexpr size_t QWS_MAXC = 120;     // u64 slot of ws: the batch's largest match count
constexpr size_t QWS_MAXL = 121;     // u64 slot of ws: most levels of a topic in a keyed batch
constexpr size_t QWS_SPILL = 128;    // u64 slots 128 + 16 x: spill chunks taken by XCD x's waves
// u64 slots 256 + 16 x (per-lane queue walks with XCD ranges; diagnostics,
// tm_debug_walk_clocks): wall clock of XCD x's first wave start (stored
// inverted: max of ~t), of its home range's first exhaustion (inverted), of
// its last wave's end, and the chunks its waves stole from other ranges
constexpr size_t QWS_CLOCK = 256;
// u64 slots 384 + c (presort 6): topics of predicted cost class c (kernels.hip
// tail_key), for the next batch's light-tail threshold
constexpr size_t QWS_CHIST = 384;
// Spill chunks (unkeyed walks): ids of a topic past its K-slot stage row go
// to chunks of SPILL_CHUNK u32 -- slot 0 the next chunk of the topic, slots
// 1.. ids in discovery order -- taken from the walking XCD's area (capacity
// spill_chunks / 8 chunks per XCD); spill_head[t] = the first chunk of a
// topic with more than K ids, or NO_SPILL when an area ran out (the
// copy-out then re-walks the topic, as keyed walks always do).  A narrow
// stage row keeps the walk's stage footprint (n x K x 4 B) small.
constexpr uint32_t SPILL_CHUNK = 128;
constexpr uint32_t NO_SPILL = 0xFFFFFFFFu;
constexpr size_t STATS_BYTES = 512;  // 8 totals + per-level diagnostic histogram

// per-batch device workspace of the queue pipeline
struct QueueBufs {
    uint32_t* twords;     // n x WREG word ids (levels < WREG)
    uint32_t* words;      // levels >= WREG of long topics, at (byte offset + topic index)
    uint32_t* meta;       // n: levels | long << 30 | dollar << 31
    uint32_t* path;       // global path of long topics, at (byte offset + 2 x topic index)
    uint32_t* stage;      // n x K: first K ids of each topic (written from the row's end)
    uint64_t* kstage;     // key_words planes of n x K order key words (sharded mode), or null
    bool shaped = false;  // keyed batch walked unkeyed: copy-out keys from ImageView::fshape (option "shape_keys")
    bool wave_walk = false;   // small batch: tm_walk_wave, one wave per topic level by level (option "wave_walk_max")
    int chunk_rows = 1;       // option "chunk_rows": 1 a taken chunk's rows staged in LDS, 0 each topic's row
                              // read from HBM when a lane takes it
    bool tok_wave = true;     // option "tok_wave": the wave-cooperative tokenizer (0: one lane per topic)
    uint64_t* scan_tmp;   // scan_tmp_elems(n)
    unsigned long long* ws;   // QWS_BYTES of queue heads
    uint32_t* perm;       // option "presort": queue position -> topic (n), or null (arrival order)
    uint32_t presort_mode = 1;   // 1: key of the first eight words; 2: the tail order (kernels.hip
                                 // tail_key: heavy topics first in each XCD range, one radix pass)
    uint32_t sort_passes = 4;    // mode 1: radix passes over the key's top 8 * sort_passes bits (1..4)
    uint32_t light_max = 31;     // mode 6: cost classes <= light_max are walked last in their XCD range
    // the radix passes of the batch's presort: the tokenizer writes the keys
    // and values where the first pass reads them, so the last ends in perm
    uint32_t presort_passes() const { return presort_mode == 2 ? 1u : presort_mode == 4 ? 2u : sort_passes; }
    // option "presort": the batch walked in the order of a 32-bit key of
    // its first eight words (each hashed, level-major: 6,5,5,4,4,3,3,2 bits),
    // so a wave's 64 lanes walk shared prefixes -- their loads of one node
    // are one request, and a prefix's nodes are hot in L2 while its topics
    // run.  An LSD radix sort of the key's top bits (presort.hip): 2n u32 keys
    // (the first n written by the tokenizer), n u32 values (ping-pong with
    // perm), presort_counts(n) u32 and
    // presort_counts(n) + 1 u64 offsets, scan_tmp_elems(presort_counts(n))
    // With chunk rows the walk reads each chunk's rows through perm; without,
    // it reads twords_s / meta_s (the rows gathered into walk order) and
    // writes stage row p for position p, and copy-out moves row p to topic
    // perm[p] (launch_copy: the perm of the batch's walk, or null).
    uint32_t* sort_keys = nullptr;
    uint32_t* sort_vals = nullptr;
    uint32_t* sort_counts = nullptr;
    uint64_t* sort_off = nullptr;
    uint64_t* sort_scan = nullptr;
    uint32_t* twords_s = nullptr;   // n x WREG
    uint32_t* meta_s = nullptr;     // n
    uint32_t* spill = nullptr;      // spill_chunks x SPILL_CHUNK (null: fan-out beyond K re-walks)
    uint32_t* spill_head = nullptr; // n
    uint32_t spill_chunks = 0;      // a multiple of 8
};
// digit counters of the presort of n topics (256 per 4096-topic tile)
uint32_t presort_counts(uint32_t n);
hipError_t launch_presort(const uint32_t* twords, const uint32_t* meta, uint32_t n, const QueueBufs& qb,
                          hipStream_t st, bool gather = true);
// true when launch_queue's walk of a presorted batch writes stage row p for
// queue position p (the copy-out then moves row p to topic perm[p]): without
// chunk rows, or keyed / stats walks.  With chunk rows the walk reads each
// chunk's rows through perm and writes stage rows, counts and spill heads by
// topic, so the ordinary copy-out (and spill) applies.
bool queue_rows_by_position(const QueueBufs& qb, bool stats_mode);

// tokenize -> NFA walk -> scan -> copy-out, all on st.  marks: 8 events,
// [2i] before / [2i+1] after stage i, or null.  out_cap == 0: counts and
// offsets only.  stats (6 x u64, zeroed by the caller) is filled when
// stats_mode: levels, visits, edge reads, matches, leaf visits, probe loads.
// qb.kstage != null: sharded mode, the order key of every id goes to out_keys
// (key_words u64 planes: word j of id p at out_keys[j * out_cap + p]; topics
// of up to 32 * key_words - 1 levels)
hipError_t launch_queue(bool stats_mode, bool xcdq, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, const QueueBufs& qb, uint32_t K, uint32_t* counts, uint64_t* out_off,
                        uint32_t* out, uint64_t* out_keys, uint64_t out_cap, uint64_t* total,
                        unsigned long long* stats, hipStream_t st, hipEvent_t* marks, uint32_t walk_blocks_per_cu = 0,
                        bool hist = false, uint32_t key_words = 1);
// tm_copy_out again over a finished launch_queue's workspace (qb, same n /
// K / key_words) into a larger output: no second walk
// a small batch in one launch (kernels.hip tm_match_small): lists placed in
// completion order, out_off[t] = topic t's start; ctl: two u64 the kernel
// leaves zeroed (zero them once when allocated)
hipError_t launch_small(const ImageView& im, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t* twords,
                        uint32_t* words, uint32_t* meta, uint32_t* gpath, uint32_t* counts, uint64_t* out_off,
                        uint32_t* out, uint64_t cap, uint64_t* total, unsigned long long* ctl, hipStream_t st);
hipError_t launch_copy(const ImageView& im, const uint8_t* bytes, const uint64_t* off, uint32_t n, const QueueBufs& qb,
                       uint32_t K, uint32_t key_words, const uint32_t* counts, const uint64_t* out_off, uint32_t* out,
                       uint64_t* out_keys, uint64_t out_cap, hipStream_t st);
size_t scan_tmp_elems(uint32_t n);
// split image (option "split"): n 32 B node records -> inner[n], leaf[n] 16 B halves
hipError_t launch_split_nodes(const void* nodes, uint64_t n, void* inner, void* leaf, hipStream_t st);
// element scatter of a commit packet [idx u32 x n][values: words u32 x n]
hipError_t launch_scatter(void* table, const uint32_t* pkt, uint64_t n, uint32_t words, hipStream_t st);
// exclusive scan of n u32 counts -> out_off[n+1] (u64), *total (tmp: scan_tmp_elems(n))
hipError_t launch_scan(const uint32_t* counts, uint32_t n, uint64_t* out_off, uint64_t* total, uint64_t* tmp,
                       hipStream_t st);

// emqx_router:match_routes/1 expansion (routes.hip) of a batch's ordered
// match lists: per topic its literal-topic routes, then each matched filter's
// routes.  exact: n uint2, rcount: n u32, tmp: scan_tmp_elems(n).  out_cap
// == 0: counts and offsets only.  av != null: also out_key[route] =
// to_rank << 32 | target rank (the aggre sort key).
hipError_t launch_routes(const RouteView& rv, const uint8_t* bytes, const uint64_t* off, uint32_t n,
                         const uint32_t* counts, const uint64_t* ids_off, const uint32_t* ids, uint4* exact,
                         uint32_t* rcount, uint64_t* out_off, uint32_t* out_src, uint32_t* out_dest,
                         uint64_t out_cap, uint64_t* total, uint64_t* scan_tmp, hipStream_t st,
                         const AggreView* av = nullptr, uint64_t* out_key = nullptr);

// emqx_broker:aggre/1 (aggre.hip) over a match_routes CSR (rcount, roff,
// src, dest, key from launch_routes with av; key rows of topics with > 4096
// group-prefix routes are sorted in place); large: n + 1 u32 (list of topics
// with > 512 routes).  Output at the route offsets: topic t's
// list is out_to / out_tg[roff[t] .. + acount[t]) (out_to = TM_ROUTE_TOPIC_ID
// or a filter id, out_tg = target id); entries at or past out_cap are dropped.
hipError_t launch_aggre(const AggreView& av, uint32_t n, const uint32_t* rcount, const uint64_t* roff,
                        const uint32_t* src, const uint32_t* dest, uint64_t* key, uint32_t* large, uint32_t* acount, uint32_t* out_to, uint32_t* out_tg, uint64_t out_cap,
                        hipStream_t st);

// Sharded mode (shard.hip): merge per-topic match lists of S filter shards
// for m topics.  counts [S][m]; source s's items start at src_base[s] of
// ids / keys and are CSR-ordered by topic, each list in descending key order.
// Output: counts[m], offsets[m+1], global ids (local * S + s) in descending
// key order = emqx_trie:match/1 order.  pre: S*m+1 u64, tmp: scan_tmp_elems(S*m).
// Keys of key_words words: word j of item g at keys[j * key_stride + g].
constexpr uint32_t MAX_SHARDS = 8;
hipError_t launch_shard_merge(uint32_t S, uint32_t m, const uint32_t* counts, const uint64_t* src_base,
                              const uint32_t* ids, const uint64_t* keys, uint32_t* out_count, uint64_t* out_off,
                              uint32_t* out_gid, uint64_t out_cap, uint64_t* total, uint64_t* pre, uint64_t* tmp,
                              hipStream_t st, uint32_t key_words = 1, uint64_t key_stride = 0);

// exchange bookkeeping (shard.hip): out[d] = ids of topic slice d of a CSR
// (offs[n+1]) cut S ways as b[d] = n*d/S, out[S+d] = the slice's first id;
// and per-source totals of a received [S][m] counts block
hipError_t launch_slice_sizes(const uint64_t* offs, uint32_t n, uint32_t S, uint64_t* out, hipStream_t st);
hipError_t launch_source_totals(const uint32_t* counts, uint32_t m, uint32_t S, uint64_t* out, hipStream_t st);

// Routed sharded mode (route.hip): each rank's batch into owner buckets.
// owner n u8, blk_cnt / blk_base ceil(n/256) x S u32, bucket S+1 u32 (topic
// base of each owner's bucket), perm / slen n u32, soff n+1 u64, scan_tmp
// scan_tmp_elems(n), sbuf the batch's bytes + 8, cuts S+1 u64 (byte base of
// each bucket).  The bucket order is stable (a source's topics keep their
// order within each owner's bucket).
constexpr uint32_t MAX_ROUTE_SHARDS = 64;
struct RoutePlanBufs {
    uint8_t* owner;
    uint32_t* blk_cnt;
    uint32_t* blk_base;
    uint32_t* bucket;
    uint32_t* perm;
    uint32_t* slen;
    uint64_t* soff;
    uint64_t* scan_tmp;
    uint8_t* sbuf;
    uint64_t* cuts;
};
hipError_t launch_route_plan(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t depth, uint32_t S,
                             const RoutePlanBufs& w, hipStream_t st);
// launch_scan, and for n = 0 out_off[0] = *total = 0
hipError_t launch_scan0(const uint32_t* counts, uint32_t n, uint64_t* out_off, uint64_t* total, uint64_t* tmp,
                        hipStream_t st);
// out[k] = in[idx[k]], k < count
hipError_t launch_gather_u64(const uint64_t* in, const uint32_t* idx, uint32_t k, uint64_t* out, hipStream_t st);
// lists returned in bucket order (rcount n, roff CSR, rids) -> the batch's own
// topic order: out_count[perm[p]] = rcount[p], out_off = scan, ids copied
hipError_t launch_route_unpermute(const uint32_t* rcount, const uint64_t* roff, const uint32_t* rids,
                                  const uint32_t* perm, uint32_t n, uint32_t* out_count, uint64_t* out_off,
                                  uint32_t* out_ids, uint64_t* total, uint64_t* scan_tmp, hipStream_t st);

}  // namespace tmx
