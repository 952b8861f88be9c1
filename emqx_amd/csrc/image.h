// image.h — layout of the subscription-trie image in HBM, shared by the host
// engine (which builds and patches it) and the HIP kernels (which walk it).
//
// The reference keeps the trie in two mnesia/ETS set tables
// (src/emqx_trie.erl:38-48, records include/emqx.hrl:93-110):
//   emqx_trie       {trie_edge{NodeIdBinary, Word}} -> ChildNodeIdBinary
//   emqx_trie_node  NodeIdBinary -> #trie_node{edge_count, topic}
// with node ids = full path binaries.  Here node ids are dense u32 and words
// are interned u32, so every probe is a fixed-size integer compare:
//
//   nodes[]  32 B per node in two 16 B halves, so every step of the walk is
//            ONE 16 B load: a visit with topic words left reads the inner
//            half {'+' child, '#' filter, one inline literal child (word,
//            child) or, for a WIDE node, a 64-bit Bloom mask of its literal
//            children's words that rejects most absent words without a probe},
//            a visit at the topic's last level reads the leaf half
//            {filter ending here, '#' filter}.  The '+' edge and the '#' edge
//            are fields of the parent, the filter ending at the '#' child is
//            carried inline (the reference's 'match_#'/2, emqx_trie.erl:140-145,
//            costs nothing beyond the visit's own load).
//   edges[]  literal edges of the wide nodes (>= 2 literal children, WIDE
//            flag) and the '#' children (word WORD_HASH, only looked up
//            for the out-of-domain topic level "#"): open addressing, 16 B
//            slots (key + child id; see TM_SLOT_RECORD), linear probing slot
//            by slot from the home slot, load <= 1/4.
//   dict[]   word dictionary: 64-bit hash -> word id, byte-verified against
//            the word arena, so tokenisation is collision-free (no hash-only
//            identity).
#pragma once
#include <stdint.h>

namespace tmx {

constexpr uint32_t ROOT       = 0u;
constexpr uint32_t NODE_MASK  = 0x1FFFFFFFu;   // node ids are 29-bit (walk path packs 3 flag bits)
constexpr uint32_t NODE_NONE  = 0x1FFFFFFFu;
constexpr uint32_t WIDE       = 0x80000000u;   // nodes[].plus bit 31: >= 2 literal children, all in
                                               // edges[]; lw:lc then hold a 64-bit Bloom mask of their words
constexpr uint32_t FILTER_NONE = 0xFFFFFFFFu;

// token ids produced by the tokenizer (emqx_topic:words/1 + word/1)
constexpr uint32_t WORD_NONE  = 0xFFFFFFFFu;   // level bytes not in the dictionary
constexpr uint32_t WORD_PLUS  = 0xFFFFFFFEu;   // level == "+"  (atom '+')
constexpr uint32_t WORD_HASH  = 0xFFFFFFFDu;   // level == "#"  (atom '#')
constexpr uint32_t WORD_MAX   = 0xFFFFFFF0u;   // interned ids are < WORD_MAX

constexpr uint32_t EDGE_EMPTY = 0xFFFFFFFFu;   // slot.parent of an empty slot

// Subtree summaries.  The 15-bit summary S(c) of the subtree below node c:
// bits 0-9 "a filter ends k levels below c" (k = 0..9), bit 10 "one ends 10
// or more below", bits 11-14 the fewest levels below c of a node whose '#'
// child holds a filter (15: none within 14).  A walk that reaches c with k
// topic levels still to consume (n - depth(c)) can match something below c
// only if sum_useful(S(c), k): a non-'#' filter must end exactly k below, a
// '#' filter fires at any visited node, i.e. within k.  Summaries are kept
// as supersets (inserts OR into them, deletes leave them, relayout rebuilds
// them exactly), so a prune is never wrong.
constexpr uint32_t SUM_TAG  = 0x80000000u;   // Node::hash_filter holds summaries, not a filter id
constexpr uint32_t SUM_ALL  = 0x7FFFu;       // summary that never prunes
constexpr uint32_t SUM_NONE = 15u << 11;     // empty subtree (no filter at all)

struct alignas(32) Node {
    // inner half: read by a visit with words left (level r < n)
    uint32_t plus;         // '+' child node id (NODE_NONE if none) | WIDE
    uint32_t hash_filter;  // filter id (< 2^31) of the '#' child (its topic), or, when there is none,
                           // SUM_TAG | S('+' child) | S(literal children, their union) << 15;
                           // FILTER_NONE (= SUM_TAG | all ones) never prunes
    uint32_t lw;           // narrow: word of the single literal child (WORD_NONE if none); WIDE: Bloom bits 0-31
    uint32_t lc;           // narrow: that child's node id; WIDE: Bloom bits 32-63
    // leaf half: read by a visit at the topic's last level (r == n)
    uint32_t self_filter;  // filter id ending at this node, FILTER_NONE if topic = undefined
    uint32_t hash_filter2; // = hash_filter
    uint32_t hash;         // '#' child node id, NODE_NONE if none
    uint32_t pad;
};
static_assert(sizeof(Node) == 32, "node record is two 16 B halves");

// Edge slot layout (build-time A/B, TM_SLOT_RECORD):
//   0: 16 B {parent, word, child, S(child)}: the probe finds the child id
//      and the child's own subtree summary (a child that cannot match below
//      is dropped), the child's visit loads its node half;
//   1: 32 B, second half {child.hash_filter, child.lw, child.lc,
//      child.self_filter}: the probe that finds the edge also delivers the
//      child's record (same 64 B sector), at twice the table footprint.
#ifndef TM_SLOT_RECORD
#define TM_SLOT_RECORD 0
#endif
constexpr bool SLOT_RECORD = TM_SLOT_RECORD != 0;
struct alignas(SLOT_RECORD ? 32 : 16) EdgeSlot {
    uint32_t parent;       // EDGE_EMPTY when free
    uint32_t word;
    uint32_t child;
    uint32_t plus;         // TM_SLOT_RECORD 0: S(child), the child's subtree summary; 1: child's record ...
#if TM_SLOT_RECORD
    uint32_t hash_filter;
    uint32_t lw;
    uint32_t lc;
    uint32_t self_filter;
#endif
};
static_assert(sizeof(EdgeSlot) == (SLOT_RECORD ? 32 : 16), "edge slot is one or two 16 B halves");

// Dictionary slot: the tokenizer's first 16 B load decides a word of <= 8
// bytes on its own (tag, id and the bytes), a word of 9-16 bytes with the
// second half (same 32 B, an L2 hit), a longer one against the arena.
struct alignas(32) DictSlot {
    uint32_t tag;          // dict_tag(hash, len): hash bits 63..40 | min(len, 255)
    uint32_t word;         // word id, WORD_NONE when free
    uint64_t head0;        // the word's bytes 0-7, zero padded
    uint64_t head1;        // bytes 8-15, zero padded
    uint32_t len;          // the exact length (read for words of 255 bytes or more)
    uint32_t pad;
};
static_assert(sizeof(DictSlot) == 32, "dictionary slot is one 32 B half line");


// device-side view of one committed image (plain pointers into HBM)
struct ImageView {
    const uint8_t*  inner;             // inner half of node v at inner + (v << node_shift)
    const uint8_t*  leaf;              // leaf half of node v at leaf + (v << node_shift)
    uint32_t        node_shift;        // 5: interleaved 32 B records; 4: split arrays of 16 B halves
    const EdgeSlot* edges;
    uint64_t        edge_slot_mask;    // slots - 1 (power of two)
    const EdgeSlot* hot_edges;         // edges of parents with id < hot_limit
    uint64_t        hot_slot_mask;
    uint32_t        hot_limit;
    const DictSlot* dict;
    uint64_t        dict_slot_mask;
    const uint8_t*  word_arena;
    const uint32_t* word_off;          // word id -> arena offset
    const uint64_t* fshape;            // filter id -> order key (filter_shape), or null (option "shape_keys" off)
    const uint8_t*  word_heat;         // word id -> floor(log2(1 + nodes it labels)) (presort mode 2)
    uint32_t        n_words;
};


// ---- route image (emqx_route bag, src/emqx_router.erl:52-59, 89-90) --------
// Routes are (topic, dest) pairs; dests are interned to u32 ids.  Each topic
// with routes owns a segment of one dest pool (bag insertion order).  The
// routes of a trie filter are found by its filter id (fr_meta: segment, count,
// to_rank); the routes of a literal topic (get_routes/1 of the publish topic
// itself) through an exact-topic hash table whose keys are verified byte for
// byte against the topic arena (8-aligned, zero padded).  The host patches
// all of it in place per add / del (engine.cpp, route image maintenance).
constexpr uint32_t TM_ROUTE_TOPIC_ID = 0xFFFFFFFFu;   // route source = the literal topic

struct alignas(32) ExactSlot {
    uint64_t hash;         // word_hash of the topic bytes (0 = empty slot)
    uint32_t len;          // topic length
    uint32_t count;        // routes of the topic
    uint64_t arena;        // topic bytes in the arena
    uint32_t dest_off;     // first route's dest in the dest pool
    uint32_t rank;         // to_rank of the topic (aggre)
};

struct RouteView {
    const uint4*     fr_meta;       // n_filters: {dest offset, count, to_rank, 0} (count 0: no routes)
    uint32_t         n_filters;
    const ExactSlot* ex_slots;      // power-of-two table, hash 0 = empty
    uint64_t         ex_slot_mask;
    const uint8_t*   ex_arena;
    const uint32_t*  dest;          // the dest pool
};

// emqx_broker:aggre/1 tables (aggre.hip): per dest id its aggre target.  A
// topic's to_rank (an order label: Erlang binary order of the topics with
// routes) rides in its fr_meta entry and its exact slot, which the route
// kernels fetch anyway.
struct AggreView {
    const uint2*    dt;             // dest id -> {target rank, target id | group << 31}
    const uint32_t* rank_src;       // to_rank -> route source of that To (filter id or TM_ROUTE_TOPIC_ID)
    const uint32_t* rank_tg;        // target rank -> target id
};

// ---- hashing (identical on host and device) ---------------------------------
#if defined(__HIPCC__)
#define TM_HD __host__ __device__ __forceinline__
#else
#define TM_HD inline
#endif

// The order key of filter f for any topic it matches (sharded mode; the
// walk's rank_sym keys, kernels.hip): per level i, '#' = 0, '+' = 2, a
// literal = 1 (it can only have matched the topic's own word), then the end
// mark 1 at position |f| unless f ends in '#' -- 2 bits per position from
// the top of a u64, positions < 32.  A topic (without literal '+' / '#'
// levels) has at most one matching filter per key, and its matches in
// descending key order are emqx_trie:match/1's order:
// the key is a property of the filter alone.
TM_HD uint64_t filter_shape(const uint32_t* ws, uint32_t len) {
    uint64_t k = 0;
    for (uint32_t i = 0; i < len && i < 32; ++i) {
        const uint64_t sym = ws[i] == 0xFFFFFFFDu ? 0u : ws[i] == 0xFFFFFFFEu ? 2u : 1u;   // WORD_HASH / WORD_PLUS
        k |= sym << (62 - 2 * i);
    }
    if ((len == 0 || ws[len - 1] != 0xFFFFFFFDu) && len < 32) k |= 1ull << (62 - 2 * len);
    return k;
}

// Routed sharded mode (topicmatch.h tm_route_of): the owner shard of a topic
// (or literal-led filter) from the word hash of its routing key (the bytes
// of its first `depth` levels), identical on host and device
TM_HD uint32_t route_shard(uint64_t key_hash, uint32_t n_shards) {
    return n_shards <= 1 ? 0u : (uint32_t)((key_hash >> 32) % n_shards);
}

// DictSlot::tag of a word: 24 hash bits and the length (capped at 255)
TM_HD uint32_t dict_tag(uint64_t h, uint32_t len) {
    return (uint32_t)(h >> 40) << 8 | (len < 255u ? len : 255u);
}

TM_HD bool sum_useful(uint32_t s, uint32_t k) {
    const uint32_t ends = k < 10 ? (s >> k) & 1u : (s >> 10) & 1u;
    return ends != 0 || ((s >> 11) & 15u) <= k;
}
TM_HD uint32_t sum_union(uint32_t a, uint32_t b) {
    const uint32_t ha = (a >> 11) & 15u, hb = (b >> 11) & 15u;
    return ((a | b) & 0x7FFu) | ((ha < hb ? ha : hb) << 11);
}
// S of a parent seen from one level up: every depth one more
TM_HD uint32_t sum_shift(uint32_t s) {
    const uint32_t ends = ((s & 0x3FFu) << 1) | (s & 0x600u ? 0x400u : 0u);   // bit 9 -> "10 or more"
    const uint32_t hm = (s >> 11) & 15u;
    return (ends & 0x7FEu) | ((hm < 15u ? hm + 1u : 15u) << 11);
}
// S of a subtree whose root ends a filter (k = 0), or fires a '#' filter
TM_HD uint32_t sum_end0() { return 1u | SUM_NONE; }
TM_HD uint32_t sum_hash0(uint32_t s) { return s & 0x7FFu; }   // hmin = 0

TM_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

TM_HD uint64_t edge_hash(uint32_t parent, uint32_t word) {
    return fmix64(((uint64_t)parent << 32) | word);
}

TM_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu;
    h ^= h >> 13; h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}

// Bloom bits of a literal word in a WIDE node's mask (2 of 64): two 6-bit
// fields of the word id's Fibonacci hash (one 32-bit multiply: the walk
// computes this at every WIDE node it visits, and 64-bit multiplies are
// several quarter-rate instructions each on CDNA)
#ifndef TM_HASH32
#define TM_HASH32 1   // A/B builds: 0 = the 64-bit mixes of round 2
#endif
TM_HD uint64_t word_bloom(uint32_t w) {
    if (!TM_HASH32) {
        const uint64_t h = fmix64(0x9E3779B97F4A7C15ULL ^ w);
        return (1ull << (h & 63)) | (1ull << ((h >> 6) & 63));
    }
    const uint32_t h = w * 0x9E3779B1u;
    return (1ull << (h >> 26)) | (1ull << ((h >> 20) & 63u));
}

// home slot of key (parent, word): a 32-bit mix (three 32-bit multiplies)
// for tables of up to 2^32 slots, the 64-bit one beyond
TM_HD uint64_t edge_home(uint32_t parent, uint32_t word, uint64_t slot_mask) {
    if (TM_HASH32 && slot_mask <= 0xFFFFFFFFull) return fmix32(parent * 0x9E3779B1u + word) & slot_mask;
    return edge_hash(parent, word) & slot_mask;
}

// word hash: 8-byte little-endian chunks folded with a multiply-xorshift; the
// value never decides identity (the dictionary verifies bytes), only placement.
// TM_WHASH32: the same with 32-bit multiplies only (two lanes of state,
// cross-mixed), for the VALU-bound tokenizer
#ifndef TM_WHASH32
#define TM_WHASH32 1
#endif
TM_HD uint64_t word_hash_step(uint64_t h, uint64_t chunk) {
    if (TM_WHASH32) {
        uint32_t a = ((uint32_t)h ^ (uint32_t)chunk) * 0x9E3779B1u;
        uint32_t b = ((uint32_t)(h >> 32) ^ (uint32_t)(chunk >> 32)) * 0x85EBCA77u;
        a ^= b >> 15;
        b ^= a >> 13;
        return ((uint64_t)b << 32) | a;
    }
    h ^= chunk; h *= 0x9E3779B97F4A7C15ULL; h ^= h >> 29;
    return h;
}
TM_HD uint64_t word_hash_final(uint64_t h, uint32_t len) {
    if (TM_WHASH32) {
        const uint32_t a = fmix32((uint32_t)h ^ (len * 0x27D4EB2Fu) ^ ((uint32_t)(h >> 32) * 0x165667B1u));
        const uint32_t b = fmix32((uint32_t)(h >> 32) ^ a);
        const uint64_t r = ((uint64_t)b << 32) | a;
        return r ? r : 1;
    }
    h = fmix64(h ^ ((uint64_t)len * 0xD6E8FEB86659FD93ULL));
    return h ? h : 1;   // 0 marks an empty dict slot
}

}  // namespace tmx
