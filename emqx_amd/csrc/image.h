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
//   nodes[]  32 B per node (half an HBM burst): the '+' edge and the '#'
//            edge are ARRAY READS (fields of the parent), the filter ending at
//            the node and the filter ending at its '#' child are carried
//            inline, so the reference's 'match_#'/2 (emqx_trie.erl:140-145)
//            costs nothing beyond the node read; up to INLINE_LIT literal
//            children live in the record too, so the deep, narrow part of the
//            trie (most of the walk) needs no hash probe at all.
//   edges[]  literal edges of the wide nodes (> INLINE_LIT literal
//            children, flag LIT_TABLE), open addressing, 16 B slots grouped
//            in 64 B buckets (one HBM burst), linear probing over slots from
//            the home bucket's first slot, load <= 1/2.
//   dict[]   word dictionary: 64-bit hash -> word id, byte-verified against
//            the word arena, so tokenisation is collision-free (no hash-only
//            identity).
#pragma once
#include <stdint.h>

namespace tmx {

constexpr uint32_t ROOT       = 0u;
constexpr uint32_t NODE_MASK  = 0x1FFFFFFFu;   // node ids are 29-bit (walk path packs 3 flag bits)
constexpr uint32_t NODE_NONE  = 0x1FFFFFFFu;
constexpr uint32_t HAS_LIT    = 0x80000000u;   // nodes[].plus bit31: has literal children
constexpr uint32_t LIT_TABLE  = 0x40000000u;   // nodes[].plus bit30: they live in edges[] (else inline)
constexpr uint32_t PLUS_FLAGS = HAS_LIT | LIT_TABLE;
constexpr int      INLINE_LIT = 2;             // literal children kept in the node record
constexpr uint32_t FILTER_NONE = 0xFFFFFFFFu;

// token ids produced by the tokenizer (emqx_topic:words/1 + word/1)
constexpr uint32_t WORD_NONE  = 0xFFFFFFFFu;   // level bytes not in the dictionary
constexpr uint32_t WORD_PLUS  = 0xFFFFFFFEu;   // level == "+"  (atom '+')
constexpr uint32_t WORD_HASH  = 0xFFFFFFFDu;   // level == "#"  (atom '#')
constexpr uint32_t WORD_MAX   = 0xFFFFFFF0u;   // interned ids are < WORD_MAX

constexpr uint32_t EDGE_EMPTY = 0xFFFFFFFFu;   // slot.parent of an empty slot
constexpr int      SLOTS_PER_BUCKET = 4;       // 4 x 16 B = 64 B

struct alignas(32) Node {
    uint32_t plus;         // '+' child node id | HAS_LIT | LIT_TABLE, NODE_NONE if none
    uint32_t hash;         // '#' child node id, NODE_NONE if none
    uint32_t hash_filter;  // filter id of the '#' child (its topic), FILTER_NONE if none
    uint32_t self_filter;  // filter id ending at this node, FILTER_NONE if topic = undefined
    uint32_t lw[INLINE_LIT];  // inline literal children: word ids (WORD_NONE = empty slot)
    uint32_t lc[INLINE_LIT];  //   and child node ids; unused when LIT_TABLE is set
};

struct alignas(16) EdgeSlot {
    uint32_t parent;       // EDGE_EMPTY when free
    uint32_t word;
    uint32_t child;
    uint32_t pad;
};

struct alignas(16) DictSlot {
    uint64_t hash;         // 64-bit word hash (0 reserved for empty)
    uint32_t word;         // word id, WORD_NONE when free
    uint32_t len;          // word length in bytes
};

// device-side view of one committed image (plain pointers into HBM)
struct ImageView {
    const Node*     nodes;
    const EdgeSlot* edges;
    uint64_t        edge_slot_mask;    // slots - 1 (power of two)
    const DictSlot* dict;
    uint64_t        dict_slot_mask;
    const uint8_t*  word_arena;
    const uint32_t* word_off;          // word id -> arena offset
};

// ---- hashing (identical on host and device) ---------------------------------
#if defined(__HIPCC__)
#define TM_HD __host__ __device__ __forceinline__
#else
#define TM_HD inline
#endif

TM_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

TM_HD uint64_t edge_hash(uint32_t parent, uint32_t word) {
    return fmix64(((uint64_t)parent << 32) | word);
}

// first slot of the home bucket of key (parent, word)
TM_HD uint64_t edge_home(uint32_t parent, uint32_t word, uint64_t slot_mask) {
    return (edge_hash(parent, word) * SLOTS_PER_BUCKET) & slot_mask;
}

// word hash: 8-byte little-endian chunks folded with a multiply-xorshift; the
// value never decides identity (the dictionary verifies bytes), only placement.
TM_HD uint64_t word_hash_step(uint64_t h, uint64_t chunk) {
    h ^= chunk; h *= 0x9E3779B97F4A7C15ULL; h ^= h >> 29;
    return h;
}
TM_HD uint64_t word_hash_final(uint64_t h, uint32_t len) {
    h = fmix64(h ^ ((uint64_t)len * 0xD6E8FEB86659FD93ULL));
    return h ? h : 1;   // 0 marks an empty dict slot
}

}  // namespace tmx
