// kernels.hip — CDNA4 (gfx950) kernels of the topic-routing hot path.
//
//   tm_match_fused  ONE launch per batch, one lane per topic:
//                   (1) emqx_topic:words/1 + word/1 (src/emqx_topic.erl:141-147):
//                       split on '/', hash each level, probe the word
//                       dictionary, byte-verify -> per-level word ids;
//                   (2) emqx_trie:match/1 (src/emqx_trie.erl:77-79, 121-145):
//                       walk the NFA over '+' / '#' / literal edges in the
//                       mirrored DFS order that IS the reference's output order
//                       (plus subtree, literal subtree, then the '#' filter; at
//                       the last level the self filter, then the '#' filter), so
//                       no sort is needed; matches are staged per lane;
//                   (3) CSR offsets by a decoupled look-back scan across
//                       workgroups (dynamic tile ids), then the staged ids are
//                       copied to their final place; lanes whose fan-out
//                       exceeded the stage re-walk and write straight through.
//   tm_tokenize / tm_match<MODE> / tm_scan_*
//                   the two-pass variant (count walk, scan, emit walk), kept for
//                   A/B measurement (TM_WALK=twopass).
//
// All integer/byte work: no MFMA.  The walk is latency-bound pointer chasing
// over the HBM image (image.h); the roofline is HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "image.h"
#include "kernels.h"

namespace tmx {

constexpr int BLOCK = 256;

// ---------------------------------------------------------------------------
// byte access: aligned 8-byte loads (an aligned word holding a valid byte
// never crosses a page), little-endian extraction.
__device__ __forceinline__ uint64_t load_u64_aligned(const uint8_t* base, uint64_t p) {
    return *reinterpret_cast<const uint64_t*>(base + (p & ~7ull));
}

// assemble up to 8 bytes [p, p+k) (k in 1..8) little-endian, zero padded
__device__ __forceinline__ uint64_t load_chunk(const uint8_t* base, uint64_t p, uint32_t k) {
    uint32_t sh = (uint32_t)(p & 7) * 8;
    uint64_t v = load_u64_aligned(base, p) >> sh;
    if (sh != 0 && (p & 7) + k > 8) v |= load_u64_aligned(base, p + 8) << (64 - sh);
    if (k < 8) v &= (~0ull) >> (64 - 8 * k);
    return v;
}

// dictionary lookup of topic bytes [p, p+len): word id, WORD_PLUS/HASH for the
// atoms '+' / '#', or WORD_NONE (bytes no filter contains: match only '+'/'#')
__device__ __forceinline__ uint32_t dict_lookup(const ImageView& im, const uint8_t* bytes,
                                                uint64_t p, uint32_t len) {
    if (len == 1) {
        uint32_t c = bytes[p];
        if (c == '+') return WORD_PLUS;
        if (c == '#') return WORD_HASH;
    }
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (uint32_t i = 0; i < len; i += 8) {
        uint32_t k = len - i < 8 ? len - i : 8;
        h = word_hash_step(h, load_chunk(bytes, p + i, k));
    }
    h = word_hash_final(h, len);
    uint64_t s = h & im.dict_slot_mask;
    for (;;) {
        DictSlot d = im.dict[s];
        if (d.word == WORD_NONE) return WORD_NONE;
        if (d.hash == h && d.len == len) {
            // byte-verify against the 8-aligned, zero-padded arena copy
            const uint64_t* a = reinterpret_cast<const uint64_t*>(im.word_arena + im.word_off[d.word]);
            bool eq = true;
            for (uint32_t i = 0; i < len && eq; i += 8) {
                uint32_t k = len - i < 8 ? len - i : 8;
                eq = (load_chunk(bytes, p + i, k) == a[i >> 3]);
            }
            if (eq) return d.word;
        }
        s = (s + 1) & im.dict_slot_mask;
    }
}

// emqx_topic:words/1 of topic [b, e): word ids to w[0..), returns n_levels
// (N slashes -> N+1 levels, empty levels kept)
__device__ __forceinline__ uint32_t tokenize_topic(const ImageView& im, const uint8_t* bytes, uint64_t b,
                                                   uint64_t e, uint32_t* w) {
    uint32_t lev = 0;
    uint64_t s = b;
    for (;;) {
        uint64_t q = s;  // next '/' at or after s, or e
        bool found = false;
        while (q < e) {
            uint64_t word8 = load_u64_aligned(bytes, q);
            uint32_t start = (uint32_t)(q & 7);
            uint64_t rem = e - (q & ~7ull);
            uint32_t stop = rem < 8 ? (uint32_t)rem : 8;
            uint64_t x = word8 ^ 0x2F2F2F2F2F2F2F2FULL;  // '/' -> 0x00
            uint64_t z = (x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL;
            z &= (~0ull) << (8 * start);
            if (stop < 8) z &= (~0ull) >> (64 - 8 * stop);
            if (z) {
                q = (q & ~7ull) + (__builtin_ctzll(z) >> 3);
                found = true;
                break;
            }
            q = (q & ~7ull) + 8;
        }
        if (!found) q = e;
        w[lev++] = dict_lookup(im, bytes, s, (uint32_t)(q - s));
        if (!found) return lev;
        s = q + 1;
    }
}

// ---------------------------------------------------------------------------
// literal edge (v, w): probing starts at a bucket boundary and advances one
// 64 B bucket (one HBM burst, 4 slots) per round
__device__ __forceinline__ uint32_t probe_edge(const ImageView& im, uint32_t v, uint32_t w) {
    uint64_t s = edge_home(v, w, im.edge_slot_mask);
    for (;;) {
        const uint4* b = reinterpret_cast<const uint4*>(im.edges + s);
        uint4 s0 = b[0], s1 = b[1], s2 = b[2], s3 = b[3];
        if (s0.x == v && s0.y == w) return s0.z;
        if (s0.x == EDGE_EMPTY) return NODE_NONE;
        if (s1.x == v && s1.y == w) return s1.z;
        if (s1.x == EDGE_EMPTY) return NODE_NONE;
        if (s2.x == v && s2.y == w) return s2.z;
        if (s2.x == EDGE_EMPTY) return NODE_NONE;
        if (s3.x == v && s3.y == w) return s3.z;
        if (s3.x == EDGE_EMPTY) return NODE_NONE;
        s = (s + SLOTS_PER_BUCKET) & im.edge_slot_mask;
    }
}

// inline literal child of a narrow node (no LIT_TABLE), NODE_NONE if absent
__device__ __forceinline__ uint32_t inline_child(const Node& rec, uint32_t w) {
    uint32_t c = NODE_NONE;
#pragma unroll
    for (int i = 0; i < INLINE_LIT; ++i) c = rec.lw[i] == w ? rec.lc[i] : c;
    return c;
}

// child of v by topic word w.  WORD_PLUS / WORD_HASH reproduce the reference
// for the out-of-domain topic levels "+" / "#": the fold over [W, '+'] at
// emqx_trie.erl:131-136 follows the '+' / '#' edge for them.
__device__ __forceinline__ uint32_t child_of(const ImageView& im, uint32_t v, const Node& rec, uint32_t w) {
    if (w >= WORD_MAX) {
        if (w == WORD_PLUS) return rec.plus & NODE_MASK;
        if (w == WORD_HASH) return rec.hash;
        return NODE_NONE;
    }
    if (!(rec.plus & HAS_LIT)) return NODE_NONE;
    if (!(rec.plus & LIT_TABLE)) return inline_child(rec, w);
    return probe_edge(im, v, w);
}

// ---------------------------------------------------------------------------
// The mirrored DFS.  path(r) = id | flags for the node on the current path
// at level r:  bits 31..30 phase (0 = first visit; 1 = literal branch next,
// probe the edge table; 3 = literal branch next, known: with bit 29 clear
// the stored id IS the pending literal child, with bit 29 set the node has a
// '#' filter too, so the id stays the node's and its record is re-read;
// 2 = both branches done), bit 29 = the node has a '#' filter to emit.  Output order equals emqx_trie:match/1 (which prepends
// every discovery to its accumulator, :127-145):
//   out(v, r<n) = out(plus(v)) ++ out(lit(v, w_r)) ++ [hash_filter(v)]
//   out(v, n)   = [self_filter(v), hash_filter(v)]
// A node record is read once per first visit; a narrow node without a '+'
// child descends into its inline literal child straight away; return visits
// need only the path word (plus a record re-read for a pending inline child
// or a '#' filter).
constexpr uint32_t P_NODE = NODE_MASK;
constexpr uint32_t P_HASH = 1u << 29;
constexpr uint32_t PH_PROBE = 1u, PH_DONE = 2u, PH_INLINE = 3u;

struct WalkStats {
    uint64_t visits = 0, edge_reads = 0;
};

struct Cursor {
    const uint32_t* w;
    uint32_t n, r, r0;
};

// '$' rule (emqx_trie.erl:121-122): a topic whose first word starts with '$'
// jumps straight to node <<W0>>, skipping root's '#' and '+' edges.
// Returns false when there is nothing to walk.
template <typename PathRef>
__device__ __forceinline__ bool walk_begin(const ImageView& im, Cursor& c, const uint32_t* w, uint32_t n,
                                           bool dollar, PathRef path) {
    uint32_t start = ROOT;
    c.w = w;
    c.n = n;
    c.r0 = 0;
    if (dollar) {
        Node root = im.nodes[ROOT];
        start = child_of(im, ROOT, root, w[0]);
        c.r0 = 1;
        if (start == NODE_NONE) return false;
    }
    c.r = c.r0;
    path(c.r) = start;
    return true;
}

// one step; true when the topic's walk is complete
template <bool STATS, typename PathRef, typename Emit>
__device__ __forceinline__ bool walk_step(const ImageView& im, Cursor& c, PathRef path, Emit& emit, WalkStats& st) {
    const uint32_t r = c.r;
    uint32_t e = path(r);
    const uint32_t v = e & P_NODE;
    uint32_t ph = e >> 30;
    uint32_t down = NODE_NONE;
    bool leaf = false;
    if (ph == 0) {
        Node rec = im.nodes[v];
        if (STATS) {
            ++st.visits;
            st.edge_reads += (r == c.n) ? 1 : 3;  // 'match_#' + fold over [W, '+'] (:132, :141)
        }
        if (r == c.n) {
            if (rec.self_filter != FILTER_NONE) emit(rec.self_filter);
            if (rec.hash_filter != FILTER_NONE) emit(rec.hash_filter);
            leaf = true;
        } else {
            const uint32_t wr = c.w[r];
            const uint32_t hb = rec.hash_filter != FILTER_NONE ? P_HASH : 0u;
            uint32_t lit_ph = PH_DONE, lc = NODE_NONE;
            if (wr >= WORD_MAX) {
                lc = child_of(im, v, rec, wr);
                lit_ph = lc != NODE_NONE ? PH_INLINE : PH_DONE;
            } else if (rec.plus & HAS_LIT) {
                if (rec.plus & LIT_TABLE) {
                    lit_ph = PH_PROBE;
                } else {
                    lc = inline_child(rec, wr);
                    lit_ph = lc != NODE_NONE ? PH_INLINE : PH_DONE;
                }
            }
            const uint32_t pc = rec.plus & NODE_MASK;
            if (pc != NODE_NONE) {
                // park the pending literal child in the path word when the
                // node has no '#' filter (no record re-read on return)
                path(r) = (lit_ph == PH_INLINE && !hb) ? (lc | (PH_INLINE << 30)) : (v | hb | (lit_ph << 30));
                down = pc;
            } else if (lit_ph == PH_INLINE) {
                path(r) = v | hb | (PH_DONE << 30);
                down = lc;
            } else if (lit_ph == PH_PROBE) {
                e = v | hb;
                ph = PH_PROBE;
            } else {
                if (hb) emit(rec.hash_filter);
                leaf = true;
            }
        }
    }
    if (down == NODE_NONE && !leaf) {
        if (ph == PH_PROBE || ph == PH_INLINE) {
            const uint32_t wr = c.w[r];
            uint32_t lc;
            if (ph == PH_PROBE) {
                lc = probe_edge(im, v, wr);
            } else if (!(e & P_HASH)) {
                lc = v;   // parked literal child
            } else {
                Node rec = im.nodes[v];
                lc = child_of(im, v, rec, wr);
            }
            e = (e & ~(3u << 30)) | (PH_DONE << 30);
            path(r) = e;
            down = lc;
        }
        if (down == NODE_NONE && (e & P_HASH)) emit(im.nodes[v].hash_filter);
    }
    if (down != NODE_NONE) {
        path(r + 1) = down;
        c.r = r + 1;
        return false;
    }
    if (r == c.r0) return true;
    c.r = r - 1;
    return false;
}

template <bool STATS, typename PathRef, typename Emit>
__device__ __forceinline__ void walk(const ImageView& im, const uint32_t* __restrict__ w, uint32_t n,
                                     bool dollar, PathRef path, Emit& emit, WalkStats& st) {
    Cursor c;
    if (!walk_begin(im, c, w, n, dollar, path)) return;
    while (!walk_step<STATS>(im, c, path, emit, st)) {
    }
}

constexpr uint32_t LDS_LEVELS = 20;   // topics with n < 20 keep their path in LDS

struct LdsPath {
    uint32_t* base;   // [level][BLOCK]
    __device__ __forceinline__ uint32_t& operator()(uint32_t r) const { return base[r * BLOCK]; }
};
struct GlobalPath {
    uint32_t* base;
    __device__ __forceinline__ uint32_t& operator()(uint32_t r) const { return base[r]; }
};

struct CountEmit {
    uint32_t cnt = 0;
    __device__ __forceinline__ void operator()(uint32_t) { ++cnt; }
};
// writes the ids at out[base + k] for skip <= k (and base + k < cap)
struct DirectEmit {
    uint32_t* out;
    uint64_t base, cap;
    uint32_t skip, cnt;
    __device__ __forceinline__ void operator()(uint32_t f) {
        if (cnt >= skip && base + cnt < cap) out[base + cnt] = f;
        ++cnt;
    }
};
// first K ids of a lane go to its stage column (stride BLOCK)
struct StageEmit {
    uint32_t* col;
    uint32_t K, cnt;
    __device__ __forceinline__ void operator()(uint32_t f) {
        if (cnt < K) col[(uint64_t)cnt * BLOCK] = f;
        ++cnt;
    }
};

template <bool STATS>
__device__ __forceinline__ void wave_stats_add(unsigned long long* stats, uint64_t a, uint64_t b, uint64_t c,
                                               uint64_t d) {
    if (!STATS) return;
    uint64_t v[4] = {a, b, c, d};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint64_t x = v[k];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(stats + k, (unsigned long long)x);
    }
}

// ---------------------------------------------------------------------------
// block scan helper (u64, BLOCK threads)
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t x, uint64_t* lds, uint64_t& total) {
    int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t inc = x;
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    uint64_t wpre = 0, tot = 0;
    for (int i = 0; i < BLOCK / 64; ++i) {
        if (i < wid) wpre += lds[i];
        tot += lds[i];
    }
    __syncthreads();
    total = tot;
    return wpre + inc - x;
}

// ---------------------------------------------------------------------------
// decoupled look-back.  status[tile] is ONE 8-byte word = {flag:2, value:62}
// (the data is the flag, so no separate payload needs ordering), written and
// polled with device-scope atomic RMWs that complete at the memory side, so
// visibility never depends on which XCD's L2 the tiles ran on.
constexpr uint64_t ST_AGG = 1ull << 62, ST_INC = 2ull << 62, ST_VAL = ST_AGG - 1;
constexpr uint32_t LOOKBACK_SPIN_LIMIT = 1u << 24;

__device__ __forceinline__ void st_publish(unsigned long long* status, uint32_t tile, uint64_t word) {
    __hip_atomic_exchange(status + tile, (unsigned long long)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// run by one full wave; returns the exclusive prefix of `tile`
__device__ __forceinline__ uint64_t look_back(unsigned long long* status, uint32_t tile, uint32_t* err) {
    int lane = threadIdx.x & 63;
    uint64_t excl = 0;
    int64_t p = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (p >= 0) {
        int64_t q = p - lane;
        uint64_t s = ST_INC;  // before tile 0: inclusive 0
        if (q >= 0)
            s = __hip_atomic_fetch_or(status + q, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!__all((s >> 62) != 0)) {
            if (++spins > LOOKBACK_SPIN_LIMIT) {  // never expected: flag it, do not hang the GPU
                if (lane == 0) atomicOr(err, 1u);
                return excl;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        uint64_t inc_mask = __ballot((s >> 62) == 2);
        int first = inc_mask ? (__ffsll((long long)inc_mask) - 1) : 64;
        uint64_t v = (lane <= first) ? (s & ST_VAL) : 0;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (first < 64) break;
        p -= 64;
    }
    return excl;
}

// ---------------------------------------------------------------------------
// the fused kernel.  Persistent workgroups pull tiles of TILE topics from a
// counter (ws[0]); every predecessor in the look-back chain therefore holds a
// tile already and runs, so progress never depends on co-residency.
// Per tile:
//   A  tokenize the tile's topics (uniform work, TILE / BLOCK per lane)
//   B  walk: lanes pull topics from an LDS queue (wave-aggregated atomics) and
//      step their own DFS; a lane that finishes takes the next topic, so no
//      lane idles behind the wave's slowest topic.  The first K ids of a
//      topic go to its contiguous stage row.
//   C  topics of >= LDS_LEVELS levels (path in global scratch), strided
//   D  block scan of the counts + decoupled look-back -> tile base offset
//   E  counts / offsets out, coalesced copy of the staged ids (binary search
//      of the output index in the tile's prefix), re-walk of topics whose
//      fan-out exceeded K, written straight through.
// ws layout (zeroed per launch): ws[0] tile counter, ws[1] error word,
// ws[2 ..] one status word per tile.
constexpr uint32_t TILE_MAX = 1024;
constexpr uint32_t META_LONG = 1u << 30, META_DOLLAR = 1u << 31, META_N = (1u << 30) - 1;
constexpr uint32_t NO_TOPIC = 0xFFFFFFFFu;

struct RowEmit {   // first K ids of a topic to its contiguous stage row (K % 4 == 0, row 16 B aligned)
    uint32_t* row;
    uint32_t K, cnt;
    uint4 buf;         // ids staged 4 at a time: one 16 B store per 4 ids
    __device__ __forceinline__ void operator()(uint32_t f) {
        const uint32_t j = cnt & 3u;
        buf.x = j == 0 ? f : buf.x;
        buf.y = j == 1 ? f : buf.y;
        buf.z = j == 2 ? f : buf.z;
        buf.w = j == 3 ? f : buf.w;
        if (j == 3 && cnt < K) *reinterpret_cast<uint4*>(row + (cnt - 3)) = buf;
        ++cnt;
    }
    __device__ __forceinline__ void flush() {   // the last 1..3 ids
        const uint32_t j = cnt & 3u, b = cnt - j;
        if (b >= K) return;
        if (j > 0) row[b] = buf.x;
        if (j > 1) row[b + 1] = buf.y;
        if (j > 2) row[b + 2] = buf.z;
    }
};

template <bool STATS, uint32_t TILE>
__global__ void __launch_bounds__(BLOCK)
tm_match_fused(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
               uint32_t n, uint32_t* __restrict__ words, uint32_t* __restrict__ path_scratch,
               uint32_t* __restrict__ stage, uint32_t K, uint32_t* __restrict__ counts,
               uint64_t* __restrict__ out_off, uint32_t* __restrict__ out, uint64_t out_cap,
               uint64_t* __restrict__ total, unsigned long long* __restrict__ ws,
               unsigned long long* __restrict__ stats) {
    __shared__ uint32_t lds_path[LDS_LEVELS * BLOCK];
    __shared__ uint32_t lds_meta[TILE];   // n_levels | long | dollar
    __shared__ uint32_t lds_inc[TILE];    // counts, then inclusive prefix within the tile
    __shared__ uint64_t lds_scan[BLOCK / 64];
    __shared__ uint64_t lds_base;
    __shared__ uint32_t lds_tile, lds_next;

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t n_tiles = (n + TILE - 1) / TILE;
    const uint64_t o0 = off[0];
    unsigned long long* status = ws + 2;
    WalkStats st;
    uint64_t levels_sum = 0, match_sum = 0;
    LdsPath lpath{lds_path + threadIdx.x};

    for (;;) {
        if (threadIdx.x == 0) {
            lds_tile = (uint32_t)__hip_atomic_fetch_add(ws, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds_next = 0;
        }
        __syncthreads();
        const uint32_t tile = lds_tile;
        if (tile >= n_tiles) break;
        const uint32_t t0 = tile * TILE;
        const uint32_t tn = n - t0 < TILE ? n - t0 : TILE;
        uint32_t* stage_tile = stage + (uint64_t)tile * TILE * K;

        // ---- A: tokenize
        for (uint32_t i = threadIdx.x; i < TILE; i += BLOCK) lds_inc[i] = 0;
        for (uint32_t i = threadIdx.x; i < tn; i += BLOCK) {
            uint64_t tb = off[t0 + i], te = off[t0 + i + 1];
            uint32_t nl = tokenize_topic(im, bytes, tb, te, words + (tb - o0) + t0 + i);
            levels_sum += nl;
            lds_meta[i] = nl | (nl >= LDS_LEVELS ? META_LONG : 0u) | ((te > tb && bytes[tb] == '$') ? META_DOLLAR : 0u);
        }
        __syncthreads();

        // ---- B: dynamic walk of the short topics
        {
            uint32_t my = NO_TOPIC;
            Cursor cur;
            RowEmit em{nullptr, K, 0, make_uint4(0, 0, 0, 0)};
            bool drained = false;
            for (;;) {
                bool need = (my == NO_TOPIC) && !drained;
                uint64_t m = __ballot(need);
                if (m) {
                    uint32_t leader = __ffsll((long long)m) - 1;
                    uint32_t basei = 0;
                    if (lane == leader) basei = atomicAdd(&lds_next, (uint32_t)__popcll(m));
                    basei = __shfl(basei, leader, 64);
                    if (need) {
                        uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        uint32_t i = basei + rank;
                        if (i >= tn) {
                            drained = true;
                        } else {
                            uint32_t meta = lds_meta[i];
                            if (!(meta & META_LONG)) {
                                uint32_t t = t0 + i;
                                em.row = stage_tile + (uint64_t)i * K;
                                em.cnt = 0;
                                if (walk_begin(im, cur, words + (off[t] - o0) + t, meta & META_N,
                                               (meta & META_DOLLAR) != 0, lpath))
                                    my = i;
                            }
                        }
                    }
                }
                if (__all(my == NO_TOPIC && drained)) break;
                if (my == NO_TOPIC) continue;
                if (walk_step<STATS>(im, cur, lpath, em, st)) {
                    em.flush();
                    lds_inc[my] = em.cnt;
                    my = NO_TOPIC;
                }
            }
        }

        // ---- C: long topics (path in global scratch)
        for (uint32_t i = threadIdx.x; i < tn; i += BLOCK) {
            uint32_t meta = lds_meta[i];
            if (!(meta & META_LONG)) continue;
            uint32_t t = t0 + i;
            uint64_t b = off[t] - o0;
            RowEmit em{stage_tile + (uint64_t)i * K, K, 0, make_uint4(0, 0, 0, 0)};
            walk<STATS>(im, words + b + t, meta & META_N, (meta & META_DOLLAR) != 0,
                        GlobalPath{path_scratch + b + 2ull * t}, em, st);
            em.flush();
            lds_inc[i] = em.cnt;
        }
        __syncthreads();

        // ---- D: tile scan (4 consecutive topics per lane) + look-back
        constexpr uint32_t PER = TILE / BLOCK;
        uint32_t c4[PER];
        uint64_t s4 = 0;
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            c4[j] = lds_inc[threadIdx.x * PER + j];
            s4 += c4[j];
        }
        match_sum += s4;
        uint64_t agg;
        uint64_t ex = block_exclusive_scan(s4, lds_scan, agg);
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) {
            ex += c4[j];
            lds_inc[threadIdx.x * PER + j] = (uint32_t)ex;   // inclusive, tile-local
        }
        if (threadIdx.x == 0) st_publish(status, tile, (tile == 0 ? ST_INC : ST_AGG) | agg);
        if (threadIdx.x < 64) {
            uint64_t excl = tile == 0 ? 0 : look_back(status, tile, reinterpret_cast<uint32_t*>(ws + 1));
            if (threadIdx.x == 0) {
                if (tile != 0) st_publish(status, tile, ST_INC | (excl + agg));
                lds_base = excl;
            }
        }
        __syncthreads();
        const uint64_t base = lds_base;

        // ---- E: offsets, coalesced copy-out, overflow re-walks
        for (uint32_t i = threadIdx.x; i < tn; i += BLOCK) {
            uint32_t inc = lds_inc[i], exc = i ? lds_inc[i - 1] : 0;
            counts[t0 + i] = inc - exc;
            out_off[t0 + i] = base + exc;
        }
        for (uint64_t j = threadIdx.x; j < agg; j += BLOCK) {
            // first topic q with inclusive prefix > j
            uint32_t lo = 0, hi = tn - 1;
            while (lo < hi) {
                uint32_t mid = (lo + hi) >> 1;
                if ((uint64_t)lds_inc[mid] > j) hi = mid; else lo = mid + 1;
            }
            uint32_t k = (uint32_t)(j - (lo ? lds_inc[lo - 1] : 0));
            if (k < K && base + j < out_cap) out[base + j] = stage_tile[(uint64_t)lo * K + k];
        }
        for (uint32_t i = threadIdx.x; i < tn; i += BLOCK) {
            uint32_t exc = i ? lds_inc[i - 1] : 0, c = lds_inc[i] - exc;
            if (c <= K) continue;
            uint32_t meta = lds_meta[i];
            uint32_t t = t0 + i;
            uint64_t b = off[t] - o0;
            DirectEmit em{out, base + exc, out_cap, K, 0};
            WalkStats s2;
            if (meta & META_LONG)
                walk<false>(im, words + b + t, meta & META_N, (meta & META_DOLLAR) != 0,
                            GlobalPath{path_scratch + b + 2ull * t}, em, s2);
            else
                walk<false>(im, words + b + t, meta & META_N, (meta & META_DOLLAR) != 0, lpath, em, s2);
        }
        if (t0 + tn == n && threadIdx.x == 0) {
            out_off[n] = base + agg;
            *total = base + agg;
        }
        __syncthreads();
    }
    wave_stats_add<STATS>(stats, levels_sum, st.visits, st.edge_reads, match_sum);
}

// ---------------------------------------------------------------------------
// variant "lane" (A/B): one topic per lane, grid = ceil(n / BLOCK), the tile
// a workgroup processes is drawn from a counter so every predecessor in the
// look-back chain is already running.  Stage in columns [k][BLOCK].
// ws layout (zeroed per launch): ws[0] tile counter, ws[1] error word,
// ws[2 ..] one status word per tile.
template <bool STATS>
__global__ void __launch_bounds__(BLOCK)
tm_match_lane(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
               uint32_t n, uint32_t* __restrict__ words, uint32_t* __restrict__ path_scratch,
               uint32_t* __restrict__ stage, uint32_t K, uint32_t* __restrict__ counts,
               uint64_t* __restrict__ out_off, uint32_t* __restrict__ out, uint64_t out_cap,
               uint64_t* __restrict__ total, unsigned long long* __restrict__ ws,
               unsigned long long* __restrict__ stats) {
    __shared__ uint32_t lds_path[LDS_LEVELS * BLOCK];
    __shared__ uint64_t lds_scan[BLOCK / 64];
    __shared__ uint64_t lds_base;
    __shared__ uint32_t lds_tile;
    if (threadIdx.x == 0)
        lds_tile = (uint32_t)__hip_atomic_fetch_add(ws, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t tile = lds_tile;
    const uint32_t t = tile * BLOCK + threadIdx.x;
    unsigned long long* status = ws + 2;

    WalkStats st;
    uint32_t cnt = 0, nlev = 0;
    uint64_t b = 0;
    const uint32_t* wv = nullptr;
    bool dollar = false;
    uint32_t* col = stage + (uint64_t)tile * K * BLOCK + threadIdx.x;
    if (t < n) {
        uint64_t tb = off[t], te = off[t + 1];
        b = tb - off[0];
        uint32_t* w = words + b + t;
        nlev = tokenize_topic(im, bytes, tb, te, w);
        dollar = (te > tb) && bytes[tb] == '$';
        wv = w;
        StageEmit em{col, K, 0};
        if (nlev < LDS_LEVELS) {
            walk<STATS>(im, wv, nlev, dollar, LdsPath{lds_path + threadIdx.x}, em, st);
        } else {
            walk<STATS>(im, wv, nlev, dollar, GlobalPath{path_scratch + b + 2ull * t}, em, st);
        }
        cnt = em.cnt;
    }
    wave_stats_add<STATS>(stats, nlev, st.visits, st.edge_reads, cnt);

    // CSR offsets: block scan + decoupled look-back
    uint64_t agg;
    uint64_t pre = block_exclusive_scan(cnt, lds_scan, agg);
    if (threadIdx.x == 0) st_publish(status, tile, (tile == 0 ? ST_INC : ST_AGG) | agg);
    if (threadIdx.x < 64) {
        uint64_t excl = tile == 0 ? 0 : look_back(status, tile, reinterpret_cast<uint32_t*>(ws + 1));
        if (threadIdx.x == 0) {
            if (tile != 0) st_publish(status, tile, ST_INC | (excl + agg));
            lds_base = excl;
        }
    }
    __syncthreads();
    const uint64_t base = lds_base + pre;
    if (t < n) {
        counts[t] = cnt;
        out_off[t] = base;
        uint32_t k1 = cnt < K ? cnt : K;
        for (uint32_t k = 0; k < k1; ++k)
            if (base + k < out_cap) out[base + k] = col[(uint64_t)k * BLOCK];
        if (cnt > K) {  // fan-out beyond the stage: walk again, write the tail in place
            DirectEmit em{out, base, out_cap, K, 0};
            WalkStats s2;
            if (nlev < LDS_LEVELS) {
                walk<false>(im, wv, nlev, dollar, LdsPath{lds_path + threadIdx.x}, em, s2);
            } else {
                walk<false>(im, wv, nlev, dollar, GlobalPath{path_scratch + b + 2ull * t}, em, s2);
            }
        }
        if (t == n - 1) {
            out_off[n] = base + cnt;
            *total = base + cnt;
        }
    }
}

// ---------------------------------------------------------------------------
// two-pass variant (A/B): tokenize, count walk, scan, emit walk

constexpr uint32_t MLONG_T = 1u << 30;   // meta: n_levels | long << 30 | dollar << 31

__global__ void __launch_bounds__(BLOCK)
tm_tokenize(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
            uint32_t n, uint32_t* __restrict__ words, uint32_t* __restrict__ meta) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t b = off[t], e = off[t + 1];
    uint32_t lev = tokenize_topic(im, bytes, b, e, words + (b - off[0]) + t);
    uint32_t dollar = (e > b && bytes[b] == '$') ? 1u : 0u;
    meta[t] = lev | (dollar << 31) | (lev >= LDS_LEVELS ? MLONG_T : 0u);
}

template <int MODE, bool LONG>
__global__ void __launch_bounds__(BLOCK)
tm_match(ImageView im, const uint64_t* __restrict__ off, uint32_t n_topics,
         const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta,
         uint32_t* __restrict__ counts, const uint64_t* __restrict__ out_off,
         uint32_t* __restrict__ out, uint64_t out_cap, uint32_t* __restrict__ path_scratch,
         unsigned long long* __restrict__ stats) {
    __shared__ uint32_t lds_path[LONG ? 1 : LDS_LEVELS * BLOCK];
    constexpr bool STATS = MODE == TM_MODE_STATS;
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    WalkStats st;
    uint32_t cnt = 0, nlev = 0;
    if (t < n_topics) {
        uint32_t m = meta[t];
        nlev = m & 0x3FFFFFFFu;
        bool dollar = (m >> 31) != 0;
        bool is_long = nlev >= LDS_LEVELS;
        if (is_long == LONG) {
            uint64_t b = off[t] - off[0];
            const uint32_t* w = words + b + t;
            if (MODE == TM_MODE_EMIT) {
                DirectEmit em{out, out_off[t], out_cap, 0, 0};
                if (LONG) walk<false>(im, w, nlev, dollar, GlobalPath{path_scratch + b + 2ull * t}, em, st);
                else walk<false>(im, w, nlev, dollar, LdsPath{lds_path + threadIdx.x}, em, st);
                cnt = em.cnt;
            } else {
                CountEmit em;
                if (LONG) walk<STATS>(im, w, nlev, dollar, GlobalPath{path_scratch + b + 2ull * t}, em, st);
                else walk<STATS>(im, w, nlev, dollar, LdsPath{lds_path + threadIdx.x}, em, st);
                cnt = em.cnt;
                counts[t] = cnt;
            }
        } else {
            nlev = 0;  // accounted by the other instantiation
        }
    }
    wave_stats_add<STATS>(stats, nlev, st.visits, st.edge_reads, cnt);
}

// ---------------------------------------------------------------------------
// variant "queue": topic-granular global load balancing.
//   tm_tokenize            words + meta of every topic (shared with two-pass)
//   tm_walk_queue<STATS>   persistent waves take topic ranges of QCHUNK from one
//                          global counter; each lane takes the next topic of its
//                          wave's range the moment its walk ends, so no lane or
//                          wave idles behind a heavy topic; writes counts[t] and
//                          the first K ids of topic t to stage row t
//   tm_scan_*              counts -> CSR offsets
//   tm_copy_out            per 256 topics: coalesced stage -> CSR copy (output
//                          index -> topic by binary search of the block's
//                          prefix), re-walk of topics with count > K
constexpr uint32_t QCHUNK = 64;
constexpr uint32_t MLONG = 1u << 30, MDOLLAR = 1u << 31, MN = (1u << 30) - 1;

template <bool STATS>
__global__ void __launch_bounds__(BLOCK)
tm_walk_queue(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ words,
              const uint32_t* __restrict__ meta, uint32_t* __restrict__ path_scratch, uint32_t* __restrict__ stage,
              uint32_t K, uint32_t* __restrict__ counts, unsigned long long* __restrict__ ws,
              unsigned long long* __restrict__ stats) {
    __shared__ uint32_t lds_path[LDS_LEVELS * BLOCK];
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t o0 = off[0];
    const LdsPath lp{lds_path + threadIdx.x};
    GlobalPath gp{nullptr};
    uint32_t qnext = 0, qend = 0;      // this wave's current range (uniform)
    bool exhausted = false;            // global counter ran past n (uniform)
    uint32_t my = NO_TOPIC;
    bool is_long = false, drained = false;
    Cursor cur;
    RowEmit em{nullptr, K, 0, make_uint4(0, 0, 0, 0)};
    WalkStats st;
    uint64_t lev_sum = 0, match_sum = 0;
    for (;;) {
        const bool need = (my == NO_TOPIC) && !drained;
        const uint64_t m = __ballot(need);
        if (m) {
            const uint32_t cm = (uint32_t)__popcll(m);
            const uint32_t avail = qend - qnext;
            uint32_t g = 0xFFFFFFFFu;
            if (avail < cm && !exhausted) {
                uint32_t x = 0;
                if (lane == (uint32_t)(__ffsll((long long)m) - 1))
                    x = (uint32_t)__hip_atomic_fetch_add(ws, (unsigned long long)QCHUNK, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                g = __shfl(x, __ffsll((long long)m) - 1, 64);
                if (g >= n) exhausted = true;
            }
            if (need) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                uint32_t i = NO_TOPIC;
                if (rank < avail) i = qnext + rank;
                else if (g != 0xFFFFFFFFu && g < n) i = g + (rank - avail);
                if (i >= n) {
                    drained = true;
                } else {
                    const uint32_t mt = meta[i];
                    const uint32_t nl = mt & MN;
                    lev_sum += nl;
                    is_long = (mt & MLONG) != 0;
                    const uint64_t b = off[i] - o0;
                    em.row = stage + (uint64_t)i * K;
                    em.cnt = 0;
                    bool go;
                    if (is_long) {
                        gp.base = path_scratch + b + 2ull * i;
                        go = walk_begin(im, cur, words + b + i, nl, (mt & MDOLLAR) != 0, gp);
                    } else {
                        go = walk_begin(im, cur, words + b + i, nl, (mt & MDOLLAR) != 0, lp);
                    }
                    if (go) my = i;
                    else counts[i] = 0;
                }
            }
            // advance the wave's range (uniform)
            if (avail >= cm) {
                qnext += cm;
            } else if (g != 0xFFFFFFFFu && g < n) {
                qnext = g + (cm - avail);
                qend = g + QCHUNK < n ? g + QCHUNK : n;
                if (qnext > qend) qnext = qend;
            } else {
                qnext = qend;
            }
        }
        if (__all(my == NO_TOPIC && drained)) break;
        if (my == NO_TOPIC) continue;
        const bool fin = is_long ? walk_step<STATS>(im, cur, gp, em, st) : walk_step<STATS>(im, cur, lp, em, st);
        if (fin) {
            em.flush();
            counts[my] = em.cnt;
            match_sum += em.cnt;
            my = NO_TOPIC;
        }
    }
    wave_stats_add<STATS>(stats, lev_sum, st.visits, st.edge_reads, match_sum);
}

__global__ void __launch_bounds__(BLOCK)
tm_copy_out(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ words,
            const uint32_t* __restrict__ meta, uint32_t* __restrict__ path_scratch,
            const uint32_t* __restrict__ stage, uint32_t K, const uint32_t* __restrict__ counts,
            const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out, uint64_t out_cap) {
    __shared__ uint32_t lds_path[LDS_LEVELS * BLOCK];
    __shared__ uint32_t lds_inc[BLOCK];
    __shared__ uint64_t lds_scan[BLOCK / 64];
    const uint32_t t0 = blockIdx.x * BLOCK;
    const uint32_t tn = n - t0 < (uint32_t)BLOCK ? n - t0 : (uint32_t)BLOCK;
    const uint32_t c = threadIdx.x < tn ? counts[t0 + threadIdx.x] : 0u;
    uint64_t agg;
    const uint64_t ex = block_exclusive_scan(c, lds_scan, agg);
    lds_inc[threadIdx.x] = (uint32_t)(ex + c);
    __syncthreads();
    const uint64_t base = out_off[t0];
    for (uint64_t j = threadIdx.x; j < agg; j += BLOCK) {
        uint32_t lo = 0, hi = tn - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)lds_inc[mid] > j) hi = mid; else lo = mid + 1;
        }
        const uint32_t k = (uint32_t)(j - (lo ? lds_inc[lo - 1] : 0u));
        if (k < K && base + j < out_cap) out[base + j] = stage[(uint64_t)(t0 + lo) * K + k];
    }
    if (threadIdx.x < tn && c > K) {   // fan-out beyond the stage row: walk again, write the tail
        const uint32_t t = t0 + threadIdx.x;
        const uint32_t mt = meta[t];
        const uint64_t b = off[t] - off[0];
        DirectEmit em{out, base + ex, out_cap, K, 0};
        WalkStats s2;
        if (mt & MLONG)
            walk<false>(im, words + b + t, mt & MN, (mt & MDOLLAR) != 0, GlobalPath{path_scratch + b + 2ull * t}, em,
                        s2);
        else
            walk<false>(im, words + b + t, mt & MN, (mt & MDOLLAR) != 0, LdsPath{lds_path + threadIdx.x}, em, s2);
    }
}

constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;

__global__ void __launch_bounds__(BLOCK)
tm_scan_reduce(const uint32_t* __restrict__ in, uint32_t n, uint64_t* __restrict__ tile_sums) {
    __shared__ uint64_t lds[BLOCK / 64];
    uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint64_t k = base + (uint64_t)i * BLOCK + threadIdx.x;
        if (k < n) s += in[k];
    }
    uint64_t tot;
    block_exclusive_scan(s, lds, tot);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK)
tm_scan_tiles(uint64_t* __restrict__ tile_sums, uint32_t n_tiles) {
    __shared__ uint64_t lds[BLOCK / 64];
    uint64_t carry = 0;
    for (uint32_t b = 0; b < n_tiles; b += BLOCK) {
        uint32_t k = b + threadIdx.x;
        uint64_t x = k < n_tiles ? tile_sums[k] : 0;
        uint64_t tot;
        uint64_t ex = block_exclusive_scan(x, lds, tot);
        if (k < n_tiles) tile_sums[k] = carry + ex;
        carry += tot;
    }
}

__global__ void __launch_bounds__(BLOCK)
tm_scan_final(const uint32_t* __restrict__ in, uint32_t n, const uint64_t* __restrict__ tile_pre,
              uint64_t* __restrict__ out_off, uint64_t* __restrict__ total) {
    __shared__ uint64_t lds[BLOCK / 64];
    uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint64_t k = base + i;
        v[i] = k < n ? in[k] : 0;
        s += v[i];
    }
    uint64_t tot;
    uint64_t ex = block_exclusive_scan(s, lds, tot) + tile_pre[blockIdx.x];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        uint64_t k = base + i;
        if (k < n) out_off[k] = ex;
        ex += v[i];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == BLOCK - 1) {
        out_off[n] = ex;
        *total = ex;
    }
}

// ---------------------------------------------------------------------------
// host launchers

static inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// ws words: counter, error, one status word per tile (smallest tile = BLOCK)
size_t fused_ws_words(uint32_t n) { return 2 + (size_t)div_up(n ? n : 1, BLOCK) + 2; }
size_t fused_stage_elems(uint32_t n, uint32_t K) { return (size_t)div_up(n ? n : 1, TILE_MAX) * TILE_MAX * K; }

template <class Kern>
static uint32_t resident_grid(Kern k, uint32_t n_tiles) {
    int dev = 0, cus = 256, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, BLOCK, 0);
    uint32_t g = (uint32_t)((per > 0 ? per : 1) * (cus > 0 ? cus : 1));
    return g < n_tiles ? g : n_tiles;
}

template <uint32_t TILE>
static hipError_t launch_fused_t(bool stats_mode, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                                 uint32_t n, uint32_t* words, uint32_t* path_scratch, uint32_t* stage, uint32_t K,
                                 uint32_t* counts, uint64_t* out_off, uint32_t* out, uint64_t out_cap,
                                 uint64_t* total, unsigned long long* ws, unsigned long long* stats, hipStream_t st) {
    uint32_t n_tiles = div_up(n, TILE);
    dim3 blk(BLOCK);
    if (stats_mode)
        hipLaunchKernelGGL((tm_match_fused<true, TILE>), dim3(resident_grid(tm_match_fused<true, TILE>, n_tiles)),
                           blk, 0, st, im, bytes, off, n, words, path_scratch, stage, K, counts, out_off, out,
                           out_cap, total, ws, stats);
    else
        hipLaunchKernelGGL((tm_match_fused<false, TILE>), dim3(resident_grid(tm_match_fused<false, TILE>, n_tiles)),
                           blk, 0, st, im, bytes, off, n, words, path_scratch, stage, K, counts, out_off, out,
                           out_cap, total, ws, stats);
    return hipGetLastError();
}

hipError_t launch_fused(int variant, bool stats_mode, const ImageView& im, const uint8_t* bytes,
                        const uint64_t* off, uint32_t n, uint32_t* words, uint32_t* path_scratch, uint32_t* stage,
                        uint32_t K, uint32_t* counts, uint64_t* out_off, uint32_t* out, uint64_t out_cap,
                        uint64_t* total, unsigned long long* ws, unsigned long long* stats, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipError_t err = hipMemsetAsync(ws, 0, fused_ws_words(n) * 8, st);
    if (err != hipSuccess) return err;
    switch (variant) {
        case TM_VARIANT_LANE: {
            dim3 g(div_up(n, BLOCK)), blk(BLOCK);
            if (stats_mode)
                hipLaunchKernelGGL(tm_match_lane<true>, g, blk, 0, st, im, bytes, off, n, words, path_scratch,
                                   stage, K, counts, out_off, out, out_cap, total, ws, stats);
            else
                hipLaunchKernelGGL(tm_match_lane<false>, g, blk, 0, st, im, bytes, off, n, words, path_scratch,
                                   stage, K, counts, out_off, out, out_cap, total, ws, stats);
            return hipGetLastError();
        }
        case TM_VARIANT_TILE256:
            return launch_fused_t<256>(stats_mode, im, bytes, off, n, words, path_scratch, stage, K, counts, out_off,
                                       out, out_cap, total, ws, stats, st);
        case TM_VARIANT_TILE512:
            return launch_fused_t<512>(stats_mode, im, bytes, off, n, words, path_scratch, stage, K, counts, out_off,
                                       out, out_cap, total, ws, stats, st);
        default:
            return launch_fused_t<1024>(stats_mode, im, bytes, off, n, words, path_scratch, stage, K, counts,
                                        out_off, out, out_cap, total, ws, stats, st);
    }
}

hipError_t launch_queue(bool stats_mode, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, uint32_t* words, uint32_t* meta, uint32_t* path_scratch, uint32_t* stage,
                        uint32_t K, uint32_t* counts, uint64_t* out_off, uint32_t* out, uint64_t out_cap,
                        uint64_t* total, uint64_t* scan_tmp, unsigned long long* ws, unsigned long long* stats,
                        hipStream_t st, hipEvent_t* marks) {
    if (n == 0) return hipSuccess;
    hipError_t err = hipMemsetAsync(ws, 0, 16, st);
    if (err != hipSuccess) return err;
    dim3 blk(BLOCK), g(div_up(n, BLOCK));
    auto mark = [&](int i) {
        if (marks) (void)hipEventRecord(marks[i], st);
    };
    mark(0);
    hipLaunchKernelGGL(tm_tokenize, g, blk, 0, st, im, bytes, off, n, words, meta);
    mark(1);
    mark(2);
    uint32_t wg = stats_mode ? resident_grid(tm_walk_queue<true>, div_up(n, 64))
                             : resident_grid(tm_walk_queue<false>, div_up(n, 64));
    if (stats_mode)
        hipLaunchKernelGGL(tm_walk_queue<true>, dim3(wg), blk, 0, st, im, off, n, words, meta, path_scratch, stage, K,
                           counts, ws, stats);
    else
        hipLaunchKernelGGL(tm_walk_queue<false>, dim3(wg), blk, 0, st, im, off, n, words, meta, path_scratch, stage,
                           K, counts, ws, stats);
    mark(3);
    mark(4);
    err = launch_scan(counts, n, out_off, total, scan_tmp, st);
    if (err != hipSuccess) return err;
    mark(5);
    mark(6);
    if (out_cap)
        hipLaunchKernelGGL(tm_copy_out, g, blk, 0, st, im, off, n, words, meta, path_scratch, stage, K, counts,
                           out_off, out, out_cap);
    mark(7);
    return hipGetLastError();
}

hipError_t launch_tokenize(const ImageView& im, const uint8_t* bytes, const uint64_t* off, uint32_t n,
                           uint32_t* words, uint32_t* meta, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(tm_tokenize, dim3(div_up(n, BLOCK)), dim3(BLOCK), 0, st, im, bytes, off, n,
                       words, meta);
    return hipGetLastError();
}

hipError_t launch_match(int mode, bool long_topics, const ImageView& im, const uint64_t* off, uint32_t n,
                        const uint32_t* words, const uint32_t* meta, uint32_t* counts,
                        const uint64_t* out_off, uint32_t* out, uint64_t out_cap,
                        uint32_t* path_scratch, unsigned long long* stats, hipStream_t st) {
    if (n == 0) return hipSuccess;
    dim3 g(div_up(n, BLOCK)), b(BLOCK);
#define TM_L(M, L)                                                                                  \
    hipLaunchKernelGGL((tm_match<M, L>), g, b, 0, st, im, off, n, words, meta, counts, out_off, out, \
                       out_cap, path_scratch, stats)
    if (!long_topics) {
        if (mode == TM_MODE_COUNT) TM_L(TM_MODE_COUNT, false);
        else if (mode == TM_MODE_EMIT) TM_L(TM_MODE_EMIT, false);
        else TM_L(TM_MODE_STATS, false);
    } else {
        if (mode == TM_MODE_COUNT) TM_L(TM_MODE_COUNT, true);
        else if (mode == TM_MODE_EMIT) TM_L(TM_MODE_EMIT, true);
        else TM_L(TM_MODE_STATS, true);
    }
#undef TM_L
    return hipGetLastError();
}

size_t scan_tmp_elems(uint32_t n) { return div_up(n ? n : 1, SCAN_TILE); }

hipError_t launch_scan(const uint32_t* counts, uint32_t n, uint64_t* out_off, uint64_t* total,
                       uint64_t* tmp, hipStream_t st) {
    if (n == 0) {
        hipError_t err = hipMemsetAsync(out_off, 0, sizeof(uint64_t), st);
        if (err == hipSuccess) err = hipMemsetAsync(total, 0, sizeof(uint64_t), st);
        return err;
    }
    uint32_t tiles = div_up(n, SCAN_TILE);
    hipLaunchKernelGGL(tm_scan_reduce, dim3(tiles), dim3(BLOCK), 0, st, counts, n, tmp);
    hipLaunchKernelGGL(tm_scan_tiles, dim3(1), dim3(BLOCK), 0, st, tmp, tiles);
    hipLaunchKernelGGL(tm_scan_final, dim3(tiles), dim3(BLOCK), 0, st, counts, n, tmp, out_off, total);
    return hipGetLastError();
}

}  // namespace tmx
