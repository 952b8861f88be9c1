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

// child of v by topic word w.  WORD_PLUS / WORD_HASH reproduce the reference
// for the out-of-domain topic levels "+" / "#": the fold over [W, '+'] at
// emqx_trie.erl:131-136 follows the '+' / '#' edge for them.
__device__ __forceinline__ uint32_t child_of(const ImageView& im, uint32_t v, Node rec, uint32_t w) {
    if (w >= WORD_MAX) {
        if (w == WORD_PLUS) return rec.plus & NODE_MASK;
        if (w == WORD_HASH) return rec.hash;
        return NODE_NONE;
    }
    if (!(rec.plus & HAS_LIT)) return NODE_NONE;
    return probe_edge(im, v, w);
}

// ---------------------------------------------------------------------------
// The mirrored DFS.  path(r) = node | flags for the node on the current path
// at level r:  bits 31..30 phase (0 = first visit, 1 = literal branch next,
// 2 = both branches done), bit 29 = the node has a '#' filter to emit.
// Output order equals emqx_trie:match/1 (which prepends every discovery to its
// accumulator, :127-145):
//   out(v, r<n) = out(plus(v)) ++ out(lit(v, w_r)) ++ [hash_filter(v)]
//   out(v, n)   = [self_filter(v), hash_filter(v)]
// A node record is read once per visit; the return visits need only the
// path word (the literal probe needs v and w_r, the '#' emission re-reads
// the record only for the few nodes that have one).
constexpr uint32_t P_NODE = NODE_MASK;
constexpr uint32_t P_HASH = 1u << 29;

struct WalkStats {
    uint64_t visits = 0, edge_reads = 0;
};

template <bool STATS, typename PathRef, typename Emit>
__device__ __forceinline__ void walk(const ImageView& im, const uint32_t* __restrict__ w, uint32_t n,
                                     bool dollar, PathRef path, Emit& emit, WalkStats& st) {
    uint32_t r0 = 0, start = ROOT;
    if (dollar) {
        // '$' rule (emqx_trie.erl:121-122): jump straight to node <<W0>>,
        // skipping root's '#' and '+' edges.
        start = child_of(im, ROOT, im.nodes[ROOT], w[0]);
        r0 = 1;
        if (start == NODE_NONE) return;
    }
    uint32_t r = r0;
    path(r) = start;
    for (;;) {
        uint32_t e = path(r);
        uint32_t v = e & P_NODE, ph = e >> 30;
        if (ph == 0) {
            Node rec = im.nodes[v];
            if (STATS) {
                ++st.visits;
                st.edge_reads += (r == n) ? 1 : 3;  // 'match_#' + fold [W, '+'] (:132, :141)
            }
            if (r == n) {
                if (rec.self_filter != FILTER_NONE) emit(rec.self_filter);
                if (rec.hash_filter != FILTER_NONE) emit(rec.hash_filter);
                goto up;
            }
            uint32_t wr = w[r];
            bool lit = wr < WORD_MAX ? (rec.plus & HAS_LIT) != 0
                                     : (wr == WORD_PLUS ? (rec.plus & NODE_MASK) != NODE_NONE
                                                        : (wr == WORD_HASH && rec.hash != NODE_NONE));
            e = v | (rec.hash_filter != FILTER_NONE ? P_HASH : 0u) | ((lit ? 1u : 2u) << 30);
            path(r) = e;
            uint32_t c = rec.plus & NODE_MASK;
            if (c != NODE_NONE) {
                path(++r) = c;
                continue;
            }
            ph = e >> 30;
        }
        if (ph == 1) {
            e = (e & ~(3u << 30)) | (2u << 30);
            path(r) = e;
            uint32_t wr = w[r];
            uint32_t c = wr < WORD_MAX ? probe_edge(im, v, wr) : child_of(im, v, im.nodes[v], wr);
            if (c != NODE_NONE) {
                path(++r) = c;
                continue;
            }
        }
        if (e & P_HASH) emit(im.nodes[v].hash_filter);
    up:
        if (r == r0) break;
        --r;
    }
}

constexpr uint32_t LDS_LEVELS = 24;   // topics with n < 24 keep their path in LDS (24 KiB: 6 WG/CU)

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
// the fused kernel.  Grid = ceil(n / BLOCK) workgroups; the tile a workgroup
// processes is drawn from a counter so every predecessor in the look-back
// chain is already running (forward progress without co-residency).
// ws layout (zeroed per launch): ws[0] tile counter, ws[1] error word,
// ws[2 ..] one status word per tile.
template <bool STATS>
__global__ void __launch_bounds__(BLOCK)
tm_match_fused(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
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

__global__ void __launch_bounds__(BLOCK)
tm_tokenize(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
            uint32_t n, uint32_t* __restrict__ words, uint32_t* __restrict__ meta) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t b = off[t], e = off[t + 1];
    uint32_t lev = tokenize_topic(im, bytes, b, e, words + (b - off[0]) + t);
    uint32_t dollar = (e > b && bytes[b] == '$') ? 1u : 0u;
    meta[t] = lev | (dollar << 31);
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
        nlev = m & 0x7FFFFFFFu;
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

size_t fused_ws_words(uint32_t n) { return 2 + (size_t)div_up(n ? n : 1, BLOCK) + 2; }
size_t fused_stage_elems(uint32_t n, uint32_t K) { return (size_t)div_up(n ? n : 1, BLOCK) * BLOCK * K; }

hipError_t launch_fused(bool stats_mode, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, uint32_t* words, uint32_t* path_scratch, uint32_t* stage, uint32_t K,
                        uint32_t* counts, uint64_t* out_off, uint32_t* out, uint64_t out_cap, uint64_t* total,
                        unsigned long long* ws, unsigned long long* stats, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipError_t err = hipMemsetAsync(ws, 0, fused_ws_words(n) * 8, st);
    if (err != hipSuccess) return err;
    dim3 g(div_up(n, BLOCK)), blk(BLOCK);
    if (stats_mode)
        hipLaunchKernelGGL(tm_match_fused<true>, g, blk, 0, st, im, bytes, off, n, words, path_scratch, stage, K,
                           counts, out_off, out, out_cap, total, ws, stats);
    else
        hipLaunchKernelGGL(tm_match_fused<false>, g, blk, 0, st, im, bytes, off, n, words, path_scratch, stage, K,
                           counts, out_off, out, out_cap, total, ws, stats);
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
