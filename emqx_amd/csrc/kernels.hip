// kernels.hip — CDNA4 (gfx950) kernels of the topic-routing hot path.
//
//   tm_tokenize   emqx_topic:words/1 + word/1 (src/emqx_topic.erl:141-147):
//                 split every topic on '/', hash each level, probe the word
//                 dictionary and byte-verify -> per-level word ids.
//   tm_match<M>   emqx_trie:match/1 (src/emqx_trie.erl:77-79, 121-145):
//                 one lane per topic walks the NFA over '+'/'#'/literal edges
//                 in the mirrored DFS order that IS the reference's output
//                 order (plus subtree, literal subtree, then the '#' filter;
//                 at the last level: self filter, then '#' filter), so no
//                 sort is needed.  M = COUNT | EMIT | STATS.
//   tm_scan_*     exclusive scan of per-topic counts -> CSR offsets.
//
// All integer/byte work: no MFMA.  The walk is latency-bound pointer chasing
// over the HBM image (image.h); the roofline is HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "image.h"
#include "kernels.h"

namespace tmx {

// ---------------------------------------------------------------------------
// byte access: aligned 8-byte loads (never cross a page past the last valid
// byte), little-endian extraction.
__device__ __forceinline__ uint64_t load_u64_aligned(const uint8_t* base, uint64_t p) {
    return *reinterpret_cast<const uint64_t*>(base + (p & ~7ull));
}

// assemble up to 8 bytes [p, p+k) (k in 1..8) little-endian, zero padded
__device__ __forceinline__ uint64_t load_chunk(const uint8_t* base, uint64_t p, uint32_t k) {
    uint32_t sh = (uint32_t)(p & 7) * 8;
    uint64_t lo = load_u64_aligned(base, p);
    uint64_t v = lo >> sh;
    if (sh != 0 && (p & 7) + k > 8) {
        uint64_t hi = load_u64_aligned(base, p + 8);
        v |= hi << (64 - sh);
    }
    if (k < 8) v &= (~0ull) >> (64 - 8 * k);
    return v;
}

// dictionary lookup of topic bytes [p, p+len): returns word id or WORD_NONE
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

// one thread per topic.  words of topic t land at words[off[t] + t + l]
// (a topic of B bytes has at most B+1 levels, so the slot range is private).
// meta[t] = n_levels | (first level starts with '$') << 31.
__global__ void __launch_bounds__(256)
tm_tokenize(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
            uint32_t n, uint32_t* __restrict__ words, uint32_t* __restrict__ meta) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint64_t b = off[t], e = off[t + 1];
    uint32_t* w = words + (b - off[0]) + t;
    uint32_t lev = 0;
    uint64_t s = b;
    uint32_t dollar = 0;
    if (e > b && bytes[b] == '$') dollar = 1u;
    // scan aligned 8-byte words for '/'
    uint64_t p = b;
    while (true) {
        uint64_t q = p;  // find next '/' at or after p, or e
        bool found = false;
        while (q < e) {
            uint64_t word8 = load_u64_aligned(bytes, q);
            uint32_t start = (uint32_t)(q & 7);
            uint32_t stop = (e - (q & ~7ull)) < 8 ? (uint32_t)(e - (q & ~7ull)) : 8;
            // bytes [start, stop) of this aligned word are in range
            uint64_t x = word8 ^ 0x2F2F2F2F2F2F2F2FULL;           // '/' -> 0x00
            uint64_t z = (x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL;
            z &= (~0ull) << (8 * start);
            if (stop < 8) z &= (~0ull) >> (64 - 8 * stop);
            if (z) { q = (q & ~7ull) + (__builtin_ctzll(z) >> 3); found = true; break; }
            q = (q & ~7ull) + 8;
        }
        if (!found) q = e;
        w[lev++] = dict_lookup(im, bytes, s, (uint32_t)(q - s));
        if (!found) break;
        s = p = q + 1;
    }
    meta[t] = lev | (dollar << 31);
}

// ---------------------------------------------------------------------------
// literal child of v by word w (WORD_PLUS / WORD_HASH reproduce the reference
// for the out-of-domain topic levels "+" / "#": the fold over [W, '+'] at
// emqx_trie.erl:131-136 follows the '+' / '#' edge for them)
__device__ __forceinline__ uint32_t child_of(const ImageView& im, uint32_t v, Node rec,
                                             uint32_t w) {
    if (w >= WORD_MAX) {
        if (w == WORD_PLUS) return rec.plus & NODE_MASK;
        if (w == WORD_HASH) return rec.hash;
        return NODE_NONE;
    }
    if (!(rec.plus & HAS_LIT)) return NODE_NONE;
    // probing starts at a bucket boundary and advances one 64 B bucket (one
    // HBM burst, 4 slots) per round
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

// The mirrored DFS.  path[r] = node | phase << 30 for the node on the current
// path at level r; phase 0 = '+' branch next, 1 = literal branch next,
// 2 = both done (emit the '#' filter).  Output order equals emqx_trie:match/1:
//   out(v, r<n) = out(plus(v)) ++ out(lit(v, w_r)) ++ [hash_filter(v)]
//   out(v, n)   = [self_filter(v), hash_filter(v)]
// (the reference prepends each discovery to its accumulator: :127-145).
template <int MODE, typename PathRef>
__device__ __forceinline__ uint32_t walk_topic(const ImageView& im, const uint32_t* __restrict__ w,
                                               uint32_t n, bool dollar, PathRef path,
                                               uint32_t* __restrict__ out, uint64_t out_base,
                                               uint64_t out_cap, uint64_t& visits,
                                               uint64_t& edge_reads) {
    uint32_t cnt = 0;
    uint32_t r0 = 0, start = ROOT;
    if (dollar) {
        // '$' rule (emqx_trie.erl:121-122): jump straight to node <<W0>>,
        // skipping root's '#' and '+' edges.
        Node root = im.nodes[ROOT];
        start = child_of(im, ROOT, root, w[0]);
        r0 = 1;
        if (start == NODE_NONE) return 0;
    }
    uint32_t r = r0;
    path(r) = start;
    for (;;) {
        uint32_t e = path(r);
        uint32_t v = e & NODE_MASK, ph = e >> 30;
        Node rec = im.nodes[v];
        if (MODE == TM_MODE_STATS && ph == 0) {
            ++visits;
            edge_reads += (r == n) ? 1 : 3;
        }
        if (r == n) {
            if (rec.self_filter != FILTER_NONE) {
                if (MODE == TM_MODE_EMIT && out_base + cnt < out_cap) out[out_base + cnt] = rec.self_filter;
                ++cnt;
            }
            if (rec.hash_filter != FILTER_NONE) {
                if (MODE == TM_MODE_EMIT && out_base + cnt < out_cap) out[out_base + cnt] = rec.hash_filter;
                ++cnt;
            }
        } else {
            if (ph == 0) {
                path(r) = v | (1u << 30);
                uint32_t c = rec.plus & NODE_MASK;
                if (c != NODE_NONE) { path(++r) = c; continue; }
                ph = 1;
            }
            if (ph == 1) {
                path(r) = v | (2u << 30);
                uint32_t c = child_of(im, v, rec, w[r]);
                if (c != NODE_NONE) { path(++r) = c; continue; }
            }
            if (rec.hash_filter != FILTER_NONE) {
                if (MODE == TM_MODE_EMIT && out_base + cnt < out_cap) out[out_base + cnt] = rec.hash_filter;
                ++cnt;
            }
        }
        if (r == r0) break;
        --r;
    }
    return cnt;
}

constexpr int BLOCK = 256;
constexpr uint32_t LDS_LEVELS = 32;   // topics with n < 32 keep their path in LDS

struct LdsPath {
    uint32_t* base;   // [level][BLOCK]
    __device__ __forceinline__ uint32_t& operator()(uint32_t r) const { return base[r * BLOCK]; }
};
struct GlobalPath {
    uint32_t* base;
    __device__ __forceinline__ uint32_t& operator()(uint32_t r) const { return base[r]; }
};

// LONG = false: topics with n < LDS_LEVELS (path in LDS), others skipped.
// LONG = true : topics with n >= LDS_LEVELS, path in a private global slice
//               path_scratch[off[t] + 2t ...] (n+1 <= bytes+2 entries).
template <int MODE, bool LONG>
__global__ void __launch_bounds__(BLOCK)
tm_match(ImageView im, const uint64_t* __restrict__ off, uint32_t n_topics,
         const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta,
         uint32_t* __restrict__ counts, const uint64_t* __restrict__ out_off,
         uint32_t* __restrict__ out, uint64_t out_cap, uint32_t* __restrict__ path_scratch,
         unsigned long long* __restrict__ stats) {
    __shared__ uint32_t lds_path[LONG ? 1 : LDS_LEVELS * BLOCK];
    uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t visits = 0, edge_reads = 0;
    uint32_t cnt = 0, nlev = 0;
    if (t < n_topics) {
        uint32_t m = meta[t];
        nlev = m & 0x7FFFFFFFu;
        bool dollar = (m >> 31) != 0;
        bool is_long = nlev >= LDS_LEVELS;
        if (is_long == LONG) {
            uint64_t b = off[t] - off[0];
            const uint32_t* w = words + b + t;
            uint64_t base = (MODE == TM_MODE_EMIT) ? out_off[t] : 0;
            if (LONG) {
                GlobalPath p{path_scratch + b + 2ull * t};
                cnt = walk_topic<MODE>(im, w, nlev, dollar, p, out, base, out_cap, visits, edge_reads);
            } else {
                LdsPath p{lds_path + threadIdx.x};
                cnt = walk_topic<MODE>(im, w, nlev, dollar, p, out, base, out_cap, visits, edge_reads);
            }
            if (MODE != TM_MODE_EMIT) counts[t] = cnt;
        } else {
            nlev = 0;   // accounted by the other instantiation
        }
    }
    if (MODE == TM_MODE_STATS) {
        // wave-reduce, one atomic per wave per counter
        uint64_t v[4] = {nlev, visits, edge_reads, cnt};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint64_t x = v[k];
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if ((threadIdx.x & 63) == 0 && x) atomicAdd(stats + k, (unsigned long long)x);
        }
    }
}

// ---------------------------------------------------------------------------
// exclusive scan u32 counts -> u64 offsets (3 kernels, ITEMS per thread)
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t x, uint64_t* lds, uint64_t& total) {
    // inclusive within the wave
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

// single block: exclusive scan of tile sums in place
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
