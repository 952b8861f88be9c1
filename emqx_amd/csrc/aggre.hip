// aggre.hip — emqx_broker:aggre/1 on the device:
//
//   publish(Msg) -> ... route(aggre(emqx_router:match_routes(Topic)), ...)
//                                              (src/emqx_broker.erl:152)
//   aggre([]) -> [];
//   aggre([#route{topic = To, dest = Node}]) when is_atom(Node) -> [{To, Node}];
//   aggre([#route{topic = To, dest = {Group, _Node}}]) -> [{To, Group}];
//   aggre(Routes) ->
//       lists:foldl(fun(#route{topic = To, dest = Node}, Acc) when is_atom(Node) ->
//                          [{To, Node} | Acc];
//                      (#route{topic = To, dest = {Group, _Node}}, Acc) ->
//                          lists:usort([{To, Group} | Acc])
//                   end, [], Routes).        (src/emqx_broker.erl:194-206)
//
// Closed form of the fold for routes r_0..r_{m-1} (the single-route clauses
// agree with it): let j be the last route whose dest is {Group, Node}.  With
// no such route the result is the routes reversed (no dedup).  Otherwise it
// is r_{m-1}, ..., r_{j+1} (reversed, no dedup) followed by the sorted,
// duplicate-free set of {To, X} over r_0..r_j (lists:usort re-sorts the whole
// accumulator, node entries included).
//
// Erlang term order of {To, X}: To (a binary) first, bytewise, a proper
// prefix first; then X: a node atom < a group binary, each by its bytes.  The
// host turns both into ranks (to_rank over every topic with routes, target
// rank over every target), so a sort key is one u64 = to_rank << 32 | rank;
// tm_route_emit writes it beside each route (routes.hip).
//
// tm_aggre: one wave per topic with up to 128 routes, all in registers: one
// round of coalesced loads (src, dest, key), a bitonic sort of 64-bit words
// (key with the element index packed under the target rank, two per lane,
// network unrolled per padded size), a ballot that keeps the first of each
// run of equal keys; up to 512 routes the same in the wave's LDS row.
// Larger topics go on a device-built list that
// tm_aggre_large works through with one 256-thread block per topic (LDS
// bitonic up to 4096 routes; beyond, the topic's key row is sorted in place:
// 4096-key chunks in LDS, then bitonic merge stages over the row in global
// memory, O(u log^2 u)), so nothing waits on the host.
// Output goes straight to the topic's route offset (aggre never grows a
// list): offsets are the route CSR's, counts are aggre's, so the lists need
// no compaction pass (measured 0.75 ms per 2M topics at C3).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "image.h"
#include "kernels.h"

namespace tmx {

constexpr int AG_BLOCK = 256;
constexpr int AG_WAVES = AG_BLOCK / 64;
constexpr uint32_t AG_GROUP_BIT = 0x80000000u;
constexpr uint32_t AG_LDS = 512;   // tm_aggre's per-wave LDS row (routes)

__device__ __forceinline__ int wave_max_i(int x) {
    for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
    return x;
}
__device__ __forceinline__ uint32_t wave_sum_u(uint32_t x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

// bitonic sort of 128 u64 keys held two per lane (element lane and lane +
// 64) in registers: cross-lane steps by shuffles, the distance-64 step inside
// the lane; ascending.  Keys only (each carries its element index in its low
// bits), so a step costs two 32-bit shuffles per element.
template <uint32_t P>
__device__ __forceinline__ void wave_sort_p(uint64_t& k0, uint64_t& k1, uint32_t lane) {
#pragma unroll
    for (uint32_t size = 2; size <= P; size <<= 1) {
#pragma unroll
        for (uint32_t d = size >> 1; d > 0; d >>= 1) {
            if (d == 64) {   // pairs (lane, lane + 64); size == 128 here, so ascending
                const uint64_t lo = k0 < k1 ? k0 : k1, hi = k0 < k1 ? k1 : k0;
                k0 = lo;
                k1 = hi;
                continue;
            }
            const bool lower = (lane & d) == 0;
            {
                const uint64_t pk = shfl_xor_u64(k0, (int)d);
                const bool up = (lane & size) == 0;            // element index lane
                if (lower == up ? pk < k0 : pk > k0) k0 = pk;
            }
            if (P > 64) {
                const uint64_t pk = shfl_xor_u64(k1, (int)d);
                const bool up = ((lane + 64) & size) == 0;     // element index lane + 64
                if (lower == up ? pk < k1 : pk > k1) k1 = pk;
            }
        }
    }
}
// the network unrolled at compile time for the padded size P (a runtime
// distance loop, and DPP picked per stage by a switch, measured slower)
__device__ __forceinline__ void wave_sort128(uint64_t& k0, uint64_t& k1, uint32_t P, uint32_t lane) {
    if (P <= 8) wave_sort_p<8>(k0, k1, lane);
    else if (P <= 16) wave_sort_p<16>(k0, k1, lane);
    else if (P <= 32) wave_sort_p<32>(k0, k1, lane);
    else if (P <= 64) wave_sort_p<64>(k0, k1, lane);
    else wave_sort_p<128>(k0, k1, lane);
}

// topics with up to 128 routes, all in registers: one round of coalesced
// loads (src, dest, key) and a gather from the small target table, then the
// fold's reversed tail and the usort go straight to the output
__device__ __forceinline__ uint32_t aggre_regs(const AggreView& av, uint32_t m, uint64_t base, uint32_t lane,
                                               const uint32_t* __restrict__ src, const uint32_t* __restrict__ dest,
                                               const uint64_t* __restrict__ gkey, uint32_t* __restrict__ out_to,
                                               uint32_t* __restrict__ out_tg, uint64_t out_cap) {
    uint64_t k0 = ~0ull, k1 = ~0ull;
    uint32_t s0 = 0, s1 = 0, g0 = 0, g1 = 0;
    if (lane < m) {
        s0 = src[base + lane];
        k0 = gkey[base + lane];
        g0 = av.dt[dest[base + lane]].y;
    }
    if (lane + 64 < m) {
        s1 = src[base + lane + 64];
        k1 = gkey[base + lane + 64];
        g1 = av.dt[dest[base + lane + 64]].y;
    }
    int j = (g1 & AG_GROUP_BIT) ? (int)lane + 64 : (g0 & AG_GROUP_BIT) ? (int)lane : -1;
    j = wave_max_i(j);
    const uint32_t tail = (uint32_t)((int)m - 1 - j);
    // r_{m-1} .. r_{j+1}: element i goes to position m - 1 - i
    if ((int)lane > j && lane < m && base + (m - 1 - lane) < out_cap) {
        out_to[base + (m - 1 - lane)] = s0;
        out_tg[base + (m - 1 - lane)] = g0 & ~AG_GROUP_BIT;
    }
    if ((int)lane + 64 > j && lane + 64 < m && base + (m - 65 - lane) < out_cap) {
        out_to[base + (m - 65 - lane)] = s1;
        out_tg[base + (m - 65 - lane)] = g1 & ~AG_GROUP_BIT;
    }
    if (j < 0) return tail;
    // lists:usort over r_0 .. r_j.  Sort word: to_rank << 32 | target rank <<
    // 7 | element index (target ranks < 2^25, checked on the host): unique,
    // so the sort needs no payload; keys past j become ~0 (above every real
    // key); equal routes are equal in the word's top 57 bits.
    const uint32_t u = (uint32_t)j + 1;
    k0 = lane < u ? (k0 & 0xFFFFFFFF00000000ull) | ((k0 & 0xFFFFFFFFull) << 7) | lane : ~0ull;
    k1 = lane + 64 < u ? (k1 & 0xFFFFFFFF00000000ull) | ((k1 & 0xFFFFFFFFull) << 7) | (lane + 64) : ~0ull;
    uint32_t P = 2;
    while (P < u) P <<= 1;
#if !(defined(TM_AGGRE_VARIANT) && TM_AGGRE_VARIANT == 2)   // EXPERIMENT 2: no sort
    wave_sort128(k0, k1, P, lane);
#endif
    const uint64_t prev0 = shfl_u64(k0, (int)((lane + 63) & 63));   // element lane - 1 (unused at lane 0)
    const uint64_t last0 = shfl_u64(k0, 63);
    uint64_t prev1 = shfl_u64(k1, (int)((lane + 63) & 63));
    if (lane == 0) prev1 = last0;                                    // element 64's predecessor is element 63
    const bool keep0 = lane < u && (lane == 0 || (k0 >> 7) != (prev0 >> 7));
    const bool keep1 = lane + 64 < u && (k1 >> 7) != (prev1 >> 7);
    // source and target of each sorted word's element, from its owner lane
    const uint32_t e0 = (uint32_t)k0 & 127u, e1 = (uint32_t)k1 & 127u;
    const uint32_t sa0 = (uint32_t)__shfl((int)s0, (int)(e0 & 63), 64), sb0 = (uint32_t)__shfl((int)s1, (int)(e0 & 63), 64);
    const uint32_t ga0 = (uint32_t)__shfl((int)g0, (int)(e0 & 63), 64), gb0 = (uint32_t)__shfl((int)g1, (int)(e0 & 63), 64);
    const uint32_t sa1 = (uint32_t)__shfl((int)s0, (int)(e1 & 63), 64), sb1 = (uint32_t)__shfl((int)s1, (int)(e1 & 63), 64);
    const uint32_t ga1 = (uint32_t)__shfl((int)g0, (int)(e1 & 63), 64), gb1 = (uint32_t)__shfl((int)g1, (int)(e1 & 63), 64);
    const uint64_t bal0 = __ballot(keep0), bal1 = __ballot(keep1);
    const uint64_t lt = (1ull << lane) - 1;
    const uint64_t o = base + tail;
    if (keep0) {
        const uint64_t pos = o + (uint32_t)__popcll(bal0 & lt);
        if (pos < out_cap) {
            out_to[pos] = e0 < 64 ? sa0 : sb0;
            out_tg[pos] = (e0 < 64 ? ga0 : gb0) & ~AG_GROUP_BIT;
        }
    }
    if (keep1) {
        const uint64_t pos = o + (uint32_t)__popcll(bal0) + (uint32_t)__popcll(bal1 & lt);
        if (pos < out_cap) {
            out_to[pos] = e1 < 64 ? sa1 : sb1;
            out_tg[pos] = (e1 < 64 ? ga1 : gb1) & ~AG_GROUP_BIT;
        }
    }
    return tail + (uint32_t)__popcll(bal0) + (uint32_t)__popcll(bal1);
}

__global__ void __launch_bounds__(AG_BLOCK)
tm_aggre(AggreView av, uint32_t n, const uint32_t* __restrict__ rcount, const uint64_t* __restrict__ roff,
         const uint32_t* __restrict__ src, const uint32_t* __restrict__ dest, const uint64_t* __restrict__ gkey,
         uint32_t* __restrict__ large, uint32_t* __restrict__ acount, uint32_t* __restrict__ out_to,
         uint32_t* __restrict__ out_tg, uint64_t out_cap) {
    __shared__ uint64_t lkey[AG_WAVES][AG_LDS];
    __shared__ uint16_t lidx[AG_WAVES][AG_LDS];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t = blockIdx.x * AG_WAVES + w;
    if (t >= n) return;   // whole wave; no block barriers below
    const uint32_t m = rcount[t];
    const uint64_t base = roff[t];
#if defined(TM_AGGRE_VARIANT) && TM_AGGRE_VARIANT == 1   // EXPERIMENT: launch + index loads only
    if (lane == 0) acount[t] = m;
    return;
#endif
    if (m <= 128) {
        const uint32_t c = aggre_regs(av, m, base, lane, src, dest, gkey, out_to, out_tg, out_cap);
        if (lane == 0) acount[t] = c;
        return;
    }
    if (m > AG_LDS) {
        if (lane == 0) large[1 + atomicAdd(&large[0], 1u)] = t;   // a block of tm_aggre_large takes it
        return;
    }
    // 129..AG_LDS routes: the wave's LDS row (a block per topic in
    // tm_aggre_large measured 0.94 ms for these at C3 vs ~0.3 ms here)
    const uint64_t* key = gkey + base;
    int j = -1;
    for (uint32_t i = lane; i < m; i += 64)
        if (av.dt[dest[base + i]].y & AG_GROUP_BIT) j = (int)i;
    j = wave_max_i(j);
    const uint32_t tail = (uint32_t)((int)m - 1 - j);   // j = -1: every route
    for (uint32_t k = lane; k < tail; k += 64) {        // r_{m-1} .. r_{j+1}, prepended by the fold
        const uint32_t i = m - 1 - k;
        if (base + k < out_cap) {
            out_to[base + k] = src[base + i];
            out_tg[base + k] = av.dt[dest[base + i]].y & ~AG_GROUP_BIT;
        }
    }
    uint32_t kept = 0;
    if (j >= 0) {
        const uint32_t u = (uint32_t)j + 1;
        uint32_t P = 1;
        while (P < u) P <<= 1;
        for (uint32_t i = lane; i < P; i += 64) {
            lkey[w][i] = i < u ? key[i] : ~0ull;
            lidx[w][i] = (uint16_t)i;
        }
        for (uint32_t size = 2; size <= P; size <<= 1) {
            for (uint32_t d = size >> 1; d > 0; d >>= 1) {
                __threadfence_block();
                __builtin_amdgcn_wave_barrier();
                for (uint32_t q = lane; q < P / 2; q += 64) {   // pair q: i has bit d clear
                    const uint32_t i = ((q & ~(d - 1)) << 1) | (q & (d - 1)), pi = i | d;
                    const uint64_t a = lkey[w][i], b = lkey[w][pi];
                    if ((a > b) == ((i & size) == 0)) {
                        lkey[w][i] = b;
                        lkey[w][pi] = a;
                        const uint16_t x = lidx[w][i];
                        lidx[w][i] = lidx[w][pi];
                        lidx[w][pi] = x;
                    }
                }
            }
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        for (uint32_t p0 = 0; p0 < u; p0 += 64) {
            const uint32_t p = p0 + lane;
            const bool keep = p < u && (p == 0 || lkey[w][p] != lkey[w][p - 1]);
            const uint64_t bal = __ballot(keep);
            if (keep) {
                const uint32_t pos = kept + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
                const uint32_t i = lidx[w][p];
                if (base + tail + pos < out_cap) {
                    out_to[base + tail + pos] = src[base + i];
                    out_tg[base + tail + pos] = av.dt[dest[base + i]].y & ~AG_GROUP_BIT;
                }
            }
            kept += (uint32_t)__popcll(bal);
        }
    }
    if (lane == 0) acount[t] = tail + kept;
}

// topics with more than 512 routes: one 256-thread block per topic
// (persistent over the list tm_aggre built), keys and route indices in LDS,
// block-wide bitonic sort; beyond AGL routes the topic's global key row is
// sorted in place and each surviving key names its pair through the inverse
// rank tables (AggreView::rank_src / rank_tg)
constexpr uint32_t AGL = 4096;

// ascending in-place sort of key[0..u) by one block (u > AGL).  Bitonic
// network in the "mirror" form (the first step of each merge compares i with
// its mirror image, later steps with i + d), whose comparators all point up:
// positions >= u act as +inf and never move, so no padding is needed.
// Steps of distance < AGL run on one LDS chunk at a time.
__device__ void sort_row_inplace(uint64_t* __restrict__ key, uint32_t u, uint64_t* lkey) {
    uint32_t P = AGL;
    while (P < u) P <<= 1;
    // compare-exchange (i < j), ascending
    auto cmpx = [](uint64_t* a, uint32_t i, uint32_t j) {
        const uint64_t x = a[i], y = a[j];
        if (x > y) {
            a[i] = y;
            a[j] = x;
        }
    };
    // pair p of a step: i has bit h clear (h = half the block for a mirror
    // step, the distance for a half-cleaner)
    auto lower = [](uint32_t p, uint32_t h) { return ((p & ~(h - 1)) << 1) | (p & (h - 1)); };
    auto mirror = [](uint32_t i, uint32_t s) { return (i & ~(s - 1)) + (s - 1) - (i & (s - 1)); };
    // one LDS chunk [c0, c0 + AGL): a full sort (full = true), or the
    // half-cleaners of distance < AGL that finish a global merge stage
    auto chunk_pass = [&](uint32_t c0, bool full) {
        for (uint32_t i = threadIdx.x; i < AGL; i += AG_BLOCK) lkey[i] = c0 + i < u ? key[c0 + i] : ~0ull;
        for (uint32_t s = full ? 2 : AGL; s <= AGL; s <<= 1) {
            if (full) {
                __syncthreads();
                for (uint32_t p = threadIdx.x; p < AGL / 2; p += AG_BLOCK) {
                    const uint32_t i = lower(p, s >> 1);
                    cmpx(lkey, i, mirror(i, s));
                }
            }
            for (uint32_t d = s >> (full ? 2 : 1); d > 0; d >>= 1) {
                __syncthreads();
                for (uint32_t p = threadIdx.x; p < AGL / 2; p += AG_BLOCK) {
                    const uint32_t i = lower(p, d);
                    cmpx(lkey, i, i | d);
                }
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < AGL; i += AG_BLOCK)
            if (c0 + i < u) key[c0 + i] = lkey[i];
        __threadfence_block();
        __syncthreads();
    };
    for (uint32_t c0 = 0; c0 < u; c0 += AGL) chunk_pass(c0, true);   // sorted runs of AGL
    for (uint32_t size = 2 * AGL; size <= P; size <<= 1) {
        for (uint32_t d = size >> 1; d >= AGL; d >>= 1) {
            for (uint32_t p = threadIdx.x; p < P / 2; p += AG_BLOCK) {
                const uint32_t i = lower(p, d);
                const uint32_t j = d == (size >> 1) ? mirror(i, size) : (i | d);
                if (j < u) cmpx(key, i, j);   // positions >= u are +inf: never move
            }
            __threadfence_block();
            __syncthreads();
        }
        for (uint32_t c0 = 0; c0 < u; c0 += AGL) chunk_pass(c0, false);
    }
}

__device__ __forceinline__ int block_max_i(int x, int* red) {
    x = wave_max_i(x);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
    __syncthreads();
    int r = red[0];
    for (int i = 1; i < AG_WAVES; ++i) r = max(r, red[i]);
    __syncthreads();
    return r;
}
// exclusive prefix of a 0/1 flag over the block, and the block total
__device__ __forceinline__ uint32_t block_prefix_flag(bool f, uint32_t* red, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t bal = __ballot(f);
    if (lane == 0) red[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t i = 0; i < (uint32_t)AG_WAVES; ++i) {
        if (i < w) pre += red[i];
        tot += red[i];
    }
    __syncthreads();
    total = tot;
    return pre + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
}

__global__ void __launch_bounds__(AG_BLOCK)
tm_aggre_large(AggreView av, const uint32_t* __restrict__ rcount, const uint64_t* __restrict__ roff,
               const uint32_t* __restrict__ src, const uint32_t* __restrict__ dest,
               uint64_t* __restrict__ gkey, const uint32_t* __restrict__ large,
               uint32_t* __restrict__ acount, uint32_t* __restrict__ out_to, uint32_t* __restrict__ out_tg,
               uint64_t out_cap) {
    __shared__ uint64_t lkey[AGL];
    __shared__ uint16_t lidx[AGL];
    __shared__ int redi[AG_WAVES];
    __shared__ uint32_t redu[AG_WAVES];
    const uint32_t nl = large[0];
    for (uint32_t q = blockIdx.x; q < nl; q += gridDim.x) {   // block-uniform
        const uint32_t t = large[1 + q];
        const uint32_t m = rcount[t];
        const uint64_t base = roff[t];
        const uint64_t* key = gkey + base;
        int j = -1;
        for (uint32_t i = threadIdx.x; i < m; i += AG_BLOCK)
            if (av.dt[dest[base + i]].y & AG_GROUP_BIT) j = (int)i;
        j = block_max_i(j, redi);
        const uint32_t tail = (uint32_t)((int)m - 1 - j);
        for (uint32_t k = threadIdx.x; k < tail; k += AG_BLOCK) {   // r_{m-1} .. r_{j+1}
            const uint32_t i = m - 1 - k;
            if (base + k < out_cap) {
                out_to[base + k] = src[base + i];
                out_tg[base + k] = av.dt[dest[base + i]].y & ~AG_GROUP_BIT;
            }
        }
        uint32_t kept = 0;
        const uint32_t u = (uint32_t)(j + 1);
        if (j >= 0 && u <= AGL) {
            uint32_t P = 1;
            while (P < u) P <<= 1;
            for (uint32_t i = threadIdx.x; i < P; i += AG_BLOCK) {
                lkey[i] = i < u ? key[i] : ~0ull;
                lidx[i] = (uint16_t)i;
            }
            for (uint32_t size = 2; size <= P; size <<= 1) {
                for (uint32_t d = size >> 1; d > 0; d >>= 1) {
                    __syncthreads();
                    for (uint32_t p = threadIdx.x; p < P / 2; p += AG_BLOCK) {   // pair p: i has bit d clear
                        const uint32_t i = ((p & ~(d - 1)) << 1) | (p & (d - 1)), pi = i | d;
                        const uint64_t a = lkey[i], b = lkey[pi];
                        if ((a > b) == ((i & size) == 0)) {
                            lkey[i] = b;
                            lkey[pi] = a;
                            const uint16_t x = lidx[i];
                            lidx[i] = lidx[pi];
                            lidx[pi] = x;
                        }
                    }
                }
            }
            __syncthreads();
            for (uint32_t p0 = 0; p0 < u; p0 += AG_BLOCK) {   // block-uniform trip count
                const uint32_t p = p0 + threadIdx.x;
                const bool keep = p < u && (p == 0 || lkey[p] != lkey[p - 1]);
                uint32_t chunk;
                const uint32_t pos = kept + block_prefix_flag(keep, redu, chunk);
                if (keep && base + tail + pos < out_cap) {
                    const uint32_t i = lidx[p];
                    out_to[base + tail + pos] = src[base + i];
                    out_tg[base + tail + pos] = av.dt[dest[base + i]].y & ~AG_GROUP_BIT;
                }
                kept += chunk;
            }
        } else if (j >= 0) {
            // the key row of r_0 .. r_j sorted in place; a kept key is the
            // first of its run and names its {To, X} by its two ranks
            uint64_t* krow = gkey + base;
            sort_row_inplace(krow, u, lkey);
            for (uint32_t p0 = 0; p0 < u; p0 += AG_BLOCK) {   // block-uniform trip count
                const uint32_t p = p0 + threadIdx.x;
                const uint64_t kx = p < u ? krow[p] : 0ull;
                const bool keep = p < u && (p == 0 || krow[p - 1] != kx);
                uint32_t chunk;
                const uint32_t pos = kept + block_prefix_flag(keep, redu, chunk);
                if (keep && base + tail + pos < out_cap) {
                    out_to[base + tail + pos] = av.rank_src[(uint32_t)(kx >> 32)];
                    out_tg[base + tail + pos] = av.rank_tg[(uint32_t)kx];
                }
                kept += chunk;
            }
        }
        if (threadIdx.x == 0) acount[t] = tail + kept;
        __syncthreads();   // LDS and redu reused by the next topic
    }
}

hipError_t launch_aggre(const AggreView& av, uint32_t n, const uint32_t* rcount, const uint64_t* roff,
                        const uint32_t* src, const uint32_t* dest, uint64_t* key, uint32_t* large,
                        uint32_t* acount, uint32_t* out_to, uint32_t* out_tg, uint64_t out_cap, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipError_t err = hipMemsetAsync(large, 0, 4, st);
    if (err != hipSuccess) return err;
    const dim3 g((n + AG_WAVES - 1) / AG_WAVES), blk(AG_BLOCK);
    hipLaunchKernelGGL(tm_aggre, g, blk, 0, st, av, n, rcount, roff, src, dest, key, large, acount, out_to, out_tg,
                       out_cap);
    // persistent: 4 blocks per CU (40 KB of LDS each) over 256 CUs
    const dim3 gl(n < 1024u ? n : 1024u);
    hipLaunchKernelGGL(tm_aggre_large, gl, blk, 0, st, av, rcount, roff, src, dest, key, large, acount,
                       out_to, out_tg, out_cap);
    return hipGetLastError();
}

}  // namespace tmx
