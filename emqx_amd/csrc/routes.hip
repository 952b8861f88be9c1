// routes.hip — emqx_router:match_routes/1 on the device:
//
//   match_routes(Topic) ->
//       Matched = mnesia:ets(fun emqx_trie:match/1, [Topic]),
//       lists:append([get_routes(To) || To <- [Topic | Matched]]).
//                                              (src/emqx_router.erl:116-118)
//
// Given a batch's ordered match lists (CSR of filter ids from the walk), the
// route image (image.h RouteView) expands every topic into its routes: first the
// routes of the literal topic (get_routes(Topic), :89-90, an exact-topic
// hash table verified byte for byte), then, for each matched filter in
// emqx_trie:match/1 order, that filter's routes (its emqx_route bag, in
// insertion order).  Output: per-topic counts and offsets, and per route the
// source (filter id, or TM_ROUTE_TOPIC_ID for the literal topic) and dest id,
// and, for aggre (aggre.hip), each route's sort key to_rank << 32 | target
// rank: a filter's to_rank shares the 16 B fr_meta entry the emit reads anyway
// (a literal topic's, its exact slot), so the keys cost no extra random loads.
//
// Two passes over blocks of 256 topics (the ids of a block are a contiguous
// CSR range, read coalesced): count, scan, emit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "image.h"
#include "kernels.h"

namespace tmx {

constexpr int RBLOCK = 256;

__device__ __forceinline__ uint64_t r_load_u64_aligned(const uint8_t* base, uint64_t p) {
    return *reinterpret_cast<const uint64_t*>(base + (p & ~7ull));
}
// bytes [p, p+k) (k in 1..8) little-endian, zero padded
__device__ __forceinline__ uint64_t r_load_chunk(const uint8_t* base, uint64_t p, uint32_t k) {
    const uint32_t sh = (uint32_t)(p & 7) * 8;
    uint64_t v = r_load_u64_aligned(base, p) >> sh;
    if (sh != 0 && (p & 7) + k > 8) v |= r_load_u64_aligned(base, p + 8) << (64 - sh);
    if (k < 8) v &= (~0ull) >> (64 - 8 * k);
    return v;
}

// get_routes(Topic) (emqx_router.erl:89-90): the exact-topic table slot of
// topic bytes [p, p+len), byte-verified; returns (dest offset, count, to_rank)
__device__ __forceinline__ uint4 exact_lookup(const RouteView& rv, const uint8_t* bytes, uint64_t p, uint32_t len) {
    if (!rv.ex_slots) return make_uint4(0, 0, 0, 0);
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (uint32_t i = 0; i < len; i += 8) {
        const uint32_t k = len - i < 8 ? len - i : 8;
        h = word_hash_step(h, r_load_chunk(bytes, p + i, k));
    }
    h = word_hash_final(h, len);
    for (uint64_t s = h & rv.ex_slot_mask;; s = (s + 1) & rv.ex_slot_mask) {
        const ExactSlot e = rv.ex_slots[s];
        if (e.hash == 0) return make_uint4(0, 0, 0, 0);
        if (e.hash == h && e.len == len) {
            const uint64_t* a = reinterpret_cast<const uint64_t*>(rv.ex_arena + e.arena);
            bool eq = true;
            for (uint32_t i = 0; i < len && eq; i += 8) {
                const uint32_t k = len - i < 8 ? len - i : 8;
                eq = r_load_chunk(bytes, p + i, k) == a[i >> 3];
            }
            if (eq) return make_uint4(e.dest_off, e.count, e.rank, 0);
        }
    }
}

__device__ __forceinline__ uint64_t r_block_exclusive_scan(uint64_t x, uint64_t* lds, uint64_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t inc = x;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    uint64_t wpre = 0, tot = 0;
    for (int i = 0; i < RBLOCK / 64; ++i) {
        if (i < wid) wpre += lds[i];
        tot += lds[i];
    }
    __syncthreads();
    total = tot;
    return wpre + inc - x;
}

// local topic of id j of the block: lds_inc holds the inclusive id prefix of
// the block's tn topics
__device__ __forceinline__ uint32_t topic_of(const uint32_t* lds_inc, uint32_t tn, uint64_t j) {
    uint32_t lo = 0, hi = tn - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((uint64_t)lds_inc[mid] > j) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// pass 1: per topic, exact-route slot and the total route count
__global__ void __launch_bounds__(RBLOCK)
tm_route_count(RouteView rv, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint32_t n,
               const uint32_t* __restrict__ counts, const uint64_t* __restrict__ ids_off,
               const uint32_t* __restrict__ ids, uint4* __restrict__ exact, uint32_t* __restrict__ rcount) {
    __shared__ uint32_t lds_inc[RBLOCK];
    __shared__ uint32_t lds_mr[RBLOCK];
    __shared__ uint64_t lds_scan[RBLOCK / 64];
    const uint32_t t0 = blockIdx.x * RBLOCK;
    const uint32_t tn = n - t0 < (uint32_t)RBLOCK ? n - t0 : (uint32_t)RBLOCK;
    const uint32_t t = t0 + threadIdx.x;
    const uint32_t c = threadIdx.x < tn ? counts[t] : 0u;
    uint64_t agg;
    const uint64_t ex = r_block_exclusive_scan(c, lds_scan, agg);
    lds_inc[threadIdx.x] = (uint32_t)(ex + c);
    lds_mr[threadIdx.x] = 0;
    uint4 xe = make_uint4(0, 0, 0, 0);
    if (threadIdx.x < tn) {
        xe = exact_lookup(rv, bytes, off[t], (uint32_t)(off[t + 1] - off[t]));
        exact[t] = xe;
    }
    __syncthreads();
    const uint64_t base = ids_off[t0];
    for (uint64_t j = threadIdx.x; j < agg; j += RBLOCK) {
        const uint32_t id = ids[base + j];
        const uint32_t rc = id < rv.n_filters ? rv.fr_meta[id].y : 0u;
        if (rc) atomicAdd(&lds_mr[topic_of(lds_inc, tn, j)], rc);
    }
    __syncthreads();
    if (threadIdx.x < tn) rcount[t] = xe.y + lds_mr[threadIdx.x];
}

// pass 2: routes of topic t at out_off[t]: its exact routes, then the
// routes of each matched filter in match order
__global__ void __launch_bounds__(RBLOCK)
tm_route_emit(RouteView rv, AggreView av, uint32_t n, const uint32_t* __restrict__ counts,
              const uint64_t* __restrict__ ids_off, const uint32_t* __restrict__ ids,
              const uint4* __restrict__ exact, const uint32_t* __restrict__ rcount,
              const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_src, uint32_t* __restrict__ out_dest,
              uint64_t* __restrict__ out_key, uint64_t out_cap) {
    __shared__ uint32_t lds_inc[RBLOCK];
    __shared__ uint64_t lds_m[RBLOCK];      // exclusive prefix of matched-route counts
    __shared__ uint64_t lds_scan[RBLOCK / 64];
    const uint32_t t0 = blockIdx.x * RBLOCK;
    const uint32_t tn = n - t0 < (uint32_t)RBLOCK ? n - t0 : (uint32_t)RBLOCK;
    const uint32_t t = t0 + threadIdx.x;
    const uint32_t c = threadIdx.x < tn ? counts[t] : 0u;
    uint64_t agg;
    const uint64_t ex = r_block_exclusive_scan(c, lds_scan, agg);
    lds_inc[threadIdx.x] = (uint32_t)(ex + c);
    const uint4 xe = threadIdx.x < tn ? exact[t] : make_uint4(0, 0, 0, 0);
    const uint32_t mr = threadIdx.x < tn ? rcount[t] - xe.y : 0u;
    uint64_t magg;
    lds_m[threadIdx.x] = r_block_exclusive_scan(mr, lds_scan, magg);
    if (threadIdx.x < tn) {   // get_routes(Topic): the literal topic's routes first
        const uint64_t o = out_off[t];
        const uint64_t xr = (uint64_t)xe.z << 32;
        for (uint32_t k = 0; k < xe.y; ++k)
            if (o + k < out_cap) {
                const uint32_t d = rv.dest[xe.x + k];
                out_src[o + k] = TM_ROUTE_TOPIC_ID;
                out_dest[o + k] = d;
                if (out_key) out_key[o + k] = xr | av.dt[d].x;
            }
    }
    __syncthreads();
    const uint64_t base = ids_off[t0];
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < agg; c0 += RBLOCK) {   // block-uniform trip count
        const uint64_t j = c0 + threadIdx.x;
        uint32_t id = 0, rc = 0, fo = 0, lo = 0, fr = 0;
        if (j < agg) {
            id = ids[base + j];
            lo = topic_of(lds_inc, tn, j);
            if (id < rv.n_filters) {
                const uint4 fm = rv.fr_meta[id];   // one 16 B load: segment, count, to_rank
                fo = fm.x;
                rc = fm.y;
                fr = fm.z;
            }
        }
        uint64_t chunk;
        const uint64_t r = carry + r_block_exclusive_scan(rc, lds_scan, chunk);
        if (rc) {
            const uint32_t tl = t0 + lo;
            const uint64_t pos = out_off[tl] + exact[tl].y + (r - lds_m[lo]);
            for (uint32_t k = 0; k < rc; ++k)
                if (pos + k < out_cap) {
                    const uint32_t d = rv.dest[fo + k];
                    out_src[pos + k] = id;
                    out_dest[pos + k] = d;
                    if (out_key) out_key[pos + k] = ((uint64_t)fr << 32) | av.dt[d].x;
                }
        }
        carry += chunk;
    }
}

static inline uint32_t rdiv_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_routes(const RouteView& rv, const uint8_t* bytes, const uint64_t* off, uint32_t n,
                         const uint32_t* counts, const uint64_t* ids_off, const uint32_t* ids, uint4* exact,
                         uint32_t* rcount, uint64_t* out_off, uint32_t* out_src, uint32_t* out_dest,
                         uint64_t out_cap, uint64_t* total, uint64_t* scan_tmp, hipStream_t st, const AggreView* av,
                         uint64_t* out_key) {
    if (n == 0) {
        hipError_t err = hipMemsetAsync(out_off, 0, 8, st);
        return err == hipSuccess ? hipMemsetAsync(total, 0, 8, st) : err;
    }
    const dim3 g(rdiv_up(n, RBLOCK)), blk(RBLOCK);
    hipLaunchKernelGGL(tm_route_count, g, blk, 0, st, rv, bytes, off, n, counts, ids_off, ids, exact, rcount);
    hipError_t err = launch_scan(rcount, n, out_off, total, scan_tmp, st);
    if (err != hipSuccess) return err;
    if (out_cap)
        hipLaunchKernelGGL(tm_route_emit, g, blk, 0, st, rv, av ? *av : AggreView{nullptr, nullptr, nullptr}, n, counts,
                           ids_off, ids, exact, rcount, out_off, out_src, out_dest, av ? out_key : nullptr, out_cap);
    return hipGetLastError();
}

}  // namespace tmx
