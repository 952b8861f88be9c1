// route.hip — the routed sharded mode's device side (topicmatch.h
// tm_route_exchange / tm_route_return).  Every rank routes its
// own publish batch: each topic goes to the shard that owns its first `depth`
// levels (the shard holding every filter that can match it, so the owner's
// walk alone is emqx_trie:match/1's whole list, src/emqx_trie.erl:121-145).
//
//   tm_route_count    owner of each topic (the word hash of its routing key,
//                     as the host's tm_route_of) and per-block counts per owner
//   tm_route_bases    per-owner exclusive scan over the blocks: each block's
//                     first position in every owner's bucket
//   tm_route_scatter  the stable bucket order: perm[pos] = topic, slen[pos]
//   tm_route_bytes    topic bytes into bucket order (after a scan of slen)
//   tm_gather_u64     out[k] = in[idx[k]] (cut points read back by the host)
//   tm_route_unpermute / tm_route_lists   the returned lists back in the
//                     source batch's own topic order
//
// Integer/byte work over HBM-resident batches; no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "image.h"
#include "kernels.h"

namespace tmx {

namespace {

constexpr int RB = 256;   // threads per block of the routing kernels

// little-endian bytes [p, p+k) (k in 1..8) of an 8-byte-readable buffer
__device__ __forceinline__ uint64_t chunk_at(const uint8_t* b, uint64_t p, uint32_t k) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(b + (p & ~7ull));
    const uint32_t sh = (uint32_t)(p & 7) * 8;
    uint64_t v = w[0] >> sh;
    if (sh && (p & 7) + k > 8) v |= w[1] << (64 - sh);
    if (k < 8) v &= (~0ull) >> (64 - 8 * k);
    return v;
}

// the owner shard of topic [b, e): word hash of its first `depth` levels
__device__ __forceinline__ uint32_t topic_owner(const uint8_t* bytes, uint64_t b, uint64_t e, uint32_t depth,
                                                uint32_t S) {
    uint64_t cut = e;
    uint32_t lev = 0;
    for (uint64_t q = b; q < e; ++q) {
        if (bytes[q] == '/' && ++lev == depth) {
            cut = q;
            break;
        }
    }
    const uint32_t len = (uint32_t)(cut - b);
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (uint32_t i = 0; i < len; i += 8) h = word_hash_step(h, chunk_at(bytes, b + i, len - i < 8 ? len - i : 8));
    return route_shard(word_hash_final(h, len), S);
}

__global__ void __launch_bounds__(RB)
tm_route_count(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint32_t n, uint32_t depth,
               uint32_t S, uint8_t* __restrict__ owner, uint32_t* __restrict__ blk_cnt) {
    __shared__ uint32_t cnt[MAX_ROUTE_SHARDS];
    for (uint32_t k = threadIdx.x; k < S; k += RB) cnt[k] = 0;
    __syncthreads();
    const uint32_t t = blockIdx.x * RB + threadIdx.x;
    if (t < n) {
        const uint32_t o = topic_owner(bytes, off[t], off[t + 1], depth, S);
        owner[t] = (uint8_t)o;
        atomicAdd(&cnt[o], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < S; k += RB) blk_cnt[(uint64_t)blockIdx.x * S + k] = cnt[k];
}

// one block: blk_cnt[b][o] -> blk_base[b][o] (first position of block b's
// topics of owner o in the bucket order), bucket[o] (first position of owner
// o's bucket), bucket[S] = n
__global__ void __launch_bounds__(RB)
tm_route_bases(const uint32_t* __restrict__ blk_cnt, uint32_t nb, uint32_t S, uint32_t* __restrict__ blk_base,
               uint32_t* __restrict__ bucket) {
    __shared__ uint32_t tot[MAX_ROUTE_SHARDS];
    __shared__ uint32_t part[RB];
    // per owner: the blocks cut into RB contiguous runs, one per thread
    const uint32_t per = (nb + RB - 1) / RB;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
    for (uint32_t o = 0; o < S; ++o) {
        uint32_t s = 0;
        for (uint32_t b = lo; b < hi; ++b) s += blk_cnt[(uint64_t)b * S + o];
        part[threadIdx.x] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int i = 0; i < RB; ++i) {
                const uint32_t x = part[i];
                part[i] = run;
                run += x;
            }
            tot[o] = run;
        }
        __syncthreads();
        uint32_t run = part[threadIdx.x];
        for (uint32_t b = lo; b < hi; ++b) {
            const uint32_t x = blk_cnt[(uint64_t)b * S + o];
            blk_base[(uint64_t)b * S + o] = run;
            run += x;
        }
        __syncthreads();
    }
    __shared__ uint32_t sb[MAX_ROUTE_SHARDS + 1];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t o = 0; o < S; ++o) {
            sb[o] = run;
            run += tot[o];
        }
        sb[S] = run;
    }
    __syncthreads();
    // bucket bases folded into the block bases (each thread into the entries it wrote)
    for (uint32_t b = lo; b < hi; ++b)
        for (uint32_t o = 0; o < S; ++o) blk_base[(uint64_t)b * S + o] += sb[o];
    if (threadIdx.x <= S) bucket[threadIdx.x] = sb[threadIdx.x];
}

// stable positions: block base + the topic's rank among the block's earlier
// topics of its owner (per-wave ballots, wave prefix in LDS)
__global__ void __launch_bounds__(RB)
tm_route_scatter(const uint64_t* __restrict__ off, uint32_t n, uint32_t S, const uint8_t* __restrict__ owner,
                 const uint32_t* __restrict__ blk_base, uint32_t* __restrict__ perm, uint32_t* __restrict__ slen) {
    __shared__ uint32_t wcnt[RB / 64][MAX_ROUTE_SHARDS];
    const uint32_t t = blockIdx.x * RB + threadIdx.x;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t o = t < n ? owner[t] : 0xFFFFFFFFu;
    uint32_t my_rank = 0;
    for (uint32_t k = 0; k < S; ++k) {
        const uint64_t m = __ballot(o == k);
        if (o == k)
            my_rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == 0) wcnt[wv][k] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (t < n) {
        uint32_t before = 0;
        for (uint32_t w = 0; w < wv; ++w) before += wcnt[w][o];
        const uint32_t pos = blk_base[(uint64_t)blockIdx.x * S + o] + before + my_rank;
        perm[pos] = t;
        slen[pos] = (uint32_t)(off[t + 1] - off[t]);
    }
}

// topic bytes into bucket order: position p's topic perm[p] to sbuf[soff[p]..)
__global__ void __launch_bounds__(RB)
tm_route_bytes(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint32_t n,
               const uint32_t* __restrict__ perm, const uint64_t* __restrict__ soff, uint8_t* __restrict__ sbuf) {
    const uint32_t p = blockIdx.x * RB + threadIdx.x;
    if (p >= n) return;
    const uint32_t t = perm[p];
    const uint64_t b = off[t], len = off[t + 1] - b, d = soff[p];
    for (uint64_t i = 0; i < len; i += 8) {
        const uint32_t k = len - i < 8 ? (uint32_t)(len - i) : 8u;
        const uint64_t v = chunk_at(bytes, b + i, k);
        for (uint32_t j = 0; j < k; ++j) sbuf[d + i + j] = (uint8_t)(v >> (8 * j));
    }
}

__global__ void tm_gather_u64(const uint64_t* __restrict__ in, const uint32_t* __restrict__ idx, uint32_t k,
                              uint64_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) out[i] = in[idx[i]];
}

// returned counts (bucket order) -> the source's topic order
__global__ void __launch_bounds__(RB)
tm_route_unpermute(const uint32_t* __restrict__ rcount, const uint32_t* __restrict__ perm, uint32_t n,
                   uint32_t* __restrict__ out_count) {
    const uint32_t p = blockIdx.x * RB + threadIdx.x;
    if (p < n) out_count[perm[p]] = rcount[p];
}

// returned lists (bucket order, CSR roff) -> the source's CSR: one wave per
// position, lanes over the ids
__global__ void __launch_bounds__(RB)
tm_route_lists(const uint32_t* __restrict__ rcount, const uint64_t* __restrict__ roff,
               const uint32_t* __restrict__ rids, const uint32_t* __restrict__ perm, uint32_t n,
               const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_ids) {
    const uint32_t p = blockIdx.x * (RB / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (p >= n) return;
    const uint32_t c = rcount[p];
    const uint64_t s = roff[p], d = out_off[perm[p]];
    for (uint32_t i = lane; i < c; i += 64) out_ids[d + i] = rids[s + i];
}

inline uint32_t blocks_of(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

}  // namespace

hipError_t launch_scan0(const uint32_t* counts, uint32_t n, uint64_t* out_off, uint64_t* total, uint64_t* tmp,
                        hipStream_t st) {
    if (n) return launch_scan(counts, n, out_off, total, tmp, st);
    hipError_t err = hipMemsetAsync(out_off, 0, 8, st);   // an empty batch: offsets {0}, total 0
    if (err == hipSuccess && total != out_off) err = hipMemsetAsync(total, 0, 8, st);
    return err;
}

hipError_t launch_route_plan(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t depth, uint32_t S,
                             const RoutePlanBufs& w, hipStream_t st) {
    if (S == 0 || S > MAX_ROUTE_SHARDS) return hipErrorInvalidValue;
    const uint32_t nb = n ? blocks_of(n, RB) : 0;
    if (n) {
        hipLaunchKernelGGL(tm_route_count, dim3(nb), dim3(RB), 0, st, bytes, off, n, depth, S, w.owner, w.blk_cnt);
    }
    hipLaunchKernelGGL(tm_route_bases, dim3(1), dim3(RB), 0, st, w.blk_cnt, nb, S, w.blk_base, w.bucket);
    if (n) {
        hipLaunchKernelGGL(tm_route_scatter, dim3(nb), dim3(RB), 0, st, off, n, S, w.owner, w.blk_base, w.perm,
                           w.slen);
    }
    hipError_t err = launch_scan0(w.slen, n, w.soff, w.soff + n, w.scan_tmp, st);
    if (err != hipSuccess) return err;
    if (n) hipLaunchKernelGGL(tm_route_bytes, dim3(nb), dim3(RB), 0, st, bytes, off, n, w.perm, w.soff, w.sbuf);
    // byte cut of every bucket: soff[bucket[o]], o = 0..S (S + 1 = 65 entries
    // at MAX_ROUTE_SHARDS: more than one 64-lane block)
    return launch_gather_u64(w.soff, w.bucket, S + 1, w.cuts, st);
}

hipError_t launch_gather_u64(const uint64_t* in, const uint32_t* idx, uint32_t k, uint64_t* out, hipStream_t st) {
    if (k) hipLaunchKernelGGL(tm_gather_u64, dim3(blocks_of(k, 64)), dim3(64), 0, st, in, idx, k, out);
    return hipGetLastError();
}

hipError_t launch_route_unpermute(const uint32_t* rcount, const uint64_t* roff, const uint32_t* rids,
                                  const uint32_t* perm, uint32_t n, uint32_t* out_count, uint64_t* out_off,
                                  uint32_t* out_ids, uint64_t* total, uint64_t* scan_tmp, hipStream_t st) {
    if (n) hipLaunchKernelGGL(tm_route_unpermute, dim3(blocks_of(n, RB)), dim3(RB), 0, st, rcount, perm, n, out_count);
    hipError_t err = launch_scan0(out_count, n, out_off, total, scan_tmp, st);
    if (err != hipSuccess) return err;
    if (n && out_ids)
        hipLaunchKernelGGL(tm_route_lists, dim3(blocks_of(n, RB / 64)), dim3(RB), 0, st, rcount, roff, rids, perm, n,
                           out_off, out_ids);
    return hipGetLastError();
}

}  // namespace tmx
