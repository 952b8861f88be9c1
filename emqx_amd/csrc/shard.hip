// shard.hip — merge of per-shard match lists (sharded mode).
//
// With the filter set partitioned over S GPUs (emqx_amd/shard.py), every
// shard walks the whole topic batch against its own sub-trie and emits each
// topic's matches in descending order key (kernels.hip, rank_sym): the key
// packs the branches the reference's fold took (emqx_trie.erl:127-145), so
// the union of the shards' lists in descending key order IS the order
// emqx_trie:match/1 returns over the whole filter set.  After the all-to-all
// exchange each GPU holds, for its slice of m topics, S sorted lists; this
// kernel merges them (one lane per topic, S <= 8 heads in registers).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

namespace tmx {

constexpr int MBLOCK = 256;

__global__ void __launch_bounds__(MBLOCK)
tm_shard_sum(uint32_t S, uint32_t m, const uint32_t* __restrict__ counts, uint32_t* __restrict__ out_count) {
    const uint32_t t = blockIdx.x * MBLOCK + threadIdx.x;
    if (t >= m) return;
    uint32_t c = 0;
    for (uint32_t s = 0; s < S; ++s) c += counts[(uint64_t)s * m + t];
    out_count[t] = c;
}

__global__ void __launch_bounds__(MBLOCK)
tm_shard_merge(uint32_t S, uint32_t m, const uint32_t* __restrict__ counts, const uint64_t* __restrict__ src_base,
               const uint64_t* __restrict__ pre, const uint32_t* __restrict__ ids, const uint64_t* __restrict__ keys,
               const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_gid, uint64_t out_cap) {
    const uint32_t t = blockIdx.x * MBLOCK + threadIdx.x;
    if (t >= m) return;
    // heads (next item) and ends of the S lists; head keys cached; unrolled
    // over MAX_SHARDS so every array stays in VGPRs
    uint64_t h[MAX_SHARDS], e[MAX_SHARDS], hk[MAX_SHARDS];
#pragma unroll
    for (uint32_t s = 0; s < MAX_SHARDS; ++s) {
        h[s] = e[s] = 0;
        hk[s] = 0;
        if (s < S) {
            h[s] = src_base[s] + pre[(uint64_t)s * (m + 1) + t];
            e[s] = h[s] + counts[(uint64_t)s * m + t];
            if (h[s] < e[s]) hk[s] = keys[h[s]];
        }
    }
    uint64_t o = out_off[t];
    for (;;) {
        uint32_t best = MAX_SHARDS;
        uint64_t bk = 0;
#pragma unroll
        for (uint32_t s = 0; s < MAX_SHARDS; ++s) {
            const bool live = h[s] < e[s];
            if (live && (best == MAX_SHARDS || hk[s] > bk)) {   // keys of one topic are distinct
                best = s;
                bk = hk[s];
            }
        }
        if (best == MAX_SHARDS) break;
#pragma unroll
        for (uint32_t s = 0; s < MAX_SHARDS; ++s) {
            if (s == best) {
                if (o < out_cap) out_gid[o] = ids[h[s]] * S + s;
                ++h[s];
                if (h[s] < e[s]) hk[s] = keys[h[s]];
            }
        }
        ++o;
    }
}

static inline uint32_t mdiv_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_shard_merge(uint32_t S, uint32_t m, const uint32_t* counts, const uint64_t* src_base,
                              const uint32_t* ids, const uint64_t* keys, uint32_t* out_count, uint64_t* out_off,
                              uint32_t* out_gid, uint64_t out_cap, uint64_t* total, uint64_t* pre, uint64_t* tmp,
                              hipStream_t st) {
    if (S == 0 || S > MAX_SHARDS) return hipErrorInvalidValue;
    if (m == 0) {
        hipError_t err = hipMemsetAsync(out_off, 0, 8, st);
        return err == hipSuccess ? hipMemsetAsync(total, 0, 8, st) : err;
    }
    for (uint32_t s = 0; s < S; ++s) {
        // per-source exclusive prefix of its counts (its total lands in pre's last slot)
        uint64_t* p = pre + (uint64_t)s * (m + 1);
        hipError_t err = launch_scan(counts + (uint64_t)s * m, m, p, p + m, tmp, st);
        if (err != hipSuccess) return err;
    }
    hipLaunchKernelGGL(tm_shard_sum, dim3(mdiv_up(m, MBLOCK)), dim3(MBLOCK), 0, st, S, m, counts, out_count);
    hipError_t err = launch_scan(out_count, m, out_off, total, tmp, st);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(tm_shard_merge, dim3(mdiv_up(m, MBLOCK)), dim3(MBLOCK), 0, st, S, m, counts, src_base, pre,
                       ids, keys, out_off, out_gid, out_cap);
    return hipGetLastError();
}

}  // namespace tmx
