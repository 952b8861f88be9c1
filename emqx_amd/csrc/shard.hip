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

// One wave per topic.  Item i of the topic's S concatenated lists (each in
// descending key order) belongs to source s with ls[s] <= i < ls[s+1]; its
// output position is its index in its own list plus, for every other list,
// the number of keys greater than its own (binary search).  Keys of one
// topic are distinct, so positions are a permutation.  The wave loads all
// items of the topic at once (one round trip) into LDS, searches there, and
// writes every id once; a topic beyond MCAP ids searches the lists in global
// memory instead (L2-resident after the first touch).  Keys of KW > 1 words
// (topics of 32+ levels, kernels.hip key_word) sit in KW planes kstride
// apart and are compared word by word in global memory.
constexpr uint32_t MCAP = 512;   // ids of one topic staged in LDS (6 KB)

// number of keys in list a[0..len) (descending, KW words, planes kstride
// apart) greater than the key at b
__device__ __forceinline__ uint32_t count_greater_w(const uint64_t* keys, uint64_t kstride, uint32_t KW, uint64_t a,
                                                    uint32_t len, uint64_t b) {
    uint32_t lo = 0, hi = len;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        bool gt = false;
        for (uint32_t j = 0; j < KW; ++j) {
            const uint64_t x = keys[j * kstride + a + mid], y = keys[j * kstride + b];
            if (x != y) {
                gt = x > y;
                break;
            }
        }
        if (gt) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

template <class Keys>
__device__ __forceinline__ uint32_t count_greater(const Keys& a, uint32_t len, uint64_t key) {
    uint32_t lo = 0, hi = len;   // a[] descending: first index with a[i] <= key
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] > key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(64)
tm_shard_merge(uint32_t S, uint32_t m, const uint32_t* __restrict__ counts, const uint64_t* __restrict__ src_base,
               const uint64_t* __restrict__ pre, const uint32_t* __restrict__ ids, const uint64_t* __restrict__ keys,
               const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out_gid, uint64_t out_cap, uint32_t KW,
               uint64_t kstride) {
    __shared__ uint64_t lk[MCAP];
    __shared__ uint32_t lg[MCAP];
    const uint32_t lane = threadIdx.x;
    for (uint32_t t = blockIdx.x; t < m; t += gridDim.x) {
        // lane s < S: head of source s's list for t and its length
        uint64_t hs = 0;
        uint32_t cs = 0;
        if (lane < S) {
            cs = counts[(uint64_t)lane * m + t];
            hs = src_base[lane] + pre[(uint64_t)lane * m + t] - pre[(uint64_t)lane * m];
        }
        // every source's (length, start in the topic, head) in registers of
        // every lane, read while the whole wave is active
        uint32_t ns[MAX_SHARDS], ls[MAX_SHARDS];
        uint64_t hh[MAX_SHARDS];
        uint32_t c = 0;
#pragma unroll
        for (uint32_t s = 0; s < MAX_SHARDS; ++s) {
            ns[s] = s < S ? (uint32_t)__shfl((int)cs, (int)s, 64) : 0u;
            hh[s] = s < S ? (uint64_t)__shfl((long long)hs, (int)s, 64) : 0ull;
            ls[s] = c;
            c += ns[s];
        }
        const uint64_t o = out_off[t];
        // item i -> (source s, index j in s's list, global position)
        auto locate = [&](uint32_t i, uint32_t& s, uint32_t& j, uint64_t& g) {
            s = 0;
            j = i;
            g = hh[0] + i;
#pragma unroll
            for (uint32_t q = 1; q < MAX_SHARDS; ++q)
                if (q < S && i >= ls[q]) {
                    s = q;
                    j = i - ls[q];
                    g = hh[q] + j;
                }
        };
        if (KW > 1) {
            for (uint32_t i = lane; i < c; i += 64) {
                uint32_t s, j;
                uint64_t g;
                locate(i, s, j, g);
                uint32_t r = j;
                for (uint32_t s2 = 0; s2 < S; ++s2)
                    if (s2 != s && ns[s2]) r += count_greater_w(keys, kstride, KW, hh[s2], ns[s2], g);
                if (o + r < out_cap) out_gid[o + r] = ids[g] * S + s;
            }
        } else if (c <= MCAP) {
            for (uint32_t i = lane; i < c; i += 64) {
                uint32_t s, j;
                uint64_t g;
                locate(i, s, j, g);
                lk[i] = keys[g];
                lg[i] = ids[g] * S + s;
            }
            __syncthreads();
            for (uint32_t i = lane; i < c; i += 64) {
                uint32_t s, j;
                uint64_t g;
                locate(i, s, j, g);
                const uint64_t key = lk[i];
                uint32_t r = j;
#pragma unroll
                for (uint32_t s2 = 0; s2 < MAX_SHARDS; ++s2)
                    if (s2 != s && ns[s2]) r += count_greater(lk + ls[s2], ns[s2], key);
                if (o + r < out_cap) out_gid[o + r] = lg[i];
            }
            __syncthreads();
        } else {
            for (uint32_t i = lane; i < c; i += 64) {
                uint32_t s, j;
                uint64_t g;
                locate(i, s, j, g);
                const uint64_t key = keys[g];
                uint32_t r = j;
#pragma unroll
                for (uint32_t s2 = 0; s2 < MAX_SHARDS; ++s2)
                    if (s2 != s && ns[s2]) r += count_greater(keys + hh[s2], ns[s2], key);
                if (o + r < out_cap) out_gid[o + r] = ids[g] * S + s;
            }
        }
    }
}

// one shard: its list of every topic is already in order, and gid = id
// (local * 1 + 0): the merge is a copy of the received block
__global__ void __launch_bounds__(MBLOCK)
tm_shard_copy1(const uint64_t* __restrict__ src_base, const uint32_t* __restrict__ ids,
               const uint64_t* __restrict__ total, uint32_t* __restrict__ out_gid, uint64_t out_cap) {
    const uint64_t nt = *total < out_cap ? *total : out_cap;
    const uint32_t* src = ids + src_base[0];
    for (uint64_t i = (uint64_t)blockIdx.x * MBLOCK + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * MBLOCK)
        out_gid[i] = src[i];
}

static inline uint32_t mdiv_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// exchange bookkeeping: out[d] = ids of topic slice d (offs[b[d+1]] -
// offs[b[d]]), out[S + d] = where slice d starts (offs[b[d]]), for
// b[d] = n * d / S
__global__ void tm_slice_sizes(const uint64_t* __restrict__ offs, uint32_t n, uint32_t S, uint64_t* __restrict__ out) {
    const uint32_t d = threadIdx.x;
    if (d >= S) return;
    const uint64_t lo = offs[(uint64_t)n * d / S], hi = offs[(uint64_t)n * (d + 1) / S];
    out[d] = hi - lo;
    out[S + d] = lo;
}

// per-source totals of a received counts block [S][m] (one block per source)
__global__ void __launch_bounds__(MBLOCK)
tm_source_totals(const uint32_t* __restrict__ counts, uint32_t m, uint64_t* __restrict__ out) {
    __shared__ uint64_t red[MBLOCK / 64];
    const uint32_t s = blockIdx.x;
    uint64_t x = 0;
    for (uint32_t t = threadIdx.x; t < m; t += MBLOCK) x += counts[(uint64_t)s * m + t];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int i = 0; i < MBLOCK / 64; ++i) t += red[i];
        out[s] = t;
    }
}

hipError_t launch_slice_sizes(const uint64_t* offs, uint32_t n, uint32_t S, uint64_t* out, hipStream_t st) {
    if (S == 0 || S > 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tm_slice_sizes, dim3(1), dim3(64), 0, st, offs, n, S, out);
    return hipGetLastError();
}

hipError_t launch_source_totals(const uint32_t* counts, uint32_t m, uint32_t S, uint64_t* out, hipStream_t st) {
    if (S == 0) return hipSuccess;
    hipLaunchKernelGGL(tm_source_totals, dim3(S), dim3(MBLOCK), 0, st, counts, m, out);
    return hipGetLastError();
}

hipError_t launch_shard_merge(uint32_t S, uint32_t m, const uint32_t* counts, const uint64_t* src_base,
                              const uint32_t* ids, const uint64_t* keys, uint32_t* out_count, uint64_t* out_off,
                              uint32_t* out_gid, uint64_t out_cap, uint64_t* total, uint64_t* pre, uint64_t* tmp,
                              hipStream_t st, uint32_t key_words, uint64_t key_stride) {
    if (S == 0 || S > MAX_SHARDS || key_words == 0) return hipErrorInvalidValue;
    if (m == 0) {
        hipError_t err = hipMemsetAsync(out_off, 0, 8, st);
        return err == hipSuccess ? hipMemsetAsync(total, 0, 8, st) : err;
    }
    if (S == 1) {   // nothing to interleave: the counts, their scan, the ids as they came
        hipError_t err = hipMemcpyAsync(out_count, counts, (size_t)m * 4, hipMemcpyDeviceToDevice, st);
        if (err == hipSuccess) err = launch_scan(counts, m, out_off, total, tmp, st);
        if (err != hipSuccess) return err;
        hipLaunchKernelGGL(tm_shard_copy1, dim3(4096), dim3(MBLOCK), 0, st, src_base, ids, total, out_gid, out_cap);
        return hipGetLastError();
    }
    // exclusive prefix of all S x m counts, source-major: within source s,
    // pre[s*m + t] - pre[s*m] is topic t's offset in s's block
    hipError_t err = launch_scan(counts, S * m, pre, pre + (uint64_t)S * m, tmp, st);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(tm_shard_sum, dim3(mdiv_up(m, MBLOCK)), dim3(MBLOCK), 0, st, S, m, counts, out_count);
    err = launch_scan(out_count, m, out_off, total, tmp, st);
    if (err != hipSuccess) return err;
    const uint32_t grid = m < 65536 ? m : 65536;
    hipLaunchKernelGGL(tm_shard_merge, dim3(grid), dim3(64), 0, st, S, m, counts, src_base, pre, ids, keys, out_off,
                       out_gid, out_cap, key_words, key_stride);
    return hipGetLastError();
}

}  // namespace tmx
