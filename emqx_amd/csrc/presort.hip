// presort.hip — the walk order of a batch (option "presort", kernels.h
// QueueBufs): topics sorted by a 32-bit key of their first eight words, so
// the 64 lanes of a wave walk shared prefixes.  Their loads of one trie node
// then coalesce into one L2 request, and the nodes under a prefix are hot in
// the XCD's L2 while its topics run.  Measured at C3 (host-sorted batches,
// bench.py --presort): whole-topic byte order -12 % walk time, 8-bit word
// hashes over all levels -11 %, 4-bit -8 %; bucketing by the first two words
// alone (the former option "group") gained nothing -- the deep levels, where
// most visits happen, carry the effect.  The walk reads the tokenized rows
// gathered into walk order (tm_presort_gather): reading them through the
// permutation (a random 64 B row and 4 B meta per topic) kept only a third
// of the gain.
//
// Key (kernels.hip presort_key, written by the tokenizer): level l's word id
// hashed to b_l bits, b = 6,5,5,4,4,3,3,2 from the most significant end
// (levels past the topic's end are 0).  Only the order in which topics are
// walked changes: counts go to each topic's index and copy-out
// (tm_copy_out_sorted) moves row p to topic perm[p]'s output range, so the
// output is identical with or without the sort.
//
// Sort: LSD radix, 4 passes of 8 bits.  Per pass: per-tile digit counts
// (digit-major), one exclusive scan, then a stable scatter: each wave ranks
// its 64 keys among equal digits with 8 ballots (multi-split), the 4 waves of
// a block combine through LDS counters round by round, so equal keys keep
// their order across rounds, waves and tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "image.h"
#include "kernels.h"

namespace tmx {

constexpr uint32_t PS_BLOCK = 256;
constexpr uint32_t PS_ROUNDS = 16;                       // keys per thread per tile
constexpr uint32_t PS_TILE = PS_BLOCK * PS_ROUNDS;       // 4096 keys per tile
constexpr uint32_t PS_WAVES = PS_BLOCK / 64;
constexpr uint32_t PS_META_N = (1u << 29) - 1;           // kernels.hip meta: level count bits (MN)

uint32_t presort_counts(uint32_t n) { return 256u * ((n + PS_TILE - 1) / PS_TILE); }

// digit counts of a tile: counts[digit * tiles + tile]
__global__ void __launch_bounds__(PS_BLOCK)
tm_presort_count(const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift, uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[256];
    hist[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t tile = blockIdx.x, base = tile * PS_TILE;
#pragma unroll 4
    for (uint32_t r = 0; r < PS_ROUNDS; ++r) {
        const uint32_t i = base + r * PS_BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&hist[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    counts[(size_t)threadIdx.x * gridDim.x + tile] = hist[threadIdx.x];
}

// stable scatter of a tile to its digits' ranges
__global__ void __launch_bounds__(PS_BLOCK)
tm_presort_scatter(const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t n,
                   uint32_t shift, const uint64_t* __restrict__ off, uint32_t* __restrict__ keys_out,
                   uint32_t* __restrict__ vals_out) {
    __shared__ uint32_t start[256];                // tile's first position per digit + keys placed so far
    __shared__ uint32_t wcnt[PS_WAVES][256];       // this round: keys per digit in each wave
    const uint32_t tile = blockIdx.x, base = tile * PS_TILE;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    start[threadIdx.x] = (uint32_t)off[(size_t)threadIdx.x * gridDim.x + tile];
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;   // lanes below this one
    for (uint32_t r = 0; r < PS_ROUNDS; ++r) {
#pragma unroll
        for (uint32_t w = 0; w < PS_WAVES; ++w) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        const uint32_t i = base + r * PS_BLOCK + threadIdx.x;
        const bool valid = i < n;
        const uint32_t k = valid ? keys_in[i] : 0u;
        const uint32_t d = (k >> shift) & 255u;
        // lanes of this wave with the same digit
        uint64_t m = __ballot(valid);
#pragma unroll
        for (uint32_t bit = 0; bit < 8; ++bit) {
            const uint64_t bb = __ballot(valid && ((d >> bit) & 1u));
            m &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = __popcll(m & lt);
        if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(m);
        __syncthreads();
        if (valid) {
            uint32_t pos = start[d] + rank;
            for (uint32_t w = 0; w < wave; ++w) pos += wcnt[w][d];
            keys_out[pos] = k;
            vals_out[pos] = vals_in[i];
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (uint32_t w = 0; w < PS_WAVES; ++w) add += wcnt[w][threadIdx.x];
        start[threadIdx.x] += add;
    }
}

// the same stable scatter through LDS (TM_PS_LOCAL): each wave ranks a
// contiguous quarter of the tile (1024 keys, 16 rounds of 64) with its own
// running per-digit counts -- no block barrier per round --, the block
// combines the waves' counts, places the tile sorted by digit in LDS, and
// writes each digit's run out with consecutive threads on consecutive
// addresses (the per-round form scatters 4 B stores one lane at a time).
#ifndef TM_PS_LOCAL
#define TM_PS_LOCAL 1
#endif
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t x, uint32_t* tmp) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) tmp[wave] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t w = 0; w < wave; ++w) pre += tmp[w];
    return pre + inc - x;
}
__global__ void __launch_bounds__(PS_BLOCK)
tm_presort_scatter_ls(const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, uint32_t n,
                      uint32_t shift, const uint64_t* __restrict__ off, uint32_t* __restrict__ keys_out,
                      uint32_t* __restrict__ vals_out) {
    __shared__ uint32_t skey[PS_TILE];
    __shared__ uint32_t sval[PS_TILE];
    __shared__ uint32_t wcnt[PS_WAVES][256];   // keys per digit in each wave, then that wave's base per digit
    __shared__ uint32_t lstart[256];           // tile-local start of each digit
    __shared__ uint32_t gstart[256];           // global start of this tile's run of each digit
    __shared__ uint32_t tmp[PS_WAVES];
    const uint32_t tile = blockIdx.x, base = tile * PS_TILE;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (uint32_t w = 0; w < PS_WAVES; ++w) wcnt[w][threadIdx.x] = 0;
    gstart[threadIdx.x] = (uint32_t)off[(size_t)threadIdx.x * gridDim.x + tile];
    __syncthreads();
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;   // lanes below this one
    uint32_t k[PS_ROUNDS], v[PS_ROUNDS], rk[PS_ROUNDS];
    const uint32_t seg = base + wave * (PS_TILE / PS_WAVES);
#pragma unroll
    for (uint32_t r = 0; r < PS_ROUNDS; ++r) {
        const uint32_t i = seg + r * 64 + lane;
        const bool valid = i < n;
        k[r] = valid ? keys_in[i] : 0u;
        v[r] = valid ? vals_in[i] : 0u;
    }
#pragma unroll
    for (uint32_t r = 0; r < PS_ROUNDS; ++r) {
        const bool valid = seg + r * 64 + lane < n;
        const uint32_t d = (k[r] >> shift) & 255u;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (uint32_t bit = 0; bit < 8; ++bit) {
            const uint64_t bb = __ballot(valid && ((d >> bit) & 1u));
            m &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = __popcll(m & lt);
        const uint32_t prior = wcnt[wave][d];   // read by every lane of the digit before its leader adds
        rk[r] = prior + rank;
        __builtin_amdgcn_wave_barrier();
        if (valid && rank == 0) wcnt[wave][d] = prior + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {   // thread = digit: the waves' bases and the digit's tile-local start
        const uint32_t d = threadIdx.x;
        uint32_t t = 0;
#pragma unroll
        for (uint32_t w = 0; w < PS_WAVES; ++w) {
            const uint32_t c = wcnt[w][d];
            wcnt[w][d] = t;
            t += c;
        }
        lstart[d] = block_excl_scan256(t, tmp);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < PS_ROUNDS; ++r) {
        if (seg + r * 64 + lane < n) {
            const uint32_t d = (k[r] >> shift) & 255u;
            const uint32_t pos = lstart[d] + wcnt[wave][d] + rk[r];
            skey[pos] = k[r];
            sval[pos] = v[r];
        }
    }
    __syncthreads();
    const uint32_t cnt = n - base < PS_TILE ? n - base : PS_TILE;
    for (uint32_t j = threadIdx.x; j < cnt; j += PS_BLOCK) {
        const uint32_t key = skey[j];
        const uint32_t d = (key >> shift) & 255u;
        const uint32_t g = gstart[d] + (j - lstart[d]);
        keys_out[g] = key;
        vals_out[g] = sval[j];
    }
}

// the rows in walk order: the 16 B chunks of words the walk reads (all of a
// long topic's row, whose later levels it reads as memory words)
__global__ void __launch_bounds__(PS_BLOCK)
tm_presort_gather(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ twords,
                  const uint32_t* __restrict__ meta, uint32_t n, uint32_t* __restrict__ twords_s,
                  uint32_t* __restrict__ meta_s) {
    const uint32_t p = blockIdx.x * PS_BLOCK + threadIdx.x;
    if (p >= n) return;
    const uint32_t t = perm[p];
    const uint32_t mt = meta[t];
    const uint32_t nl = mt & PS_META_N;
    const uint32_t chunks = nl >= WREG ? WREG / 4 : (nl + 3) / 4;
    const uint4* src = reinterpret_cast<const uint4*>(twords + (size_t)t * WREG);
    uint4* dst = reinterpret_cast<uint4*>(twords_s + (size_t)p * WREG);
#pragma unroll
    for (uint32_t k = 0; k < WREG / 4; ++k)
        if (k < chunks) dst[k] = src[k];
    meta_s[p] = mt;
}

hipError_t launch_presort(const uint32_t* twords, const uint32_t* meta, uint32_t n, const QueueBufs& qb,
                          hipStream_t st, bool gather) {
    if (n == 0) return hipSuccess;
    const uint32_t tiles = (n + PS_TILE - 1) / PS_TILE, nc = 256u * tiles;
    // ping-pong: keys A = sort_keys, B = sort_keys + n; values A = perm, B = sort_vals;
    // an even number of passes starts in A, an odd one in B, so the last ends
    // in A and perm holds the order (the tokenizer wrote the keys and values
    // t there: kernels.hip presort_key / tail_key).  Passes sort the key's
    // top 8 * passes bits (the tail order's key is 8 bits: one pass).
    const uint32_t passes = qb.presort_passes();
    if (passes < 1 || passes > 4) return hipErrorInvalidValue;
    uint32_t *ka = qb.sort_keys, *kb = qb.sort_keys + n, *va = qb.perm, *vb = qb.sort_vals;
    if (passes & 1u) {
        ka = qb.sort_keys + n;
        kb = qb.sort_keys;
        va = qb.sort_vals;
        vb = qb.perm;
    }
    // the lowest key bit sorted: the range-keyed orders (2, 4, 5) sort their
    // whole 8 / 16-bit key, the word-hash key (1) its top 8 x passes bits
    const uint32_t low = qb.presort_mode >= 2 ? 0u : 32u - 8u * passes;
    for (uint32_t pass = 0; pass < passes; ++pass) {
        const uint32_t shift = low + 8 * pass;
        hipLaunchKernelGGL(tm_presort_count, dim3(tiles), dim3(PS_BLOCK), 0, st, ka, n, shift, qb.sort_counts);
        hipError_t err = launch_scan(qb.sort_counts, nc, qb.sort_off, qb.sort_off + nc, qb.sort_scan, st);
        if (err != hipSuccess) return err;
        if (TM_PS_LOCAL)
            hipLaunchKernelGGL(tm_presort_scatter_ls, dim3(tiles), dim3(PS_BLOCK), 0, st, ka, va, n, shift,
                               qb.sort_off, kb, vb);
        else
            hipLaunchKernelGGL(tm_presort_scatter, dim3(tiles), dim3(PS_BLOCK), 0, st, ka, va, n, shift,
                               qb.sort_off, kb, vb);
        uint32_t* t = ka;
        ka = kb;
        kb = t;
        t = va;
        va = vb;
        vb = t;
    }
    if (gather)   // rows into walk order (a walk with chunk rows reads them through perm instead)
        hipLaunchKernelGGL(tm_presort_gather, dim3((n + PS_BLOCK - 1) / PS_BLOCK), dim3(PS_BLOCK), 0, st, qb.perm,
                           twords, meta, n, qb.twords_s, qb.meta_s);
    return hipGetLastError();
}

}  // namespace tmx
