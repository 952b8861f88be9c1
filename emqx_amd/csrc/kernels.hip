// kernels.hip — CDNA4 (gfx950) kernels of the topic-routing hot path
// (emqx_trie:match/1 over a batch of publish topics).  Four launches on one
// stream:
//
//   tm_tokenize    emqx_topic:words/1 + word/1 (src/emqx_topic.erl:141-147):
//                  one lane per topic splits on '/', hashes each level, probes
//                  the word dictionary and byte-verifies -> per-level word ids.
//   tm_walk_queue  emqx_trie:match/1 (src/emqx_trie.erl:77-79, 121-145):
//                  persistent waves dequeue 64-topic chunks; every lane walks
//                  its own topic's NFA over '+' / '#' / literal edges and takes
//                  the next topic the moment it finishes.  One step = ONE 16 B
//                  load of a node half (image.h); the per-level pending '+'
//                  children sit in LDS, the topic's words in VGPRs.  The walk
//                  runs in the reference's DISCOVERY order and writes ids from
//                  the end of the topic's stage row backwards: the reference
//                  prepends every discovery, so the reversed discovery order IS
//                  its output order and no sort is needed.
//   tm_scan_*      counts -> CSR offsets.
//   tm_copy_out    coalesced stage -> CSR copy; topics whose fan-out exceeds
//                  the stage row re-walk and write the remainder directly.
//
// All integer/byte work: no MFMA.  The walk is bound by the vector-memory
// address path of divergent 16 B gathers over the HBM image.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "image.h"
#include "kernels.h"

namespace tmx {

constexpr int BLOCK = 256;

// Non-temporal loads and stores.  TM_NT_STREAM (A/B builds): the once-read
// and once-written streams of the pipeline -- the tokenizer's topic bytes
// and rows, the walk's chunk-row fill, the copy-out's stage reads -- marked
// non-temporal, so they do not push the trie's lines out of the caches
// between walks (the Infinity Cache keeps a line only while everything any
// kernel touches between two of its uses fits in its 256 MiB)
#ifndef TM_NT_STREAM
#define TM_NT_STREAM 0
#endif
typedef uint32_t u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load16(const void* p) {
    const u32x4_nt x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void nt_store16(void* p, uint4 v) {
    u32x4_nt x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4_nt*>(p));
}
template <class T>
__device__ __forceinline__ T stream_load(const T* p) {
    if (TM_NT_STREAM) return __builtin_nontemporal_load(p);
    return *p;
}
template <class T>
__device__ __forceinline__ void stream_store(T* p, T v) {
    if (TM_NT_STREAM) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ uint4 stream_load16(const void* p) {
    if (TM_NT_STREAM) return nt_load16(p);
    return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void stream_store16(void* p, uint4 v) {
    if (TM_NT_STREAM) nt_store16(p, v);
    else *reinterpret_cast<uint4*>(p) = v;
}

__device__ __forceinline__ void wave_sync_lds() {
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
// byte access: aligned 8-byte words (an aligned word holding a valid byte
// never crosses a page), little-endian extraction.  Topic bytes are read
// either from global memory or from a wave's LDS window (tm_tokenize stages
// the bytes of its 64 topics with coalesced loads first).
struct GlobalBytes {
    const uint8_t* p;
    __device__ __forceinline__ uint64_t word(uint64_t q) const {
        return *reinterpret_cast<const uint64_t*>(p + (q & ~7ull));
    }
    __device__ __forceinline__ uint32_t byte(uint64_t q) const { return p[q]; }
};
struct LdsBytes {
    const uint64_t* w;   // LDS words of bytes [base, ...), base 8-aligned
    uint64_t base;
    __device__ __forceinline__ uint64_t word(uint64_t q) const { return w[(q - base) >> 3]; }
    __device__ __forceinline__ uint32_t byte(uint64_t q) const {
        return (uint32_t)(word(q) >> (8 * (q & 7))) & 0xFFu;
    }
};

// assemble up to 8 bytes [p, p+k) (k in 1..8) little-endian, zero padded
template <class B>
__device__ __forceinline__ uint64_t load_chunk(const B& bytes, uint64_t p, uint32_t k) {
    uint32_t sh = (uint32_t)(p & 7) * 8;
    uint64_t v = bytes.word(p) >> sh;
    if (sh != 0 && (p & 7) + k > 8) v |= bytes.word(p + 8) << (64 - sh);
    if (k < 8) v &= (~0ull) >> (64 - 8 * k);
    return v;
}

// dictionary lookup of topic bytes [p, p+len): word id, WORD_PLUS/HASH for the
// atoms '+' / '#', or WORD_NONE (bytes no filter contains: match only '+'/'#').
// Split in two so the tokenizer can issue a level's slot load (dict_begin),
// scan and hash the next level while it is in flight, then resolve it
// (dict_end: byte-verify, probe on).
struct DictProbe {         // 8 VGPRs: the tokenizer holds TM_TOK_DEPTH + 1 of them
    uint32_t rel, s;          // the word's offset in its topic; the home slot
    uint32_t tag, len;
    uint4 d0;                 // the home slot's first half: tag, word, bytes 0-7
};
template <class B>
__device__ __forceinline__ DictProbe dict_begin(const ImageView& im, const B& bytes, uint64_t b, uint64_t p,
                                                uint32_t len) {
    DictProbe q;
    q.rel = (uint32_t)(p - b);
    q.len = len;
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (uint32_t i = 0; i < len; i += 8) {
        uint32_t k = len - i < 8 ? len - i : 8;
        h = word_hash_step(h, load_chunk(bytes, p + i, k));
    }
    h = word_hash_final(h, len);
    q.tag = dict_tag(h, len);
    q.s = (uint32_t)(h & im.dict_slot_mask);
    q.d0 = reinterpret_cast<const uint4*>(im.dict + q.s)[0];
    return q;
}
// a word of <= 8 bytes is decided by the slot's first 16 B alone (tag, id,
// bytes); 9-16 bytes also read the second half (same 32 B), longer words the
// zero-padded arena
template <class B>
__device__ __forceinline__ uint32_t dict_end(const ImageView& im, const B& bytes, uint64_t b, DictProbe q) {
    const uint64_t p = b + q.rel;
    const uint32_t len = q.len;
    if (len == 1) {   // the atoms '+' / '#'
        const uint32_t c = bytes.byte(p);
        if (c == '+') return WORD_PLUS;
        if (c == '#') return WORD_HASH;
    }
    const uint32_t tag = q.tag;
    uint64_t s = q.s;
    uint4 d0 = q.d0;
    for (;;) {
        const uint32_t word = d0.y;
        if (word == WORD_NONE) return WORD_NONE;
        if (d0.x == tag) {
            const uint64_t head0 = ((uint64_t)d0.w << 32) | d0.z;
            bool eq = len == 0 || load_chunk(bytes, p, len < 8 ? len : 8) == head0;
            if (eq && len > 8) {
                const uint4 d1 = reinterpret_cast<const uint4*>(im.dict + s)[1];   // head1, exact len
                const uint64_t head1 = ((uint64_t)d1.y << 32) | d1.x;
                eq = d1.z == len && load_chunk(bytes, p + 8, len < 16 ? len - 8 : 8) == head1;
                if (eq && len > 16) {
                    const uint64_t* a = reinterpret_cast<const uint64_t*>(im.word_arena + im.word_off[word]);
                    for (uint32_t i = 16; i < len && eq; i += 8) {
                        uint32_t k = len - i < 8 ? len - i : 8;
                        eq = (load_chunk(bytes, p + i, k) == a[i >> 3]);
                    }
                }
            }
            if (eq) return word;
        }
        s = (s + 1) & im.dict_slot_mask;
        d0 = reinterpret_cast<const uint4*>(im.dict + s)[0];
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

// exact per-byte '/' test of an 8-byte word: 0x80 in each byte that is '/'.
// (The borrow form (x - 0x01..) & ~x & 0x80.. also flags a byte 0x01 above
// a zero byte, i.e. a '.' right after a '/': a scan resumed after that '/'
// split "a/.b" at the '.'; tests/test_gpu_tokenize.py)
__device__ __forceinline__ uint64_t slash_bytes(uint64_t x) {
    constexpr uint64_t M = 0x7F7F7F7F7F7F7F7FULL;
    x ^= 0x2F2F2F2F2F2F2F2FULL;   // '/' -> 0x00
    return ~(((x & M) + M) | x | M);
}

// the next '/' of topic bytes [q, e) eight bytes at a time (e when none)
template <class B>
__device__ __forceinline__ uint64_t next_slash(const B& bytes, uint64_t q, uint64_t e, bool& found) {
    found = false;
    while (q < e) {
        uint64_t word8 = bytes.word(q);
        uint32_t start = (uint32_t)(q & 7);
        uint64_t rem = e - (q & ~7ull);
        uint32_t stop = rem < 8 ? (uint32_t)rem : 8;
        uint64_t z = slash_bytes(word8);
        z &= (~0ull) << (8 * start);
        if (stop < 8) z &= (~0ull) >> (64 - 8 * stop);
        if (z) {
            found = true;
            return (q & ~7ull) + (__builtin_ctzll(z) >> 3);
        }
        q = (q & ~7ull) + 8;
    }
    return e;
}

// emqx_topic:words/1 of topic [b, e): word id of level k to tw[k] (k < WREG,
// registers: AND-mask updates, no dynamic index) or lw[k] (k >= WREG);
// returns the number of levels (N slashes -> N+1 levels, empty levels kept).
// Software-pipelined by TM_TOK_DEPTH levels: levels k+1 .. k+D are scanned,
// hashed and their dictionary slots requested before level k's slot is
// resolved.
#ifndef TM_TOK_LEAN
#define TM_TOK_LEAN 0   // A/B builds: tokenizer without LDS staging or pipelining (fewer registers, no LDS)
#endif
#ifndef TM_TOK_DEPTH
#define TM_TOK_DEPTH 2
#endif
template <class B>
__device__ __forceinline__ uint32_t tokenize_topic(const ImageView& im, const B& bytes, uint64_t b, uint64_t e,
                                                   uint32_t (&tw)[WREG], uint32_t* lw, bool& ood) {
    uint32_t lev = 0;
    ood = false;
    bool found;
    if (TM_TOK_LEAN) {   // one level at a time
        uint64_t s = b;
        for (;;) {
            const uint64_t q = next_slash(bytes, s, e, found);
            const uint32_t w = dict_end(im, bytes, b, dict_begin(im, bytes, b, s, (uint32_t)(q - s)));
            ood |= w == WORD_PLUS || w == WORD_HASH;
            if (lev < WREG) {
#pragma unroll
                for (uint32_t k = 0; k < WREG; ++k) tw[k] = lev == k ? w : tw[k];
            } else {
                lw[lev] = w;
            }
            ++lev;
            if (!found) return lev;
            s = q + 1;
        }
    }
    auto put = [&](uint32_t w) {
        ood |= w == WORD_PLUS || w == WORD_HASH;
        if (lev < WREG) {
#pragma unroll
            for (uint32_t k = 0; k < WREG; ++k) tw[k] = lev == k ? w : tw[k];
        } else {
            lw[lev] = w;
        }
        ++lev;
    };
    uint64_t q = next_slash(bytes, b, e, found);
    DictProbe cur = dict_begin(im, bytes, b, b, (uint32_t)(q - b));
    if (TM_TOK_DEPTH >= 2) {
        // two levels ahead: c1 (level lev + 1, valid if v1) and the next
        // (lev + 2) are in flight while level lev resolves
        DictProbe c1;
        bool v1 = false;
        if (found) {
            const uint64_t s = q + 1;
            q = next_slash(bytes, s, e, found);
            c1 = dict_begin(im, bytes, b, s, (uint32_t)(q - s));
            v1 = true;
        }
        for (;;) {
            DictProbe c2;
            bool v2 = false;
            if (v1 && found) {
                const uint64_t s = q + 1;
                q = next_slash(bytes, s, e, found);
                c2 = dict_begin(im, bytes, b, s, (uint32_t)(q - s));
                v2 = true;
            }
            put(dict_end(im, bytes, b, cur));
            if (!v1) return lev;
            cur = c1;
            c1 = c2;
            v1 = v2;
        }
    }
    for (;;) {
        const bool more = found;
        DictProbe nxt;
        if (more) {
            const uint64_t s = q + 1;
            q = next_slash(bytes, s, e, found);
            nxt = dict_begin(im, bytes, b, s, (uint32_t)(q - s));
        }
        put(dict_end(im, bytes, b, cur));
        if (!more) return lev;
        cur = nxt;
    }
}

// meta bits: levels | MOOD (a level is the atom '+' or '#': out of the
// publish domain, emqx_packet.erl:63) | MLONG (more than WREG levels) | MDOLLAR
constexpr uint32_t MOOD = 1u << 29, MLONG = 1u << 30, MDOLLAR = 1u << 31, MN = (1u << 29) - 1;

constexpr uint32_t TOK_WIN_WORDS = 512;   // LDS bytes window per wave: 4 KiB (64 topics of <= 64 B)

// option "presort" (presort.hip): a topic's walk-order key -- its first
// eight words hashed to 6,5,5,4,4,3,3,2 bits, level-major (levels past the
// topic's end are 0)
__device__ __forceinline__ uint32_t presort_key(const uint32_t (&tw)[WREG], uint32_t lev) {
    constexpr uint32_t bits[8] = {6, 5, 5, 4, 4, 3, 3, 2};
    uint32_t k = 0;
#pragma unroll
    for (uint32_t l = 0; l < 8; ++l) k = (k << bits[l]) | (l < lev ? (tw[l] * 0x9E3779B1u) >> (32 - bits[l]) : 0u);
    return k;
}

// option "presort" 2, the tail order: within each of the walk's 8 XCD ranges
// (QRANGES, by topic index), the topics whose words label the most trie
// nodes first -- they lead into the most filters and take the longest walks,
// so the lanes that finish last are the ones on light topics.  Key: the
// range (3 bits) over 31 - the summed heat of the first eight levels / 4
// (5 bits), one radix pass (presort.hip).
// the walk's XCD range of queue position t: [n r / 8, n (r+1) / 8)
// (an f32 estimate, then exact: no 64-bit division)
__device__ __forceinline__ uint32_t range_of(uint32_t t, uint32_t n) {
    uint32_t r = (uint32_t)__builtin_fminf(8.0f * (float)t * __builtin_amdgcn_rcpf((float)n), 7.0f);
    while (r > 0 && (uint64_t)n * r / 8 > t) --r;
    while (r < 7 && (uint64_t)n * (r + 1) / 8 <= t) ++r;
    return r;
}
__device__ __forceinline__ uint32_t tail_key(const ImageView& im, const uint32_t (&tw)[WREG], uint32_t lev,
                                             uint32_t t, uint32_t n) {
    uint32_t cost = 0;
#pragma unroll
    for (uint32_t l = 0; l < 8; ++l) {
        const uint32_t w = tw[l];
        if (l < lev && w < im.n_words) cost += im.word_heat[w];
    }
    const uint32_t c = cost >> 2 < 31 ? cost >> 2 : 31u;
    return (range_of(t, n) << 5) | (31u - c);
}

// a tokenized topic's row (levels < WREG), meta and presort key; returns
// the topic's cost class (presort 6) or 32
__device__ __forceinline__ uint32_t tok_store(const ImageView& im, uint32_t t, uint32_t n, uint32_t lev,
                                              const uint32_t (&tw)[WREG], bool ood, uint32_t dollar,
                                              uint32_t* __restrict__ twords, uint32_t* __restrict__ meta,
                                              uint32_t* __restrict__ skeys, uint32_t* __restrict__ svals,
                                              uint32_t key_mode) {
    // the row as whole 16 B stores (per-level 4 B stores from 64 lanes to
    // 64 rows were partial-line writes: read-modify-write traffic), only the
    // quads the walk reads (4k < levels: 32 B for an 8-level topic)
    uint4* row = reinterpret_cast<uint4*>(twords + (uint64_t)t * WREG);
#pragma unroll
    for (uint32_t k = 0; k < WREG / 4; ++k)
        if (4 * k < lev || k == 0) stream_store16(row + k, make_uint4(tw[4 * k], tw[4 * k + 1], tw[4 * k + 2], tw[4 * k + 3]));
    stream_store(meta + t, lev | (dollar << 31) | (lev > WREG ? MLONG : 0u) | (ood ? MOOD : 0u));
    if (skeys) {   // option "presort": the walk-order key (presort.hip)
        // 2: the tail order (8 bits); 4: the tail order, then the word-hash
        // key's top 8 bits within a heat class (16); 5: the XCD range, then
        // the word-hash key's top 13 bits (16); 1: the word-hash key (32)
        // (key_mode: the order | its key bits << 8 | the light-tail class
        // bound << 16; 5 takes the range's 3 bits over the word-hash key's
        // top bits - 3; 6 the range's 3 bits, a light-tail bit, then the
        // word-hash key's top bits - 4)
        const uint32_t mode = key_mode & 255u, bits = (key_mode >> 8) & 255u;
        if (mode == 6) {
            const uint32_t tk = tail_key(im, tw, lev, t, n), c = 31u - (tk & 31u);
            const uint32_t light = c <= ((key_mode >> 16) & 255u) ? 1u : 0u;
            skeys[t] = (tk >> 5) << (bits - 3) | light << (bits - 4) | presort_key(tw, lev) >> (36 - bits);
            svals[t] = t;
            return c;
        }
        skeys[t] = mode == 2   ? tail_key(im, tw, lev, t, n)
                   : mode == 4 ? tail_key(im, tw, lev, t, n) << 8 | presort_key(tw, lev) >> 24
                   : mode == 5 ? range_of(t, n) << (bits - 3) | presort_key(tw, lev) >> (35 - bits)   // (no heat)
                               : presort_key(tw, lev);
        svals[t] = t;
    }
    return 32u;   // (presort 6: the topic's cost class)
}

template <class B>
__device__ __forceinline__ uint32_t tokenize_one(const ImageView& im, const B& bytes,
                                             const uint64_t* __restrict__ off, uint32_t t, uint32_t n,
                                             uint32_t* __restrict__ twords, uint32_t* __restrict__ words,
                                             uint32_t* __restrict__ meta, uint32_t* __restrict__ skeys,
                                             uint32_t* __restrict__ svals, uint32_t key_mode) {
    const uint64_t b = off[t], e = off[t + 1];
    uint32_t tw[WREG];
#pragma unroll
    for (uint32_t k = 0; k < WREG; ++k) tw[k] = WORD_NONE;
    bool ood;
    const uint32_t lev = tokenize_topic(im, bytes, b, e, tw, words + (b - off[0]) + t, ood);
    const uint32_t dollar = (e > b && bytes.byte(b) == '$') ? 1u : 0u;
    return tok_store(im, t, n, lev, tw, ood, dollar, twords, meta, skeys, svals, key_mode);
}

// The wave-cooperative tokenizer.  The per-lane scan
// above walks each topic level by level on one lane (a '/' scan, the hash,
// the dictionary probe, then the next level): ~300 VALU instructions and one
// dependent round trip per level, with 64 lanes doing it in lockstep.  Here
// a wave's 64 topics are split into their levels first, and the lanes then
// take the levels, not the topics:
//   1. each lane counts the '/' of its topic in the LDS window (an exact
//      zero-byte test per 8 bytes, popcount), a wave prefix sum gives every
//      topic its first level's index in the wave's level list, and the lane
//      writes its levels' {start, length} there;
//   2. lane j takes levels j, j + 64, ...: hashes the level's bytes and
//      issues its dictionary slot load, TOK_BATCH levels at a time with all
//      their loads in flight, then resolves them (byte-verified, dict_end)
//      and writes the word id over the level's entry;
//   3. each lane reads its topic's word ids back (consecutive entries) and
//      stores the row, meta and presort key as before (tok_store).
// emqx_topic:words/1 semantics are unchanged: N slashes make N + 1 levels,
// empty levels are kept, '+' / '#' levels are the atoms.
// levels per wave's list: one u32 each (the level's {start, length}, then
// its word id); 1000 keeps a 4-wave block at 32.5 KB of LDS, 5 blocks per CU
// (5 waves per SIMD, as the VGPRs allow); a wave with more: the per-lane path
constexpr uint32_t TOK_LMAX = 1000;
constexpr uint32_t TOK_WAVE = 1u << 24;   // key_mode bit: the wave path (option "tok_wave"; 0: per lane)
#ifndef TM_TOK_BATCH
#define TM_TOK_BATCH 3   // dictionary probes in flight per lane (4 held to 96 VGPRs, or at 97 and 4 waves:
                         // the same or slower, profiles/r06_h_ab, r06_i_ab)
#endif
// bytes [o, o + k) of a wave's LDS window, k in 1..8, zero padded (32-bit
// offsets: the window is at most 4 KiB)
__device__ __forceinline__ uint64_t win_chunk(const uint64_t* w, uint32_t o, uint32_t k) {
    const uint32_t q = o >> 3, sh = (o & 7u) * 8u;
    uint64_t v = w[q] >> sh;
    if (sh != 0 && (o & 7u) + k > 8) v |= w[q + 1] << (64 - sh);
    return k < 8 ? v & (~0ull >> (64 - 8 * k)) : v;
}
// The wave path's dictionary probe: dict_begin / dict_end over the LDS
// window, with the word's first 16 bytes kept from the hash pass for the
// byte compare (dict_end re-assembles them from the bytes)
struct WaveProbe {
    uint32_t s, tag, len, off;   // home slot, tag, word length, window offset
    uint64_t h0, h1;             // bytes 0-7, 8-15, zero padded
    uint4 d0;                    // the home slot's first half
};
__device__ __forceinline__ WaveProbe wave_dict_begin(const ImageView& im, const uint64_t* w, uint32_t o,
                                                     uint32_t len) {
    WaveProbe q;
    q.off = o;
    q.len = len;
    uint64_t h = 0x243F6A8885A308D3ULL;   // (dict_begin's hash, chunk by chunk)
    q.h0 = len ? win_chunk(w, o, len < 8 ? len : 8u) : 0ull;
    q.h1 = len > 8 ? win_chunk(w, o + 8, len < 16 ? len - 8 : 8u) : 0ull;
    if (len) h = word_hash_step(h, q.h0);
    if (len > 8) h = word_hash_step(h, q.h1);
    for (uint32_t i = 16; i < len; i += 8) h = word_hash_step(h, win_chunk(w, o + i, len - i < 8 ? len - i : 8u));
    h = word_hash_final(h, len);
    q.tag = dict_tag(h, len);
    q.s = (uint32_t)(h & im.dict_slot_mask);
    q.d0 = reinterpret_cast<const uint4*>(im.dict + q.s)[0];
    return q;
}
__device__ __forceinline__ uint32_t wave_dict_end(const ImageView& im, const uint64_t* w, const WaveProbe& q) {
    const uint32_t len = q.len;
    if (len == 1) {   // the atoms '+' / '#'
        const uint32_t c = (uint32_t)q.h0;
        if (c == '+') return WORD_PLUS;
        if (c == '#') return WORD_HASH;
    }
    uint64_t s = q.s;
    uint4 d0 = q.d0;
    for (;;) {
        const uint32_t word = d0.y;
        if (word == WORD_NONE) return WORD_NONE;
        if (d0.x == q.tag) {
            bool eq = len == 0 || q.h0 == (((uint64_t)d0.w << 32) | d0.z);
            if (eq && len > 8) {
                const uint4 d1 = reinterpret_cast<const uint4*>(im.dict + s)[1];   // head1, exact len
                eq = d1.z == len && q.h1 == (((uint64_t)d1.y << 32) | d1.x);
                if (eq && len > 16) {
                    const uint64_t* a = reinterpret_cast<const uint64_t*>(im.word_arena + im.word_off[word]);
                    for (uint32_t i = 16; i < len && eq; i += 8)
                        eq = win_chunk(w, q.off + i, len - i < 8 ? len - i : 8u) == a[i >> 3];
                }
            }
            if (eq) return word;
        }
        s = (s + 1) & im.dict_slot_mask;
        d0 = reinterpret_cast<const uint4*>(im.dict + s)[0];
    }
}

__global__ void __launch_bounds__(BLOCK)
tm_tokenize(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint32_t n,
            uint32_t* __restrict__ twords, uint32_t* __restrict__ words, uint32_t* __restrict__ meta,
            uint32_t* __restrict__ skeys, uint32_t* __restrict__ svals, uint32_t key_mode,
            unsigned long long* __restrict__ ws_hist) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (TM_TOK_LEAN) {
        if (t < n) tokenize_one(im, GlobalBytes{bytes}, off, t, n, twords, words, meta, skeys, svals, key_mode);
        return;
    }
    __shared__ uint64_t win[BLOCK / 64][TOK_WIN_WORDS];
    __shared__ uint32_t tok_lev[BLOCK / 64][TOK_LMAX];   // the wave's levels: start | length << 16, then the id
    __shared__ uint32_t chist[32];   // presort 6: the block's cost-class histogram (QWS_CHIST)
    const bool hist = skeys && (key_mode & 255u) == 6u;
    if (hist && threadIdx.x < 32) chist[threadIdx.x] = 0;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // the wave's 64 topics are contiguous bytes: stage them in LDS with
    // coalesced loads (per-lane 8 B loads of 64 different topics touch 64
    // lines per instruction); a window that does not fit reads global memory
    const uint32_t t0 = t - lane;
    uint64_t wbase = 0;
    bool lds = false;
    if (t0 < n) {
        const uint32_t t1 = t0 + 64 < n ? t0 + 64 : n;
        wbase = off[t0] & ~7ull;
        const uint64_t nw = (off[t1] - wbase + 7) >> 3;
        lds = nw <= TOK_WIN_WORDS;
        if (lds)
            for (uint64_t k = lane; k < nw; k += 64)
                win[wv][k] = stream_load(reinterpret_cast<const uint64_t*>(bytes + wbase + 8 * k));
    }
    __syncthreads();
    uint32_t c = 32u;
    // 1. levels of the lane's topic: count, wave prefix sum, descriptors
    uint32_t b = 0, e = 0, nl = 0;
    uint64_t mlo = ~0ull, mhi = ~0ull;   // the topic's bytes in its first / last window word
    auto tmask = [&](uint32_t q) -> uint64_t {   // the topic's bytes of window word q: two selects
        return (q == b >> 3 ? mlo : ~0ull) & (q == (e - 1) >> 3 ? mhi : ~0ull);
    };
    if (lds && t < n) {
        b = (uint32_t)(off[t] - wbase);
        e = (uint32_t)(off[t + 1] - wbase);
        mlo = ~0ull << (8 * (b & 7u));
        mhi = (e & 7u) ? ~0ull >> (64 - 8 * (e & 7u)) : ~0ull;
        for (uint32_t q = b >> 3; 8 * q < e; ++q)
            nl += (uint32_t)__popcll(slash_bytes(win[wv][q]) & tmask(q));
        nl += 1;
    }
    uint32_t first = nl;   // inclusive, then exclusive prefix over the wave
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)first, o, 64);
        if ((int)lane >= o) first += y;
    }
    const uint32_t L = (uint32_t)__shfl((int)first, 63, 64);
    first -= nl;
    if (lds && L <= TOK_LMAX && (key_mode & TOK_WAVE)) {   // (uniform per wave)
        uint32_t* lv = tok_lev[wv];
        if (t < n) {
            uint32_t k = first, s0 = b;
            for (uint32_t q = b >> 3; 8 * q < e; ++q) {
                uint64_t z = slash_bytes(win[wv][q]) & tmask(q);
                while (z) {
                    const uint32_t p = 8 * q + ((uint32_t)__builtin_ctzll(z) >> 3);
                    z &= z - 1;
                    lv[k++] = s0 | (p - s0) << 16;
                    s0 = p + 1;
                }
            }
            lv[k] = s0 | (e - s0) << 16;
        }
        wave_sync_lds();
        // 2. lanes over levels: TM_TOK_BATCH dictionary loads in flight per lane
        const LdsBytes lb{win[wv], wbase};
        for (uint32_t i0 = 0; i0 < L; i0 += 64 * TM_TOK_BATCH) {
            WaveProbe q[TM_TOK_BATCH];
#pragma unroll
            for (uint32_t j = 0; j < TM_TOK_BATCH; ++j) {
                const uint32_t i = i0 + 64 * j + lane;
                if (i < L) {
                    const uint32_t d = lv[i];
                    q[j] = wave_dict_begin(im, win[wv], d & 0xFFFFu, d >> 16);
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < TM_TOK_BATCH; ++j) {
                const uint32_t i = i0 + 64 * j + lane;
                if (i < L) lv[i] = wave_dict_end(im, win[wv], q[j]);   // (only this lane reads entry i)
            }
        }
        wave_sync_lds();
        // 3. the lane's topic: its word ids, row, meta and key
        if (t < n) {
            uint32_t tw[WREG];
            bool ood = false;
#pragma unroll
            for (uint32_t k = 0; k < WREG; ++k) {
                const uint32_t w = k < nl ? lv[first + k] : WORD_NONE;
                ood |= w == WORD_PLUS || w == WORD_HASH;
                tw[k] = w;
            }
            if (nl > WREG) {   // levels >= WREG of a long topic: global, beside its bytes
                uint32_t* lw = words + (off[t] - off[0]) + t;
                for (uint32_t k = WREG; k < nl; ++k) {
                    const uint32_t w = lv[first + k];
                    ood |= w == WORD_PLUS || w == WORD_HASH;
                    lw[k] = w;
                }
            }
            const uint32_t dollar = (e > b && lb.byte(wbase + b) == '$') ? 1u : 0u;
            c = tok_store(im, t, n, nl, tw, ood, dollar, twords, meta, skeys, svals, key_mode);
        }
    } else if (t < n) {
        if (lds)
            c = tokenize_one(im, LdsBytes{win[wv], wbase}, off, t, n, twords, words, meta, skeys, svals, key_mode);
        else
            c = tokenize_one(im, GlobalBytes{bytes}, off, t, n, twords, words, meta, skeys, svals, key_mode);
    }
    if (hist) {   // (uniform per block: the key mode is one for the launch)
        if (c < 32u) atomicAdd(&chist[c], 1u);
        __syncthreads();
        if (threadIdx.x < 32 && chist[threadIdx.x])
            atomicAdd(ws_hist + threadIdx.x, (unsigned long long)chist[threadIdx.x]);
    }
}



// ---------------------------------------------------------------------------
// The child found by a probe, with its record when the edge table delivered
// it: the inner half {plus, hash_filter, lw, lc} and the filter ending at
// the child.
struct Hit {
    uint32_t child;
    uint32_t plus, hf, lw, lc, sf;   // (no HIP vector type here: its union
    bool have;                       // layout sends the struct to scratch)
};

// TM_NT_PROBE (A/B builds): edge-table loads below the hot top non-temporal
#ifndef TM_NT_PROBE
#define TM_NT_PROBE 0
#endif
#ifndef TM_WALK_CLOCKS
#define TM_WALK_CLOCKS 0   // diagnostic builds: the queue walk's per-XCD phase clocks (QWS_CLOCK,
                           // tm_debug_walk_clocks); 4 VGPRs of the walk, so off in the product build
#endif
// literal (or '#') edge (v, w) in the edge table: linear probing, one 16 B
// key half per slot (load factor <= 1/4: ~1.2 loads per hit); on a hit the
// slot's second half completes the child's record
template <bool STATS>
__device__ __forceinline__ Hit probe_edge(const ImageView& im, uint32_t v, uint32_t w, uint64_t& loads) {
    const bool hot = v < im.hot_limit;   // the top of the trie: a small table of its own
    const EdgeSlot* tab = hot ? im.hot_edges : im.edges;
    const uint64_t mask = hot ? im.hot_slot_mask : im.edge_slot_mask;
    uint64_t s = edge_home(v, w, mask);
    for (;;) {
        const uint4* slot = reinterpret_cast<const uint4*>(tab + s);
        const uint4 e = (TM_NT_PROBE && !hot) ? nt_load16(slot) : slot[0];
        // TM_SLOT_RECORD: the record half is loaded with the key half (same
        // 32 B, one dependent step), so a found child is visited without a
        // load of its own
        uint4 d = make_uint4(0, 0, 0, 0);
        if (SLOT_RECORD) d = slot[1];   // hash_filter, lw, lc, self_filter
        if (STATS) ++loads;
        if (e.x == v && e.y == w) {
            if (!SLOT_RECORD) return Hit{e.z, e.w, 0, 0, 0, 0, false};   // plus: the child's summary S(c)
            return Hit{e.z, e.w, d.x, d.y, d.z, d.w, true};
        }
        if (e.x == EDGE_EMPTY) return Hit{NODE_NONE, 0, 0, 0, 0, 0, false};
        s = (s + 1) & mask;
    }
}

// child of v by topic word w, given v's inner half {plus, lw, lc}.
// WORD_PLUS / WORD_HASH reproduce the reference for the out-of-domain topic
// levels "+" / "#": the fold over [W, '+'] at emqx_trie.erl:131-136 follows
// the '+' / '#' edge.
template <bool STATS>
__device__ __forceinline__ Hit lit_child(const ImageView& im, uint32_t v, uint32_t plus, uint32_t lw, uint32_t lc,
                                         uint32_t w, uint64_t& loads) {
    const Hit none{NODE_NONE, 0, 0, 0, 0, 0, false};
    if (w < WORD_MAX) {
        if (!(plus & WIDE)) return Hit{lw == w ? lc : NODE_NONE, SUM_ALL, 0, 0, 0, 0, false};
        const uint64_t b = word_bloom(w);
        const uint64_t mask = ((uint64_t)lc << 32) | lw;
        return (mask & b) == b ? probe_edge<STATS>(im, v, w, loads) : none;
    }
    if (w == WORD_PLUS) return Hit{plus & NODE_MASK, SUM_ALL, 0, 0, 0, 0, false};
    if (w == WORD_HASH) return probe_edge<STATS>(im, v, WORD_HASH, loads);
    return none;   // WORD_NONE: bytes no filter contains
}

// Cache policy (A/B builds): TM_NT_LEVEL = d marks node loads at depth >= d
// (and leaf halves) non-temporal, so deep, rarely re-used nodes do not push
// the shared upper levels out of L2; TM_NT_STAGE marks the stage-row stores
// non-temporal.  0 / unset: ordinary loads and stores.
#ifndef TM_NT_LEVEL
#define TM_NT_LEVEL 0
#endif
#ifndef TM_NT_ROWS
#define TM_NT_ROWS 0   // the walk's reads of the tokenized rows (once per topic) non-temporal
#endif
#ifndef TM_NT_STAGE
#define TM_NT_STAGE 1   // A/B at C3: walk 11.9-12.2 vs 12.4-12.6 ms (profiles/r02_ab)
#endif
__device__ __forceinline__ uint4 load_half(const ImageView& im, uint32_t v, bool leaf, uint32_t r = 0) {
    const uint4* p = reinterpret_cast<const uint4*>((leaf ? im.leaf : im.inner) + ((uint64_t)v << im.node_shift));
    if (TM_NT_LEVEL > 0 && (leaf || r >= (uint32_t)TM_NT_LEVEL)) return nt_load16(p);
    return *p;
}
#ifndef TM_STAGE_IDS
#define TM_STAGE_IDS 8   // ids per stage-row store group (4, 8 or 16): RowEmit
#endif
constexpr uint32_t STAGE_IDS = TM_STAGE_IDS, STAGE_Q = TM_STAGE_IDS / 4;
static_assert(STAGE_IDS == 4 || STAGE_IDS == 8 || STAGE_IDS == 16, "TM_STAGE_IDS: 4, 8 or 16");
__device__ __forceinline__ void store_stage(uint32_t* p, uint4 x) {
    if (TM_NT_STAGE) nt_store16(p, x);
    else *reinterpret_cast<uint4*>(p) = x;
}

// ---------------------------------------------------------------------------
// The walk, in the reference's discovery order (emqx_trie.erl:127-145):
//   at level r < n:  'match_#' (the '#' filter), then the subtree of the
//                    topic word's edge, then the subtree of the '+' edge;
//   at level n:      'match_#', then the node's own filter
// (the reference prepends each discovery, so its result is this sequence
// reversed).  path(r) holds the '+' child still pending at level r while the
// literal subtree below it runs; a step visits one node with one 16 B load
// and then either descends or pops to the deepest pending '+' child.
struct WalkStats {
    uint64_t visits = 0, edge_reads = 0, leaf_visits = 0, probe_loads = 0, prunable = 0;
    unsigned long long* hist = nullptr;   // STATS diagnostics: [visits, probe loads, failed probes] x 16 levels
};
constexpr int HIST_OFF = 8;   // hist = stats + HIST_OFF

// TM_PF1 (A/B builds): a step that visits v at level r also loads the half
// of v's pending '+' sibling (path(r-1)) beside v's own, into one register
// slot; when v turns out to be a dead end the pop to that sibling needs no
// load of its own (one dependent step per topic saved each time)
#ifndef TM_PF1
#define TM_PF1 0
#endif
// TM_PEND_MASK: levels with a pending '+' child as a bit mask in the cursor
// (LDS paths, levels < 32), so a pop reads one path entry (the highest set
// bit below r) instead of scanning the levels down one LDS read at a time
#ifndef TM_PEND_MASK
#define TM_PEND_MASK 1   // A/B at C3: walk 9.78 vs 10.08-10.09 ms (profiles/r03_ab)
#endif
struct Cursor {
    uint32_t v, r, n, r0;   // node to visit next and its level; topic levels; start level
    uint32_t pend;          // TM_PEND_MASK: bit k = path(k) holds a '+' child still to visit (k < r)
    uint64_t key;           // KEYS: fold branches taken above level r (rank_sym), key word 0
    uint32_t pf_id;         // TM_PF1: node whose half is in pf (NODE_NONE: none)
    uint4 pf;
};

// Order keys (sharded mode).  Every match of a topic is identified by the
// branches the reference's fold took to discover it: at level i 'match_#'
// (0), the topic word's edge (1) or the '+' edge (2), and for a node's own
// filter at the last level n an end mark (1).  Discovery order is ascending
// lexicographic order of these sequences (emqx_trie.erl:127-145; SURVEY
// Appendix A.3), so packing them 2 bits per level from the top of u64 words
// makes a key whose DESCENDING order is the reference's output order, and
// per-shard lists merge by key.  Word j holds symbol positions 32j..32j+31;
// a batch keyed with KW words covers topics of up to 32*KW-1 levels.  The
// cursor carries word 0 incrementally; the symbols of positions >= 32 (only
// topics longer than WREG, whose path is in global memory) are read back from
// the path, where every level records the branch it descended by.
__device__ __forceinline__ uint64_t rank_sym(uint32_t level, uint64_t s) {
    return level < 32 ? s << (62 - 2 * level) : 0ull;
}
__device__ __forceinline__ uint64_t rank_prefix(uint64_t key, uint32_t level) {   // symbols of levels < level
    return level == 0 ? 0ull : level >= 32 ? key : key & (~0ull << (64 - 2 * level));
}
// path(k) (KEYS): node id of the '+' child pending at level k (or NODE_NONE)
// | the branch taken at k in bits 29-30
constexpr uint32_t SYM_LIT = 1u << 29, SYM_PLUS = 2u << 29;
// key word j >= 1 of an emission at level r with final symbol sym
template <class Path>
__device__ __forceinline__ uint64_t key_word(const Path& path, uint32_t j, uint32_t r, uint32_t sym) {
    const uint32_t lo = 32 * j;
    if (r < lo) return 0ull;
    uint64_t w = 0;
    const uint32_t hi = r < lo + 32 ? r : lo + 32;
    for (uint32_t p = lo; p < hi; ++p) w |= (uint64_t)((path(p) >> 29) & 3u) << (62 - 2 * (p - lo));
    if (r < lo + 32) w |= (uint64_t)sym << (62 - 2 * (r - lo));
    return w;
}

// topic words in VGPRs (n <= WREG): dynamic index r < WREG by a select tree
// on the bits of r (15 v_cndmask + 4 bit tests; the AND-mask form it
// replaces took three VALU instructions per word, 48 per visit)
#ifndef TM_WSEL_TREE
#define TM_WSEL_TREE 1
#endif
// lane-wise m ? a : b, m a lane mask (v_cndmask_b32 picks src1 where the mask bit is set)
__device__ __forceinline__ uint32_t sel(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t x;
    asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(x) : "v"(b), "v"(a), "s"(m));
    return x;
}
struct RegWords {
    uint32_t w[WREG];
    __device__ __forceinline__ uint32_t operator()(uint32_t r) const {
        static_assert(WREG == 16, "select tree over 16 words");
        if (TM_WSEL_TREE) {
            // the selects as opaque v_cndmask (plain ternaries get turned
            // back into a scratch array indexed by r by the compiler)
            const uint64_t b0 = __ballot((r & 1u) != 0), b1 = __ballot((r & 2u) != 0),
                           b2 = __ballot((r & 4u) != 0), b3 = __ballot((r & 8u) != 0);
            const uint32_t a0 = sel(b0, w[1], w[0]), a1 = sel(b0, w[3], w[2]), a2 = sel(b0, w[5], w[4]),
                           a3 = sel(b0, w[7], w[6]), a4 = sel(b0, w[9], w[8]), a5 = sel(b0, w[11], w[10]),
                           a6 = sel(b0, w[13], w[12]), a7 = sel(b0, w[15], w[14]);
            const uint32_t c0 = sel(b1, a1, a0), c1 = sel(b1, a3, a2), c2 = sel(b1, a5, a4), c3 = sel(b1, a7, a6);
            const uint32_t d0 = sel(b2, c1, c0), d1 = sel(b2, c3, c2);
            return sel(b3, d1, d0);
        }
        uint32_t x = 0;
#pragma unroll
        for (uint32_t k = 0; k < WREG; ++k) x |= w[k] & (0u - (uint32_t)(r == k));
        return x;
    }
};
// topic words in global memory (long topics, re-walks)
struct MemWords {
    const uint32_t* tw;   // levels < WREG
    const uint32_t* lw;   // levels >= WREG
    __device__ __forceinline__ uint32_t operator()(uint32_t r) const { return r < WREG ? tw[r] : lw[r]; }
};

struct LdsPath {
    static constexpr bool kMask = TM_PEND_MASK != 0;   // levels < WREG: the cursor's pending mask applies
    uint32_t* base;   // [level][BLOCK]
    __device__ __forceinline__ uint32_t& operator()(uint32_t r) const { return base[r * BLOCK]; }
};
struct GlobalPath {
    static constexpr bool kMask = false;
    uint32_t* base;
    __device__ __forceinline__ uint32_t& operator()(uint32_t r) const { return base[r]; }
};

// '$' rule (emqx_trie.erl:121-122): a topic whose first word starts with '$'
// starts at node <<W0>>, skipping root's '#' and '+' edges.  false: nothing
// to walk.
template <class Words>
__device__ __forceinline__ bool walk_begin(const ImageView& im, Cursor& c, uint32_t n, bool dollar, const Words& W,
                                           WalkStats& st) {
    c.n = n;
    c.key = 0;
    c.pend = 0;
    c.pf_id = NODE_NONE;
    if (!dollar) {
        c.v = ROOT;
        c.r = c.r0 = 0;
        return true;
    }
    c.key = rank_sym(0, 1);
    const uint4 q = load_half(im, ROOT, false);
    c.v = lit_child<false>(im, ROOT, q.x, q.z, q.w, W(0), st.probe_loads).child;
    c.r = c.r0 = 1;
    return c.v != NODE_NONE;
}

// one step; true when the topic's walk is complete.  A step loads ONE node
// half; a literal child found through the edge table arrives with its record
// (EdgeSlot, TM_SLOT_RECORD builds), so it is visited in the same step, and
// so on down a chain of table children, until a child needs its own load or
// the walk pops.  (A variant that resolved edge probes one slot per step,
// walk_step1, measured 4.10 vs 3.59 ms at C3 and was removed:
// profiles/r01_v12_heat/walk1_ab.json.)
// pop from level r to the deepest pending '+' child; true when the walk is complete
template <bool STATS, bool KEYS, class Path>
__device__ __forceinline__ bool walk_pop(Cursor& c, Path path, uint32_t r, uint64_t key, WalkStats& st) {
    if (Path::kMask) {   // the deepest pending level below r, one path read
        const uint32_t m = c.pend & ((1u << r) - 1u);
        if (!m) return true;
        const uint32_t k = 31u - (uint32_t)__builtin_clz(m);
        const uint32_t p = KEYS ? path(k) & NODE_MASK : path(k);
        if (STATS && st.hist) atomicAdd(st.hist + 50, 1ull);
        if (KEYS) path(k) = NODE_NONE | SYM_PLUS;
        c.pend &= ~(1u << k);
        c.v = p;
        c.r = k + 1;
        if (KEYS) c.key = rank_prefix(key, k) | rank_sym(k, 2);
        return false;
    }
    for (uint32_t k = r; k > c.r0;) {   // scan the path down
        --k;
        const uint32_t p = KEYS ? path(k) & NODE_MASK : path(k);
        if (p != NODE_NONE) {
            if (STATS && st.hist) atomicAdd(st.hist + 50, 1ull);
            path(k) = KEYS ? (NODE_NONE | SYM_PLUS) : NODE_NONE;
            c.v = p;
            c.r = k + 1;
            if (KEYS) c.key = rank_prefix(key, k) | rank_sym(k, 2);
            return false;
        }
    }
    return true;
}

template <bool STATS, bool KEYS, class Path, class Words, class Emit>
__device__ __forceinline__ bool walk_step(const ImageView& im, Cursor& c, Path path, const Words& W, Emit& emit,
                                          WalkStats& st) {
    uint32_t v = c.v, r = c.r;
    uint64_t key = KEYS ? c.key : 0ull;
    bool leaf = r == c.n;
    uint4 h;
    if (TM_PF1 && !STATS) {
        const uint32_t sib = r > c.r0 ? (KEYS ? path(r - 1) & NODE_MASK : path(r - 1)) : NODE_NONE;
        const bool cached = c.pf_id == v;
        const bool pre = sib != NODE_NONE && sib != c.pf_id && sib != v;
        uint4 ph = make_uint4(0, 0, 0, 0);
        h = cached ? c.pf : load_half(im, v, leaf, r);   // the sibling's half is loaded beside v's
        if (pre) ph = load_half(im, sib, leaf, r);
        if (pre) {
            c.pf_id = sib;
            c.pf = ph;
        }
    } else {
        h = load_half(im, v, leaf, r);   // inner {plus, hf, lw, lc} / leaf {sf, hf, hash, pad}
    }
    uint32_t plus = h.x, hf = h.y, lw = h.z, lc = h.w, sf = h.x;
    for (;;) {
        if (STATS) {
            ++st.visits;
            st.edge_reads += leaf ? 1 : 3;   // 'match_#' (:141) + fold over [W, '+'] (:132)
            st.leaf_visits += leaf ? 1 : 0;
        }
        if (!(hf & SUM_TAG)) emit(hf, key, path, r, 0u);   // 'match_#': the '#' filter
        if (leaf) {
            if (sf != FILTER_NONE) emit(sf, KEYS ? key | rank_sym(r, 1) : 0ull, path, r, 1u);   // own filter (:128)
            break;
        }
        const uint64_t pl0 = st.probe_loads;
        // subtree summaries (image.h): a child whose subtree cannot match
        // with k = n - r - 1 levels left below it is never loaded.  The
        // stats walk (STATS) prunes nothing, so its E and visits are the
        // reference's, and counts what the summaries would skip.
        const uint32_t w = W(r);
        bool lit_ok = true, plus_ok = true;
        if (hf & SUM_TAG) {
            const uint32_t k = c.n - r - 1;
            plus_ok = sum_useful(hf & SUM_ALL, k);
            lit_ok = w < WORD_MAX ? sum_useful((hf >> 15) & SUM_ALL, k) : w == WORD_PLUS ? plus_ok : true;
        }
        Hit g = (!STATS && !lit_ok) ? Hit{NODE_NONE, 0, 0, 0, 0, 0, false}
                                    : lit_child<STATS>(im, v, plus, lw, lc, w, st.probe_loads);
        // a table child's own summary (its edge slot's fourth word): the
        // union summary above admitted the literal children as a whole
        const bool child_ok = SLOT_RECORD || g.child == NODE_NONE || sum_useful(g.plus & SUM_ALL, c.n - r - 1);
        if (STATS) st.prunable += (g.child != NODE_NONE && lit_ok && !child_ok) ? 1u : 0u;
        if (!STATS && !child_ok) g.child = NODE_NONE;
        if (STATS && st.hist) {
            const uint32_t lv = r < 15 ? r : 15;
            atomicAdd(st.hist + lv, 1ull);
            if (st.probe_loads != pl0) atomicAdd(st.hist + 16 + lv, (unsigned long long)(st.probe_loads - pl0));
            if (st.probe_loads != pl0 && g.child == NODE_NONE) atomicAdd(st.hist + 32 + lv, 1ull);
        }
        if (STATS) st.prunable += (g.child != NODE_NONE && !lit_ok ? 1u : 0u) +
                                  ((plus & NODE_MASK) != NODE_NONE && !plus_ok ? 1u : 0u);
        const uint32_t pc = (STATS || plus_ok) ? (plus & NODE_MASK) : NODE_NONE;
        if (STATS && st.hist) {   // how the next visit is reached: [48] inline literal, [49] table literal,
                                  // [50] '+' (here or by a later pop: counted at the pop)
            if (g.child != NODE_NONE) atomicAdd(st.hist + ((plus & WIDE) ? 49 : 48), 1ull);
            else if ((plus & NODE_MASK) != NODE_NONE) atomicAdd(st.hist + 50, 1ull);
        }
        if (g.child != NODE_NONE) {   // literal subtree first, '+' child pending at level r
            path(r) = KEYS ? (pc | SYM_LIT) : pc;
            if (Path::kMask) c.pend = pc != NODE_NONE ? (c.pend | (1u << r)) : (c.pend & ~(1u << r));
            v = g.child;
            if (KEYS) key |= rank_sym(r, 1);
            ++r;
            if (!g.have) {
                c.v = v;
                c.r = r;
                if (KEYS) c.key = key;
                return false;
            }
            plus = g.plus;
            hf = g.hf;
            lw = g.lw;
            lc = g.lc;
            sf = g.sf;
            leaf = r == c.n;
            continue;
        }
        if (pc != NODE_NONE) {        // no literal child: straight into the '+' subtree
            path(r) = KEYS ? (NODE_NONE | SYM_PLUS) : NODE_NONE;
            if (Path::kMask) c.pend &= ~(1u << r);
            c.v = pc;
            c.r = r + 1;
            if (KEYS) c.key = key | rank_sym(r, 2);
            return false;
        }
        break;
    }
    return walk_pop<STATS, KEYS>(c, path, r, key, st);   // pop to the deepest pending '+' child
}

template <bool STATS, bool KEYS, class Path, class Words, class Emit>
__device__ __forceinline__ void walk(const ImageView& im, uint32_t n, bool dollar, Path path, const Words& W,
                                     Emit& emit, WalkStats& st) {
    Cursor c;
    if (!walk_begin(im, c, n, dollar, W, st)) return;
    while (!walk_step<STATS, KEYS>(im, c, path, W, emit, st)) {
    }
}

// discovery k of a topic goes to stage row slot K-1-k (k < K); the row's
// last `count` slots are then the output in order.  The ids of a group of
// STAGE_IDS slots are held in registers and stored by back-to-back 16 B
// stores once the group is full: 8 ids = one whole 32 B sector, so the L2
// writes whole sectors to HBM instead of half-filled ones (round 3's one
// store per 4 ids wrote 2.2x the id bytes; at C3 8 ids
// per group cut the walk's fabric write requests from 64.5M to 36.9M per
// launch and the walk from 10.07-10.38 to 9.24-9.40 ms, profiles/r04_g).
// A row ending inside a group (K not a multiple of STAGE_IDS) stores its
// last quads when the row fills.
// KEYS: key word 0 to the same slot of the topic's key row; words j >= 1
// (KW > 1) to key plane j, kplane u64 further on.
template <bool KEYS>
struct RowEmit {
    uint32_t* row;
    uint64_t* krow;
    uint32_t K, cnt;
    uint4 bq[STAGE_Q];   // quad q: slots K-4(q+1)-g .. K-1-4q-g of the current group g (.w highest)
    uint64_t kb;   // KEYS: key of the last even discovery, stored with the next one (16 B)
    uint32_t KW;
    uint64_t kplane;
    // !KEYS: discoveries past K go to spill chunks of this XCD's area
    uint32_t* spill = nullptr;
    unsigned long long* sctr = nullptr;
    uint32_t sbase = 0, scap = 0;
    uint32_t shead = 0, scur = 0;
    bool sfail = false;
    template <class Path>
    __device__ __forceinline__ void operator()(uint32_t f, uint64_t key, const Path& path, uint32_t r, uint32_t sym) {
        if (KEYS && cnt < K) {
            if (!(cnt & 1u)) {
                kb = key;
            } else {   // slots K-2-(cnt-1) and K-1-(cnt-1): this key, then the even one
                *reinterpret_cast<uint4*>(krow + K - 1 - cnt) =
                    make_uint4((uint32_t)key, (uint32_t)(key >> 32), (uint32_t)kb, (uint32_t)(kb >> 32));
            }
            for (uint32_t j = 1; j < KW; ++j) krow[j * kplane + K - 1 - cnt] = key_word(path, j, r, sym);
        }
        if (cnt < K) {
            const uint32_t s = cnt & (STAGE_IDS - 1), g = cnt - s;
#pragma unroll
            for (uint32_t q = 0; q < STAGE_Q; ++q) {
                bq[q].w = s == 4 * q ? f : bq[q].w;
                bq[q].z = s == 4 * q + 1 ? f : bq[q].z;
                bq[q].y = s == 4 * q + 2 ? f : bq[q].y;
                bq[q].x = s == 4 * q + 3 ? f : bq[q].x;
            }
            if (s == STAGE_IDS - 1 || cnt + 1 == K) store_group(s + 1, g);
        } else if (!KEYS && spill && !sfail) {
            const uint32_t o = cnt - K, j = o % (SPILL_CHUNK - 1);
            if (j == 0) {   // a new chunk, linked from the previous one
                const uint32_t c = (uint32_t)atomicAdd(sctr, 1ull);
                if (c >= scap) {
                    sfail = true;
                } else {
                    if (o == 0) shead = sbase + c;
                    else spill[(uint64_t)scur * SPILL_CHUNK] = sbase + c;
                    scur = sbase + c;
                }
            }
            if (!sfail) spill[(uint64_t)scur * SPILL_CHUNK + 1 + j] = f;
        }
        ++cnt;
    }
    // the quads holding the group's first m slots, lowest address first
    __device__ __forceinline__ void store_group(uint32_t m, uint32_t g) {
#pragma unroll
        for (int q = (int)STAGE_Q - 1; q >= 0; --q)
            if (4u * (uint32_t)q < m) store_stage(row + K - 4 * (q + 1) - g, bq[q]);
    }
    __device__ __forceinline__ void flush() {
        const uint32_t s = cnt & (STAGE_IDS - 1);
        if (s && cnt < K) store_group(s, cnt - s);   // a part-filled group (a filled row stored itself)
        if (KEYS && (cnt & 1u) && cnt <= K) krow[K - cnt] = kb;   // the unpaired last even discovery
    }
};
// re-walk of a topic with total > K ids: discovery k >= K goes to output
// position total-1-k (KEYS: with its key words, plane stride kstride)
template <bool KEYS>
struct TailEmit {
    uint32_t* out;
    uint64_t* kout;
    uint64_t base, cap;
    uint32_t K, total, cnt;
    uint32_t KW;
    uint64_t kstride;
    template <class Path>
    __device__ __forceinline__ void operator()(uint32_t f, uint64_t key, const Path& path, uint32_t r, uint32_t sym) {
        if (cnt >= K && cnt < total) {
            const uint64_t p = base + (total - 1 - cnt);
            if (p < cap) {
                out[p] = f;
                if (KEYS) {
                    kout[p] = key;
                    for (uint32_t j = 1; j < KW; ++j) kout[j * kstride + p] = key_word(path, j, r, sym);
                }
            }
        }
        ++cnt;
    }
};

template <bool STATS>
__device__ __forceinline__ void wave_stats_add(unsigned long long* stats, uint64_t lev, uint64_t matches,
                                               const WalkStats& st) {
    if (!STATS) return;
    uint64_t v[7] = {lev, st.visits, st.edge_reads, matches, st.leaf_visits, st.probe_loads, st.prunable};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        uint64_t x = v[k];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(stats + k, (unsigned long long)x);
    }
}

// XCD id of the executing wave (0-7): placement hint only, never correctness
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

// ---------------------------------------------------------------------------
// tm_walk_queue: persistent waves; a wave takes QCHUNK topics at a time from
// a dequeue head, each lane takes the next topic of its wave's chunk the
// moment its walk ends, so no lane or wave idles behind a heavy topic.
// XCDQ: the batch is cut into QRANGES contiguous ranges with one head each
// (ws[16 * r], 128 B apart); a wave drains its own XCD's range first and then
// steals, so neighbouring topics share one XCD's L2.  Otherwise one head.
// Writes counts[t] and the first K ids of t to stage row t.  With perm
// (option "presort"), queue position p walks topic perm[p] from the sorted
// rows twords_s / meta_s, into stage row p (copy-out finds it by pos_of).
constexpr uint32_t QCHUNK = 64;
constexpr uint32_t QRANGES = 8;
constexpr uint32_t NO_TOPIC = 0xFFFFFFFFu;

#if TM_PF1
#define TM_WALK_ATTR __attribute__((amdgpu_waves_per_eu(7, 8)))   // the prefetch slot within 7 waves/SIMD
#elif TM_WALK_WAVES
#define TM_WALK_ATTR __attribute__((amdgpu_waves_per_eu(TM_WALK_WAVES, 8)))   // A/B builds: a register cap
#else
#define TM_WALK_ATTR
#endif
// Chunk rows (CH_ROWS, unkeyed walks in arrival order): when a wave takes a
// chunk, its 64 lanes copy the chunk's rows and meta to LDS at once (lane j
// topic g + j: coalesced, one round trip per chunk), and a lane that takes a
// topic reads its words from LDS instead of waiting on two dependent loads
// (meta, then the row) in the middle of the walk: walk 10.87-10.88 vs
// 11.10-11.13 ms at C3 (profiles/r03_ab/README.md).  Topics of more than CW
// levels read their global row.  (A variant that tokenized the chunk in the
// walk itself, dropping tm_tokenize, measured 13.15-15.89 ms: the tokenizer's
// registers cut the walk's occupancy.)
constexpr uint32_t CW = 8;   // words per topic in the chunk's LDS rows
constexpr int CH_NONE = 0, CH_ROWS = 1;
struct ChunkRows {
    uint32_t w[QCHUNK][CW];
    uint32_t meta[QCHUNK];
    uint32_t topic[QCHUNK];   // the topic at each queue position (presorted batches: perm)
};
template <bool STATS, bool XCDQ, bool KEYS, int CH>
__device__ __forceinline__ void
walk_queue_body(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ twords,
              const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta, uint32_t* __restrict__ gpath,
              uint32_t* __restrict__ stage, uint64_t* __restrict__ kstage, uint32_t K, uint32_t KW,
              uint32_t* __restrict__ counts,
              unsigned long long* __restrict__ ws, unsigned long long* __restrict__ stats,
              unsigned long long* __restrict__ hist, const uint32_t* __restrict__ perm,
              const uint32_t* __restrict__ twords_s, const uint32_t* __restrict__ meta_s,
              uint32_t* __restrict__ spill, uint32_t* __restrict__ spill_head, uint32_t spill_chunks) {
    static_assert(CH == CH_NONE || (!STATS && !KEYS), "chunk rows: unkeyed walks in arrival order only");
    const uint32_t nq = n;
    __shared__ uint32_t lds_path[WREG * BLOCK];
    __shared__ ChunkRows lds_chunk[CH != CH_NONE ? BLOCK / 64 : 1];
    const uint32_t lane = threadIdx.x & 63;
    ChunkRows& CR = lds_chunk[CH != CH_NONE ? threadIdx.x >> 6 : 0];
    const LdsPath lp{lds_path + threadIdx.x};
    GlobalPath gp{nullptr};
    RegWords rw;
    MemWords mw{nullptr, nullptr};
    uint32_t qnext = 0, qend = 0;      // this wave's current chunk (uniform)
    uint32_t cbase = 0;                // CH: queue position of the chunk's LDS row 0 (uniform)
    bool exhausted = false;            // every head ran past its range (uniform)
    const uint32_t home = XCDQ ? xcc_id() : 0u;
    uint32_t qr = 0;                   // ranges given up so far (uniform)
    uint32_t my = NO_TOPIC, myt = 0;   // the lane's queue position and its topic
    bool is_long = false, drained = false;
    Cursor cur;
    RowEmit<KEYS> em{nullptr, nullptr, K, 0, {}, 0ull, KW, (uint64_t)n * K};
    if (!KEYS && spill) {   // this XCD's spill area and counter (placement only: any XCD id is valid)
        const uint32_t x = xcc_id();
        em.spill = spill;
        em.sctr = ws + QWS_SPILL + 16 * x;
        em.scap = spill_chunks / QRANGES;
        em.sbase = x * em.scap;
    }
    WalkStats st;
    if (STATS) st.hist = hist;
    uint64_t lev_sum = 0, match_sum = 0;
    uint32_t maxc = 0;                 // largest list of this lane's topics (stage-row sizing)
    uint32_t maxl = 0;                 // most levels of this lane's topics (key width check of keyed batches)
    // clocks of the walk's phases per XCD (QWS_CLOCK), written as they happen
    // (no registers held across the loop)
    if (TM_WALK_CLOCKS && XCDQ && lane == 0) atomicMax(ws + QWS_CLOCK + 16 * home, (unsigned long long)~wall_clock64());
    for (;;) {
        const bool need = (my == NO_TOPIC) && !drained;
        const uint64_t m = __ballot(need);
        if (m) {
            const uint32_t cm = (uint32_t)__popcll(m);
            uint32_t avail = qend - qnext;
            const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
            uint32_t g = 0, gend = 0;      // new chunk [g, gend), empty if none
            // chunk rows: one chunk in LDS at a time, the next taken once it is used up
            if ((CH != CH_NONE ? avail == 0 : avail < cm) && !exhausted) {
                if (XCDQ) {
                    while (qr < QRANGES) {
                        const uint32_t r = (home + qr) & (QRANGES - 1);
                        const uint32_t rb = (uint32_t)((uint64_t)nq * r / QRANGES);
                        const uint32_t re = (uint32_t)((uint64_t)nq * (r + 1) / QRANGES);
                        uint32_t x = 0;
                        if (lane == leader)
                            x = (uint32_t)__hip_atomic_fetch_add(ws + 16 * r, (unsigned long long)QCHUNK,
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        x = __shfl(x, leader, 64);
                        if (x < re - rb) {
                            g = rb + x;
                            gend = g + QCHUNK < re ? g + QCHUNK : re;
                            if (TM_WALK_CLOCKS && qr != 0 && lane == leader) atomicAdd(ws + QWS_CLOCK + 16 * home + 3, 1ull);
                            break;
                        }
                        if (TM_WALK_CLOCKS && qr == 0 && lane == leader)
                            atomicMax(ws + QWS_CLOCK + 16 * home + 1, (unsigned long long)~wall_clock64());
                        ++qr;
                    }
                    if (qr == QRANGES) exhausted = true;
                } else {
                    uint32_t x = 0;
                    if (lane == leader)
                        x = (uint32_t)__hip_atomic_fetch_add(ws, (unsigned long long)QCHUNK, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
                    x = __shfl(x, leader, 64);
                    if (x < nq) {
                        g = x;
                        gend = g + QCHUNK < nq ? g + QCHUNK : nq;
                    } else {
                        exhausted = true;
                    }
                }
            }
            if (CH != CH_NONE && g < gend) {
                // a new chunk: its rows to LDS, all lanes at once (uniform branch)
                const uint32_t t = g + lane;
                if (t < gend) {
                    // a presorted batch: queue position t walks topic perm[t], whose row
                    // is read here (the rows are not gathered into walk order)
                    const uint32_t tt = perm ? stream_load(perm + t) : t;
                    CR.topic[lane] = tt;
                    CR.meta[lane] = stream_load(meta + tt);
                    const uint4* src = reinterpret_cast<const uint4*>(twords + (uint64_t)tt * WREG);
                    const uint4 a0 = stream_load16(src), a1 = stream_load16(src + 1);   // quad 1 may be stale: unread
                    *reinterpret_cast<uint4*>(&CR.w[lane][0]) = a0;
                    *reinterpret_cast<uint4*>(&CR.w[lane][4]) = a1;
                }
                cbase = g;
                qnext = g;
                qend = gend;
                avail = gend - g;
                g = gend = 0;
                wave_sync_lds();
            }
            if (need) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                uint32_t i = NO_TOPIC;
                if (rank < avail) i = qnext + rank;
                else if (g + (rank - avail) < gend) i = g + (rank - avail);
                if (i != NO_TOPIC) {
                    // i: queue position = stage row; item = ti: the topic, whose
                    // stage row / count / spill head it is (CH: by topic, so a
                    // presorted batch needs no position-ordered copy-out)
                    const uint32_t item = CH != CH_NONE ? CR.topic[i - cbase] : perm ? perm[i] : i;
                    const uint32_t ti = item;
                    const uint32_t* tws = CH == CH_NONE && perm ? twords_s : twords;
                    const uint32_t mt = CH != CH_NONE ? CR.meta[i - cbase] : perm ? meta_s[i] : meta[i];
                    const uint32_t nl = mt & MN;
                    const bool dollar = (mt & MDOLLAR) != 0;
                    lev_sum += nl;
                    maxl = nl > maxl ? nl : maxl;
                    is_long = (mt & MLONG) != 0;
                    em.row = stage + (uint64_t)(CH != CH_NONE ? item : i) * K;
                    if (KEYS) em.krow = kstage + (uint64_t)i * K;
                    em.cnt = 0;
                    em.sfail = false;
                    const uint32_t* tw = tws + (uint64_t)(CH != CH_NONE ? ti : i) * WREG;
                    bool go;
                    if (!is_long && CH != CH_NONE && nl <= CW) {
                        const uint32_t* cw = CR.w[i - cbase];
                        const uint4 a0 = *reinterpret_cast<const uint4*>(cw);
                        const uint4 a1 = *reinterpret_cast<const uint4*>(cw + 4);
                        rw.w[0] = a0.x;
                        rw.w[1] = a0.y;
                        rw.w[2] = a0.z;
                        rw.w[3] = a0.w;
                        rw.w[4] = a1.x;
                        rw.w[5] = a1.y;
                        rw.w[6] = a1.z;
                        rw.w[7] = a1.w;
                        go = walk_begin(im, cur, nl, dollar, rw, st);
                    } else if (!is_long) {
#pragma unroll
                        for (uint32_t k = 0; k < WREG / 4; ++k) {
                            if (4 * k < nl) {
                                const uint4 x = TM_NT_ROWS ? nt_load16(reinterpret_cast<const uint4*>(tw) + k)
                                                           : reinterpret_cast<const uint4*>(tw)[k];
                                rw.w[4 * k] = x.x;
                                rw.w[4 * k + 1] = x.y;
                                rw.w[4 * k + 2] = x.z;
                                rw.w[4 * k + 3] = x.w;
                            }
                        }
                        go = walk_begin(im, cur, nl, dollar, rw, st);
                    } else {
                        const uint64_t b = off[ti] - off[0];
                        mw = MemWords{tw, words + b + ti};
                        gp.base = gpath + b + 2ull * ti;
                        go = walk_begin(im, cur, nl, dollar, mw, st);
                    }
                    if (go) {
                        my = i;
                        myt = item;
                    } else {
                        counts[item] = 0;
                    }
                } else if (exhausted) {
                    drained = true;
                }
            }
            // advance the wave's chunk (uniform)
            if (CH != CH_NONE) {
                qnext += avail < cm ? avail : cm;
            } else if (avail >= cm) {
                qnext += cm;
            } else if (g < gend) {
                qnext = g + (cm - avail);
                qend = gend;
                if (qnext > qend) qnext = qend;
            } else {
                qnext = qend;
            }
        }
        if (__all(my == NO_TOPIC && drained)) break;
        if (my == NO_TOPIC) continue;
        const bool fin = is_long ? walk_step<STATS, KEYS>(im, cur, gp, mw, em, st)
                                 : walk_step<STATS, KEYS>(im, cur, lp, rw, em, st);
        if (fin) {
            em.flush();
            counts[myt] = em.cnt;
            if (!KEYS && spill && em.cnt > K) spill_head[myt] = em.sfail ? NO_SPILL : em.shead;
            match_sum += em.cnt;
            maxc = em.cnt > maxc ? em.cnt : maxc;
            my = NO_TOPIC;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)maxc, o, 64);
        maxc = y > maxc ? y : maxc;
    }
    if (lane == 0 && maxc) atomicMax(ws + QWS_MAXC, (unsigned long long)maxc);
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)maxl, o, 64);
        maxl = y > maxl ? y : maxl;
    }
    if (lane == 0 && maxl) atomicMax(ws + QWS_MAXL, (unsigned long long)maxl);
    if (TM_WALK_CLOCKS && XCDQ && lane == 0) atomicMax(ws + QWS_CLOCK + 16 * home + 2, (unsigned long long)wall_clock64());
    wave_stats_add<STATS>(stats, lev_sum, match_sum, st);
}

template <bool STATS, bool XCDQ, bool KEYS, int CH = CH_NONE>
__global__ void __launch_bounds__(BLOCK) TM_WALK_ATTR
tm_walk_queue(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ twords,
              const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta, uint32_t* __restrict__ gpath,
              uint32_t* __restrict__ stage, uint64_t* __restrict__ kstage, uint32_t K, uint32_t KW,
              uint32_t* __restrict__ counts,
              unsigned long long* __restrict__ ws, unsigned long long* __restrict__ stats,
              unsigned long long* __restrict__ hist, const uint32_t* __restrict__ perm,
              const uint32_t* __restrict__ twords_s, const uint32_t* __restrict__ meta_s,
              uint32_t* __restrict__ spill, uint32_t* __restrict__ spill_head, uint32_t spill_chunks) {
    walk_queue_body<STATS, XCDQ, KEYS, CH>(im, off, n, twords, words, meta, gpath, stage, kstage, K, KW, counts, ws, stats, hist, perm, twords_s, meta_s,
                                     spill, spill_head, spill_chunks);
}
// ---------------------------------------------------------------------------
// tm_walk_wave: the low-latency walk (small batches: engine option
// "wave_walk_max").  One wave per topic, level by level: at level r the
// lanes take the frontier's nodes (one load each, all in flight together),
// emit, and push the children, so a topic costs about two dependent loads
// per level instead of one per visited node (the per-lane walk above, which
// is what a large batch wants: no idle lanes).  Every emission carries its
// rank key (rank_sym: the fold's branch per level, emqx_trie.erl:127-145),
// and sorting the topic's emissions by key restores the reference's
// discovery order, whose first K go to the stage row as the
// per-lane walk writes them (discovery k at slot K-1-k).  A topic beyond the
// wave's frontier or emission capacity, or past WREG levels, takes the
// per-lane walk on lane 0; lists past K are re-walked by the copy-out.
constexpr uint32_t WV_F = 256;   // frontier entries per level, per wave
constexpr uint32_t WV_E = 512;   // emissions per topic held for the sort
struct WaveLds {
    uint32_t fnode[2][WV_F];
    uint64_t fkey[2][WV_F];
    uint64_t ekey[WV_E];
    uint32_t eid[WV_E];
    uint32_t words[WREG];
};

// lane-ordered append of this lane's item when `has`: returns the slot, adds
// the wave's count to `n` (uniform)
__device__ __forceinline__ uint32_t wave_append(bool has, uint32_t& n) {
    const uint64_t m = __ballot(has);
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const uint32_t at = n + r;
    n += (uint32_t)__popcll(m);
    return at;
}

// one topic's level-synchronous walk by one wave: the topic's words are in
// L.words; on return the emissions are in L.eid[0, ec) in discovery order
// (ascending key), or the result is false: the frontier or the emissions
// outgrew the wave's LDS (the caller walks the topic per lane instead)
__device__ __forceinline__ bool wave_walk_topic(const ImageView& im, WaveLds& L, uint32_t nl, bool dollar,
                                                uint32_t lane, uint32_t& ec_out) {
    uint32_t ec = 0;
    bool fallback = false;
    // the start: root, or (the '$' rule, emqx_trie.erl:121-122) the root's
    // literal child by the first word, skipping '#' and '+'
    uint32_t fc = 0, p = 0, r = 0;
    if (lane == 0) {
        if (!dollar) {
            L.fnode[0][0] = ROOT;
            L.fkey[0][0] = 0;
            fc = 1;
        } else {
            uint64_t ld = 0;
            const uint4 q = load_half(im, ROOT, false);
            const uint32_t c = lit_child<false>(im, ROOT, q.x, q.z, q.w, L.words[0], ld).child;
            if (c != NODE_NONE) {
                L.fnode[0][0] = c;
                L.fkey[0][0] = rank_sym(0, 1);
                fc = 1;
            }
        }
    }
    fc = (uint32_t)__shfl((int)fc, 0, 64);
    r = dollar ? 1u : 0u;
    wave_sync_lds();
    for (; fc && !fallback; ++r) {
        const bool leaf = r == nl;
        const uint32_t w = leaf ? 0u : L.words[r];
        const uint32_t kleft = nl - r - 1;
        uint32_t nf = 0;
        for (uint32_t base = 0; base < fc; base += 64) {
            const uint32_t i = base + lane;
            const bool act = i < fc;
            const uint32_t v = act ? L.fnode[p][i] : NODE_NONE;
            const uint64_t key = act ? L.fkey[p][i] : 0ull;
            uint4 h = make_uint4(FILTER_NONE, FILTER_NONE, WORD_NONE, NODE_NONE);
            if (act) h = load_half(im, v, leaf, r);
            // 'match_#': the '#' child's filter, discovered first (rank 0 at r)
            uint32_t e1 = act && !(h.y & SUM_TAG) ? h.y : FILTER_NONE;
            uint32_t e2 = FILTER_NONE, c1 = NODE_NONE, c2 = NODE_NONE;
            if (act && leaf) {
                e2 = h.x;   // the node's own filter (emqx_trie.erl:128), end mark 1
            } else if (act) {
                const uint32_t plus = h.x, hf = h.y;
                bool lit_ok = true, plus_ok = true;
                if (hf & SUM_TAG) {
                    plus_ok = sum_useful(hf & SUM_ALL, kleft);
                    lit_ok = w < WORD_MAX ? sum_useful((hf >> 15) & SUM_ALL, kleft)
                                          : w == WORD_PLUS ? plus_ok : true;
                }
                uint64_t ld = 0;
                if (lit_ok) {
                    const Hit g = lit_child<false>(im, v, plus, h.z, h.w, w, ld);
                    if (g.child != NODE_NONE && (SLOT_RECORD || sum_useful(g.plus & SUM_ALL, kleft)))
                        c1 = g.child;
                }
                if (plus_ok) c2 = plus & NODE_MASK;
            }
            // emissions (any order: the keys sort them)
            uint32_t a = wave_append(e1 != FILTER_NONE, ec);
            if (e1 != FILTER_NONE && a < WV_E) {
                L.ekey[a] = key;
                L.eid[a] = e1;
            }
            a = wave_append(e2 != FILTER_NONE, ec);
            if (e2 != FILTER_NONE && a < WV_E) {
                L.ekey[a] = key | rank_sym(r, 1);
                L.eid[a] = e2;
            }
            // children for level r + 1: the topic word's edge (1), the '+' edge (2)
            a = wave_append(c1 != NODE_NONE, nf);
            if (c1 != NODE_NONE && a < WV_F) {
                L.fnode[1 - p][a] = c1;
                L.fkey[1 - p][a] = key | rank_sym(r, 1);
            }
            a = wave_append(c2 != NODE_NONE, nf);
            if (c2 != NODE_NONE && a < WV_F) {
                L.fnode[1 - p][a] = c2;
                L.fkey[1 - p][a] = key | rank_sym(r, 2);
            }
        }
        wave_sync_lds();
        if (nf > WV_F || ec > WV_E) fallback = true;   // uniform
        if (leaf) break;
        fc = nf;
        p = 1 - p;
    }
    if (fallback) return false;
    // discovery order = ascending key: bitonic sort of the topic's emissions
    // in LDS (padded with keys that sort last)
    uint32_t P = 64;
    while (P < ec) P <<= 1;
    for (uint32_t i = ec + lane; i < P; i += 64) {
        L.ekey[i] = ~0ull;
        L.eid[i] = FILTER_NONE;
    }
    wave_sync_lds();
    if (ec > 1) {
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = lane; i < P; i += 64) {
                    const uint32_t l = i ^ j;
                    if (l > i) {
                        const uint64_t x = L.ekey[i], y = L.ekey[l];
                        if ((x > y) == ((i & k) == 0)) {
                            const uint32_t xi = L.eid[i];
                            L.ekey[i] = y;
                            L.ekey[l] = x;
                            L.eid[i] = L.eid[l];
                            L.eid[l] = xi;
                        }
                    }
                }
                wave_sync_lds();
            }
        }
    }
    ec_out = ec;
    return true;
}

__global__ void __launch_bounds__(BLOCK)
tm_walk_wave(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ twords,
             const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta, uint32_t* __restrict__ gpath,
             uint32_t* __restrict__ stage, uint32_t K, uint32_t* __restrict__ counts,
             uint32_t* __restrict__ spill_head, unsigned long long* __restrict__ ws) {
    __shared__ WaveLds lds_all[BLOCK / 64];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    WaveLds& L = lds_all[wv];
    uint32_t maxl = 0;   // most levels of the wave's topics (QWS_MAXL: key width check of keyed batches)
    for (uint32_t t = blockIdx.x * (BLOCK / 64) + wv; t < n; t += gridDim.x * (BLOCK / 64)) {
        const uint32_t mt = meta[t];
        const uint32_t nl = mt & MN;
        maxl = nl > maxl ? nl : maxl;   // uniform: one topic per wave
        const bool dollar = (mt & MDOLLAR) != 0;
        const uint32_t* row = twords + (uint64_t)t * WREG;
        uint32_t* srow = stage + (uint64_t)t * K;
        bool fallback = (mt & MLONG) != 0 || nl > 31;
        uint32_t ec = 0;
        if (!fallback) {
            if (lane < WREG && lane < nl) L.words[lane] = row[lane];
            wave_sync_lds();
            fallback = !wave_walk_topic(im, L, nl, dollar, lane, ec);
        }
        if (!fallback) {
            const uint32_t m = ec < K ? ec : K;
            for (uint32_t k = lane; k < m; k += 64) srow[K - 1 - k] = L.eid[k];
            if (lane == 0) {
                counts[t] = ec;
                if (ec > K && spill_head) spill_head[t] = NO_SPILL;   // the copy-out re-walks the head
            }
        } else if (lane == 0) {
            // beyond the wave's capacity: the per-lane walk, on one lane
            const uint64_t b = off[t] - off[0];
            const MemWords mw{row, words + b + t};
            RowEmit<false> em{srow, nullptr, K, 0, {}, 0ull, 1u, 0ull};
            WalkStats s2;
            walk<false, false>(im, nl, dollar, GlobalPath{gpath + b + 2ull * t}, mw, em, s2);
            em.flush();
            counts[t] = em.cnt;
            if (em.cnt > K && spill_head) spill_head[t] = NO_SPILL;
        }
        wave_sync_lds();
    }
    if (lane == 0 && maxl && ws) atomicMax(ws + QWS_MAXL, (unsigned long long)maxl);
}

// tm_match_small: a small batch in ONE launch (the micro-batcher's path,
// engine.cpp match_small; a small batch's time is per-operation latency).
// One wave per topic: lane 0 tokenizes it (tokenize_one: the row, words and
// meta as tm_tokenize writes them), the wave walks it level by level
// (wave_walk_topic), reserves its list's range with one atomic and writes
// the list in emqx_trie:match/1 order (reverse discovery order) straight to
// the output.  Lists are contiguous per topic but placed in completion
// order: out_off[t] is topic t's start, not an exclusive scan.  Topics past
// the wave's capacity walk per lane on lane 0, twice (count, then emit).
// ctl[0] = ids placed, ctl[1] = waves done: the last wave to finish writes
// *total and zeroes both for the next launch on the same ctl (the engine
// keeps one per batch slot, zeroed when it is allocated).
__global__ void __launch_bounds__(BLOCK)
tm_match_small(ImageView im, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint32_t n,
               uint32_t* __restrict__ twords, uint32_t* __restrict__ words, uint32_t* __restrict__ meta,
               uint32_t* __restrict__ gpath, uint32_t* __restrict__ counts, uint64_t* __restrict__ out_off,
               uint32_t* __restrict__ out, uint64_t cap, uint64_t* __restrict__ total,
               unsigned long long* __restrict__ ctl) {
    __shared__ WaveLds lds_all[BLOCK / 64];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    WaveLds& L = lds_all[wv];
    for (uint32_t t = blockIdx.x * (BLOCK / 64) + wv; t < n; t += gridDim.x * (BLOCK / 64)) {
        const uint64_t b = off[t] - off[0];
        uint32_t mt = 0;
        if (lane == 0) {
            tokenize_one(im, GlobalBytes{bytes}, off, t, n, twords, words, meta, nullptr, nullptr, 0u);
            mt = meta[t];   // this lane's own store
            const uint32_t* row = twords + (uint64_t)t * WREG;
#pragma unroll
            for (uint32_t k = 0; k < WREG; ++k) L.words[k] = row[k];
        }
        mt = (uint32_t)__shfl((int)mt, 0, 64);
        wave_sync_lds();
        const uint32_t nl = mt & MN;
        const bool dollar = (mt & MDOLLAR) != 0;
        uint32_t ec = 0;
        bool fallback = (mt & MLONG) != 0 || nl > 31;
        if (!fallback) fallback = !wave_walk_topic(im, L, nl, dollar, lane, ec);
        if (!fallback) {
            uint64_t base = 0;
            if (lane == 0) base = atomicAdd(ctl, (unsigned long long)ec);
            base = __shfl(base, 0, 64);
            if (base + ec <= cap)
                for (uint32_t j = lane; j < ec; j += 64) out[base + j] = L.eid[ec - 1 - j];
            if (lane == 0) {
                counts[t] = ec;
                out_off[t] = base;
            }
        } else if (lane == 0) {
            // the per-lane walk: count, reserve, then emit at base + (c-1-k)
            const MemWords mw{twords + (uint64_t)t * WREG, words + b + t};
            const GlobalPath gp{gpath + b + 2ull * t};
            RowEmit<false> cnt{nullptr, nullptr, 0u, 0, {}, 0ull, 1u, 0ull};
            WalkStats s2;
            walk<false, false>(im, nl, dollar, gp, mw, cnt, s2);
            const uint64_t base = atomicAdd(ctl, (unsigned long long)cnt.cnt);
            if (base + cnt.cnt <= cap) {
                TailEmit<false> em{out, nullptr, base, cap, 0u, cnt.cnt, 0, 1u, 0ull};
                walk<false, false>(im, nl, dollar, gp, mw, em, s2);
            }
            counts[t] = cnt.cnt;
            out_off[t] = base;
        }
        wave_sync_lds();
    }
    // the last wave out publishes the total and re-arms ctl
    if (lane == 0) {
        __threadfence();
        const unsigned long long waves = (unsigned long long)gridDim.x * (BLOCK / 64);
        if (atomicAdd(ctl + 1, 1ull) == waves - 1) {
            *total = atomicAdd(ctl, 0ull);
            atomicExch(ctl, 0ull);
            atomicExch(ctl + 1, 0ull);
        }
    }
}

// tm_copy_out: per 256 topics, the block's output range is copied from the
// stage rows with coalesced writes (output index -> topic by binary search of
// the block's inclusive prefix); output j of a topic with c ids is row slot
// K-c+j; a topic with c > K re-walks and writes its first c-K outputs.
// blocks whose mean fan-out reaches COPY_WAVE_MIN ids per topic copy one
// topic per wave (no per-id search)
#ifndef TM_COPY_FLAT
#define TM_COPY_FLAT 0   // A/B builds: the flat coalesced copy for every block
#endif
#ifndef TM_COPY_WAVE_MIN
#define TM_COPY_WAVE_MIN 16   // A/B at C3: copy-out 0.322 (64) vs 0.283-0.293 ms (16, 0)
#endif
constexpr uint32_t COPY_WAVE_MIN = TM_COPY_WAVE_MIN;
#ifndef TM_COPY_NT
#define TM_COPY_NT 0   // A/B builds: the unkeyed copy-out's stage reads and output stores non-temporal
#endif
#ifndef TM_COPY_U
#define TM_COPY_U 8   // unkeyed copy-out: topics per wave with their row loads in flight together (1: one at a time;
                      // 8 vs 4: 0.803-0.809 vs 0.827-0.843 ms at C3 8M, profiles/r06_h_ab, r06_i_ab)
#endif
constexpr uint32_t COPY_U = TM_COPY_U;

// SHAPED (option "shape_keys"): a keyed batch walked unkeyed; each id's key
// is its filter's order key im.fshape[id] (image.h filter_shape), and a
// topic with a literal '+' / '#' level (MOOD: its walk repeats subtrees, so
// keys by filter would tie) is re-walked keyed here, all of its outputs.
template <bool KEYS, bool SHAPED>
__global__ void __launch_bounds__(BLOCK)
tm_copy_out(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ twords,
            const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta, uint32_t* __restrict__ gpath,
            const uint32_t* __restrict__ stage, const uint64_t* __restrict__ kstage, uint32_t K, uint32_t KW,
            const uint32_t* __restrict__ counts, const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out,
            uint64_t* __restrict__ kout, uint64_t out_cap, const uint32_t* __restrict__ spill,
            const uint32_t* __restrict__ spill_head) {
    const uint64_t kplane = (uint64_t)n * K;   // KEYS: key word j of stage slot x at kstage[j * kplane + x],
                                               // of output p at kout[j * out_cap + p]
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
    // topics copied by the loops below: not out-of-domain (SHAPED)
    auto ood = [&](uint32_t lt) { return SHAPED && (meta[t0 + lt] & MOOD) != 0; };
    auto put = [&](uint64_t p, uint32_t id) {
        if (TM_COPY_NT) __builtin_nontemporal_store(id, out + p);
        else out[p] = id;
        if (SHAPED) kout[p] = im.fshape[id];
    };
    if (TM_COPY_FLAT) {
        // flat and coalesced: thread x copies outputs base + x, base + x +
        // BLOCK, ... (U of them in flight); the topic of an output advances
        // monotonically per thread over the block's inclusive prefix
        constexpr int U = 4;
        uint32_t lo = 0;
        for (uint64_t j0 = threadIdx.x; j0 < agg; j0 += (uint64_t)BLOCK * U) {
            uint32_t v[U];
            uint64_t src[U];
            bool ok[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t j = j0 + (uint64_t)u * BLOCK;
                ok[u] = false;
                if (j >= agg) continue;
                while ((uint64_t)lds_inc[lo] <= j) ++lo;
                const uint32_t prev = lo ? lds_inc[lo - 1] : 0u;
                const uint32_t ct = lds_inc[lo] - prev;
                const int64_t slot = (int64_t)K - (int64_t)ct + (int64_t)(j - prev);   // < 0: head past K
                ok[u] = slot >= 0 && base + j < out_cap && !ood(lo);
                src[u] = (uint64_t)(t0 + lo) * K + (uint64_t)(slot < 0 ? 0 : slot);
                if (ok[u]) v[u] = stage[src[u]];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ok[u]) continue;
                const uint64_t p = base + j0 + (uint64_t)u * BLOCK;
                put(p, v[u]);
                if (KEYS)
                    for (uint32_t q = 0; q < KW; ++q) kout[q * out_cap + p] = kstage[q * kplane + src[u]];
            }
        }
    } else if (!KEYS && COPY_U > 1 && agg >= (uint64_t)COPY_WAVE_MIN * tn) {
        // high fan-out block, unkeyed: each wave copies a contiguous quarter
        // of the block's topics, COPY_U topics at a time with all their row
        // loads (two per lane: 128 ids) issued before the first store, so a
        // wave has 2 x COPY_U loads in flight instead of one topic's; ids of
        // a row past 128 (widened rows) in a loop after
        const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const uint32_t q = (tn + 3) / 4, la = w * q, lz = la + q < tn ? la + q : tn;
        for (uint32_t l0 = la; l0 < lz; l0 += COPY_U) {
            uint32_t v0[COPY_U], v1[COPY_U];
#pragma unroll
            for (uint32_t u = 0; u < COPY_U; ++u) {
                const uint32_t lt = l0 + u;
                v0[u] = v1[u] = 0;
                if (lt < lz) {
                    const uint32_t prev = lt ? lds_inc[lt - 1] : 0u;
                    const uint32_t ct = lds_inc[lt] - prev;
                    const uint32_t j = (ct > K ? ct - K : 0u) + lane;
                    const uint64_t row = (uint64_t)(t0 + lt) * K + K - ct;
                    if (j < ct) v0[u] = TM_COPY_NT || TM_NT_STREAM ? __builtin_nontemporal_load(stage + row + j) : stage[row + j];
                    if (j + 64 < ct)
                        v1[u] = TM_COPY_NT || TM_NT_STREAM ? __builtin_nontemporal_load(stage + row + j + 64)
                                                          : stage[row + j + 64];
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < COPY_U; ++u) {
                const uint32_t lt = l0 + u;
                if (lt >= lz || ood(lt)) continue;
                const uint32_t prev = lt ? lds_inc[lt - 1] : 0u;
                const uint32_t ct = lds_inc[lt] - prev;
                const uint64_t ob = base + prev;
                const uint64_t row = (uint64_t)(t0 + lt) * K + K - ct;
                const uint32_t j = (ct > K ? ct - K : 0u) + lane;
                if (j < ct && ob + j < out_cap) put(ob + j, v0[u]);
                if (j + 64 < ct && ob + j + 64 < out_cap) put(ob + j + 64, v1[u]);
                for (uint32_t jj = j + 128; jj < ct; jj += 64)
                    if (ob + jj < out_cap) put(ob + jj, stage[row + jj]);
            }
        }
    } else if (agg >= (uint64_t)COPY_WAVE_MIN * tn) {
        // high fan-out block: one wave per topic, its lanes stride the row
        // (no per-id search); output j of a topic with ct ids is row slot
        // K-ct+j, staged for j >= ct-K
        const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        for (uint32_t lt = w; lt < tn; lt += BLOCK / 64) {
            const uint32_t prev = lt ? lds_inc[lt - 1] : 0u;
            const uint32_t ct = lds_inc[lt] - prev;
            if (ood(lt)) continue;
            const uint64_t ob = base + prev;
            const uint64_t row = (uint64_t)(t0 + lt) * K + K - ct;   // + j: slot of output j
            for (uint32_t j = (ct > K ? ct - K : 0u) + lane; j < ct; j += 64) {
                if (ob + j < out_cap) {
                    put(ob + j, stage[row + j]);
                    if (KEYS)
                        for (uint32_t q = 0; q < KW; ++q) kout[q * out_cap + ob + j] = kstage[q * kplane + row + j];
                }
            }
        }
    } else for (uint64_t j = threadIdx.x; j < agg; j += BLOCK) {
        uint32_t lo = 0, hi = tn - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)lds_inc[mid] > j) hi = mid; else lo = mid + 1;
        }
        const uint32_t prev = lo ? lds_inc[lo - 1] : 0u;
        const uint32_t k = (uint32_t)(j - prev);
        const uint32_t ct = lds_inc[lo] - prev;
        const int64_t slot = (int64_t)K - (int64_t)ct + (int64_t)k;
        if (slot >= 0 && base + j < out_cap && !ood(lo)) {
            put(base + j, stage[(uint64_t)(t0 + lo) * K + (uint64_t)slot]);
            if (KEYS)
                for (uint32_t q = 0; q < KW; ++q)
                    kout[q * out_cap + base + j] = kstage[q * kplane + (uint64_t)(t0 + lo) * K + (uint64_t)slot];
        }
    }
    if (!KEYS && spill) {
        // the head of a list past K ids (outputs [0, ct - K), in reverse
        // discovery order) from its spill chunks, one wave per topic
        const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        for (uint32_t lt = w; lt < tn; lt += BLOCK / 64) {
            const uint32_t prev = lt ? lds_inc[lt - 1] : 0u;
            const uint32_t ct = lds_inc[lt] - prev;
            if (ct <= K || ood(lt)) continue;
            uint32_t cur = spill_head[t0 + lt];
            if (cur == NO_SPILL) continue;   // re-walked below
            const uint32_t m = ct - K;
            const uint64_t ob = base + prev;
            for (uint32_t o0 = 0; o0 < m; o0 += SPILL_CHUNK - 1) {
                for (uint32_t j = lane; j < SPILL_CHUNK - 1 && o0 + j < m; j += 64) {
                    const uint64_t p = ob + m - 1 - (o0 + j);
                    if (p < out_cap) put(p, spill[(uint64_t)cur * SPILL_CHUNK + 1 + j]);
                }
                if (o0 + SPILL_CHUNK - 1 < m) cur = spill[(uint64_t)cur * SPILL_CHUNK];
            }
        }
    }
    const bool tail = c > K && (KEYS || !spill || spill_head[t0 + threadIdx.x] == NO_SPILL);
    if (threadIdx.x < tn && (tail || ood(threadIdx.x))) {
        // fan-out beyond the stage row and no spill: walk again, write the
        // head; SHAPED: keyed, and every output of an out-of-domain topic
        const uint32_t t = t0 + threadIdx.x;
        const uint32_t mt = meta[t];
        const uint64_t b = off[t] - off[0];
        const MemWords mw{twords + (uint64_t)t * WREG, words + b + t};
        constexpr bool WK = KEYS || SHAPED;
        TailEmit<WK> em{out, kout, base + ex, out_cap, ood(threadIdx.x) ? 0u : K, c, 0, KW, out_cap};
        WalkStats s2;
        // the topic's global path area (the walk's, for long topics): no LDS
        // path here, so the copy-out's blocks stay small (1.3 KB of LDS)
        walk<false, WK>(im, mt & MN, (mt & MDOLLAR) != 0, GlobalPath{gpath + b + 2ull * t}, mw, em, s2);
    }
}

// tm_copy_out over a presorted walk (option "presort"): stage row p holds
// topic perm[p].  A block takes 256 positions: its threads fetch each one's
// topic, count and output offset at once (the random reads overlap), then
// one wave per position copies the row to the topic's output range (rows
// read in order, each topic's output written contiguously); a topic past K
// ids has its head re-walked by its thread
template <bool KEYS>
__global__ void __launch_bounds__(BLOCK)
tm_copy_out_sorted(ImageView im, const uint64_t* __restrict__ off, uint32_t n, const uint32_t* __restrict__ twords,
                   const uint32_t* __restrict__ words, const uint32_t* __restrict__ meta,
                   uint32_t* __restrict__ gpath, const uint32_t* __restrict__ stage,
                   const uint64_t* __restrict__ kstage, uint32_t K, uint32_t KW, const uint32_t* __restrict__ counts,
                   const uint64_t* __restrict__ out_off, uint32_t* __restrict__ out, uint64_t* __restrict__ kout,
                   uint64_t out_cap, const uint32_t* __restrict__ perm) {
    __shared__ uint32_t s_c[BLOCK];
    __shared__ uint64_t s_o[BLOCK];
    const uint64_t kplane = (uint64_t)n * K;
    const uint32_t p0 = blockIdx.x * BLOCK;
    const uint32_t tn = n - p0 < (uint32_t)BLOCK ? n - p0 : (uint32_t)BLOCK;
    uint32_t t = 0, c = 0;
    uint64_t ob = 0;
    if (threadIdx.x < tn) {
        t = perm[p0 + threadIdx.x];
        c = counts[t];
        ob = out_off[t];
    }
    s_c[threadIdx.x] = c;
    s_o[threadIdx.x] = ob;
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t lt = w; lt < tn; lt += BLOCK / 64) {
        const uint32_t ct = s_c[lt];
        const uint64_t o = s_o[lt];
        const uint64_t row = (uint64_t)(p0 + lt) * K + K - ct;   // + j: slot of output j (j >= ct - K)
        for (uint32_t j = (ct > K ? ct - K : 0u) + lane; j < ct; j += 64)
            if (o + j < out_cap) {
                out[o + j] = stage[row + j];
                if (KEYS)
                    for (uint32_t q = 0; q < KW; ++q) kout[q * out_cap + o + j] = kstage[q * kplane + row + j];
            }
    }
    if (threadIdx.x < tn && c > K) {   // fan-out beyond the stage row: walk again, write the head
        const uint32_t mt = meta[t];
        const uint64_t b = off[t] - off[0];
        const MemWords mw{twords + (uint64_t)t * WREG, words + b + t};
        TailEmit<KEYS> em{out, kout, ob, out_cap, K, c, 0, KW, out_cap};
        WalkStats s2;
        walk<false, KEYS>(im, mt & MN, (mt & MDOLLAR) != 0, GlobalPath{gpath + b + 2ull * t}, mw, em, s2);
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

// one resident wave set: blocks per CU at full occupancy x CUs
template <typename Kern>
static uint32_t resident_grid(Kern k, uint32_t n_tiles, uint32_t cap_per_cu = 0) {
    int dev = 0, cus = 256, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, BLOCK, 0);
    if (cap_per_cu && per > (int)cap_per_cu) per = (int)cap_per_cu;
    uint32_t g = (uint32_t)((per > 0 ? per : 1) * (cus > 0 ? cus : 1));
    return g < n_tiles ? g : n_tiles;
}

// split image: node records -> separate arrays of inner and leaf halves
__global__ void __launch_bounds__(BLOCK)
tm_split_nodes(const uint4* __restrict__ nodes, uint64_t n, uint4* __restrict__ inner, uint4* __restrict__ leaf) {
    for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < n; v += (uint64_t)gridDim.x * BLOCK) {
        inner[v] = nodes[2 * v];
        leaf[v] = nodes[2 * v + 1];
    }
}


hipError_t launch_split_nodes(const void* nodes, uint64_t n, void* inner, void* leaf, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(tm_split_nodes, dim3((uint32_t)(blocks < 8192 ? blocks : 8192)), dim3(BLOCK), 0, st,
                       (const uint4*)nodes, n, (uint4*)inner, (uint4*)leaf);
    return hipGetLastError();
}

// commit: the elements a host table changed since an image last saw it, as
// one packet [idx u32 x n][values: words u32 x n], written into the image's
// copy of the table (later duplicates of an index carry the same value)
__global__ void __launch_bounds__(BLOCK)
tm_scatter(uint32_t* __restrict__ table, const uint32_t* __restrict__ pkt, uint64_t n, uint32_t words) {
    const uint32_t* vals = pkt + n;
    const uint64_t total = n * words;
    for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < total; t += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t i = t / words;
        table[(uint64_t)pkt[i] * words + (t - i * words)] = vals[t];
    }
}

hipError_t launch_scatter(void* table, const uint32_t* pkt, uint64_t n, uint32_t words, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n * words + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(tm_scatter, dim3((uint32_t)(blocks < 16384 ? blocks : 16384)), dim3(BLOCK), 0, st,
                       (uint32_t*)table, pkt, n, words);
    return hipGetLastError();
}

size_t scan_tmp_elems(uint32_t n) { return div_up(n ? n : 1, SCAN_TILE); }

// a small batch's scan in one launch: one block over the tiles in turn,
// carrying the running total (a small batch's time is per-launch latency)
__global__ void __launch_bounds__(BLOCK)
tm_scan_single(const uint32_t* __restrict__ in, uint32_t n, uint64_t* __restrict__ out_off,
               uint64_t* __restrict__ total) {
    __shared__ uint64_t lds[BLOCK / 64];
    uint64_t carry = 0;
    for (uint64_t t0 = 0; t0 < n; t0 += SCAN_TILE) {
        const uint64_t base = t0 + (uint64_t)threadIdx.x * SCAN_ITEMS;
        uint32_t v[SCAN_ITEMS];
        uint64_t s = 0;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const uint64_t k = base + i;
            v[i] = k < n ? in[k] : 0;
            s += v[i];
        }
        uint64_t tot;
        uint64_t ex = block_exclusive_scan(s, lds, tot) + carry;
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const uint64_t k = base + i;
            if (k < n) out_off[k] = ex;
            ex += v[i];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        out_off[n] = carry;
        *total = carry;
    }
}
constexpr uint32_t SCAN_SINGLE_MAX = 32768;   // batches up to this size scan in one launch

hipError_t launch_scan(const uint32_t* counts, uint32_t n, uint64_t* out_off, uint64_t* total, uint64_t* tmp,
                       hipStream_t st) {
    if (n <= SCAN_SINGLE_MAX) {
        hipLaunchKernelGGL(tm_scan_single, dim3(1), dim3(BLOCK), 0, st, counts, n, out_off, total);
        return hipGetLastError();
    }
    uint32_t tiles = div_up(n, SCAN_TILE);
    hipLaunchKernelGGL(tm_scan_reduce, dim3(tiles), dim3(BLOCK), 0, st, counts, n, tmp);
    hipLaunchKernelGGL(tm_scan_tiles, dim3(1), dim3(BLOCK), 0, st, tmp, tiles);
    hipLaunchKernelGGL(tm_scan_final, dim3(tiles), dim3(BLOCK), 0, st, counts, n, tmp, out_off, total);
    return hipGetLastError();
}

hipError_t launch_small(const ImageView& im, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t* twords,
                        uint32_t* words, uint32_t* meta, uint32_t* gpath, uint32_t* counts, uint64_t* out_off,
                        uint32_t* out, uint64_t cap, uint64_t* total, unsigned long long* ctl, hipStream_t st) {
    if (n == 0) return hipMemsetAsync(total, 0, 8, st);
    const uint32_t wb = div_up(n, BLOCK / 64);
    hipLaunchKernelGGL(tm_match_small, dim3(wb < 65535 ? wb : 65535), dim3(BLOCK), 0, st, im, bytes, off, n, twords,
                       words, meta, gpath, counts, out_off, out, cap, total, ctl);
    return hipGetLastError();
}

// tm_copy_out alone, over the stage rows, counts and offsets a finished
// launch_queue left in qb (same n, K, key_words): the ids into a larger
// output after the first one overflowed, without walking again
hipError_t launch_copy(const ImageView& im, const uint8_t* bytes, const uint64_t* off, uint32_t n, const QueueBufs& qb,
                       uint32_t K, uint32_t key_words, const uint32_t* counts, const uint64_t* out_off, uint32_t* out,
                       uint64_t* out_keys, uint64_t out_cap, hipStream_t st) {
    if (n == 0 || out_cap == 0) return hipSuccess;
    dim3 blk(BLOCK), g(div_up(n, BLOCK));
    if (qb.perm) {   // a presorted walk: stage row p is topic perm[p]
        if (qb.kstage)
            hipLaunchKernelGGL(tm_copy_out_sorted<true>, g, blk, 0, st, im, off, n, qb.twords, qb.words, qb.meta,
                               qb.path, qb.stage, qb.kstage, K, key_words, counts, out_off, out, out_keys, out_cap,
                               qb.perm);
        else
            hipLaunchKernelGGL(tm_copy_out_sorted<false>, g, blk, 0, st, im, off, n, qb.twords, qb.words, qb.meta,
                               qb.path, qb.stage, nullptr, K, 1u, counts, out_off, out, nullptr, out_cap, qb.perm);
    } else if (qb.kstage) {
        hipLaunchKernelGGL((tm_copy_out<true, false>), g, blk, 0, st, im, off, n, qb.twords, qb.words, qb.meta,
                           qb.path, qb.stage, qb.kstage, K, key_words, counts, out_off, out, out_keys, out_cap,
                           nullptr, nullptr);
    } else if (qb.shaped) {
        if (!out_keys || key_words != 1 || !im.fshape) return hipErrorInvalidValue;
        hipLaunchKernelGGL((tm_copy_out<false, true>), g, blk, 0, st, im, off, n, qb.twords, qb.words, qb.meta,
                           qb.path, qb.stage, nullptr, K, 1u, counts, out_off, out, out_keys, out_cap,
                           qb.spill_chunks >= QRANGES ? qb.spill : nullptr, qb.spill_head);
    } else {
        hipLaunchKernelGGL((tm_copy_out<false, false>), g, blk, 0, st, im, off, n, qb.twords, qb.words, qb.meta,
                           qb.path, qb.stage, nullptr, K, 1u, counts, out_off, out, nullptr, out_cap,
                           qb.spill_chunks >= QRANGES ? qb.spill : nullptr, qb.spill_head);
    }
    return hipGetLastError();
}

hipError_t launch_queue(bool stats_mode, bool xcdq, const ImageView& im, const uint8_t* bytes, const uint64_t* off,
                        uint32_t n, const QueueBufs& qb, uint32_t K, uint32_t* counts, uint64_t* out_off,
                        uint32_t* out, uint64_t* out_keys, uint64_t out_cap, uint64_t* total,
                        unsigned long long* stats, hipStream_t st, hipEvent_t* marks, uint32_t walk_blocks_per_cu,
                        bool hist, uint32_t key_words) {
    auto mark = [&](int i) {
        if (marks) (void)hipEventRecord(marks[i], st);
    };
    if (n == 0) {
        hipError_t err = hipMemsetAsync(out_off, 0, sizeof(uint64_t), st);
        if (err == hipSuccess) err = hipMemsetAsync(total, 0, sizeof(uint64_t), st);
        for (int i = 0; i < 8; ++i) mark(i);
        return err;
    }
    if (K == 0 || (K & 3u) || key_words == 0) return hipErrorInvalidValue;
    hipError_t err = hipMemsetAsync(qb.ws, 0, QWS_BYTES, st);
    if (err != hipSuccess) return err;
    dim3 blk(BLOCK), g(div_up(n, BLOCK));
    const bool keys = qb.kstage != nullptr;
    // chunk rows (option "chunk_rows"): the walk of an unkeyed batch in
    // arrival order stages each chunk's rows in LDS
    const bool lane_walk = !(qb.wave_walk && !keys && !stats_mode && !qb.perm);
    const int ch = (lane_walk && !keys && !stats_mode && qb.chunk_rows) ? CH_ROWS : CH_NONE;
    const bool by_pos = queue_rows_by_position(qb, stats_mode);   // presorted without chunk rows
    mark(0);
    // presort keys / values where launch_presort's first pass reads them (an
    // odd number of passes starts from the second halves, so it ends in perm)
    const bool odd = (qb.presort_passes() & 1u) != 0;
    hipLaunchKernelGGL(tm_tokenize, g, blk, 0, st, im, bytes, off, n, qb.twords, qb.words, qb.meta,
                       qb.perm ? qb.sort_keys + (odd ? n : 0u) : nullptr,
                       qb.perm ? (odd ? qb.sort_vals : qb.perm) : nullptr,
                       qb.presort_mode | (8u * qb.presort_passes()) << 8 | (qb.light_max & 255u) << 16 |
                           (qb.tok_wave ? TOK_WAVE : 0u),
                       qb.ws + QWS_CHIST);
    if (qb.perm) {   // option "presort": perm (and the rows in walk order unless chunk rows read them by perm)
        err = launch_presort(qb.twords, qb.meta, n, qb, st, by_pos);
        if (err != hipSuccess) return err;
    }
    mark(1);
    mark(2);
    if (!lane_walk) {
        // small batch: the wave-per-topic walk (latency); lists past K have
        // spill_head = NO_SPILL, so the copy-out re-walks their heads
        const uint32_t wb = div_up(n, BLOCK / 64);
        hipLaunchKernelGGL(tm_walk_wave, dim3(wb < 65535 ? wb : 65535), blk, 0, st, im, off, n, qb.twords, qb.words,
                           qb.meta, qb.path, qb.stage, K, counts, qb.spill_chunks >= QRANGES ? qb.spill_head : nullptr,
                           qb.ws);
        mark(3);
        mark(4);
        err = launch_scan(counts, n, out_off, total, qb.scan_tmp, st);
        if (err != hipSuccess) return err;
        mark(5);
        mark(6);
        if (out_cap) {
            err = launch_copy(im, bytes, off, n, qb, K, key_words, counts, out_off, out, out_keys, out_cap, st);
            if (err != hipSuccess) return err;
        }
        mark(7);
        return hipGetLastError();
    }
    // spill chunks: unkeyed walks in arrival order (presorted rows re-walk)
    uint32_t* const spill = (!keys && !by_pos && qb.spill_chunks >= QRANGES) ? qb.spill : nullptr;
    const uint32_t wg = ch == CH_ROWS ? resident_grid(tm_walk_queue<false, true, false, CH_ROWS>, div_up(n, 64),
                                                      walk_blocks_per_cu)
                                      : resident_grid(tm_walk_queue<false, false, false>, div_up(n, 64),
                                                      walk_blocks_per_cu);
#define TM_Q(S, X, Y, C)                                                                                           \
    hipLaunchKernelGGL((tm_walk_queue<S, X, Y, C>), dim3(wg), blk, 0, st, im, off, n, qb.twords, qb.words,       \
                       qb.meta, qb.path, qb.stage, qb.kstage, K, key_words, counts, qb.ws, stats,                \
                       hist ? stats + HIST_OFF : nullptr, qb.perm, qb.twords_s, qb.meta_s, spill, qb.spill_head,   \
                       qb.spill_chunks)
    if (ch == CH_ROWS) {
        if (xcdq) TM_Q(false, true, false, CH_ROWS); else TM_Q(false, false, false, CH_ROWS);
    } else if (keys) {
        if (stats_mode) TM_Q(true, true, true, CH_NONE); else TM_Q(false, true, true, CH_NONE);
    } else if (stats_mode) {
        if (xcdq) TM_Q(true, true, false, CH_NONE); else TM_Q(true, false, false, CH_NONE);
    } else {
        if (xcdq) TM_Q(false, true, false, CH_NONE); else TM_Q(false, false, false, CH_NONE);
    }
#undef TM_Q
    mark(3);
    mark(4);
    err = launch_scan(counts, n, out_off, total, qb.scan_tmp, st);
    if (err != hipSuccess) return err;
    mark(5);
    mark(6);
    if (out_cap) {
        QueueBufs qc = qb;
        if (!by_pos) qc.perm = nullptr;   // stage rows by topic
        err = launch_copy(im, bytes, off, n, qc, K, key_words, counts, out_off, out, out_keys, out_cap, st);
        if (err != hipSuccess) return err;
    }
    mark(7);
    return hipGetLastError();
}

bool queue_rows_by_position(const QueueBufs& qb, bool stats_mode) {
    const bool keys = qb.kstage != nullptr;
    return qb.perm != nullptr && (keys || stats_mode || !qb.chunk_rows);
}

}  // namespace tmx
