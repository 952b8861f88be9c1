/*
 * workload.c — deterministic synthetic subscriptions and publish topics for
 * the configs of SURVEY.md §8(d) (bench and test input; not on the match path).
 *
 *   PRNG      xoshiro256** seeded through splitmix64
 *   words     ASCII "w<level>_<k>", k ~ Zipf(s = 1.0) over the level's vocab V_i
 *   filters   length ~ U[1, L]; each level '+' with p_plus; with p_hash the last
 *             level becomes '#'; filters without a wildcard are resampled (the
 *             trie only ever holds wildcard filters: src/emqx_router.erl:158-160);
 *             a fraction sys_frac gets first level "$SYS"; a fraction share_frac
 *             is written "$share/g<k>/<filter>" (emqx_topic:parse/2 strips it,
 *             src/emqx_topic.erl:189-197); distinct raw strings when asked
 *   topics    exactly L levels from the same vocab; sys_frac get first level "$SYS"
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define WK_MAX_LEVELS 64

typedef struct wk_params {
    uint32_t levels;
    uint32_t share_groups;
    double p_plus, p_hash;
    double sys_frac;      /* fraction of $SYS filters / topics */
    double share_frac;    /* fraction of $share/g<k>/ subscriptions */
    uint32_t vocab[WK_MAX_LEVELS];
} wk_params;

typedef struct { uint64_t s[4]; } rng_t;

static uint64_t splitmix(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t* r, uint64_t seed) {
    for (int i = 0; i < 4; ++i) r->s[i] = splitmix(&seed);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t rng_next(rng_t* r) {  /* xoshiro256** */
    uint64_t* s = r->s;
    uint64_t res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static inline double rng_u01(rng_t* r) { return (double)(rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }

/* Zipf(1.0) CDF per level */
typedef struct { double* cdf[WK_MAX_LEVELS]; uint32_t v[WK_MAX_LEVELS]; } zipf_t;

static void zipf_init(zipf_t* z, const wk_params* p) {
    for (uint32_t l = 0; l < p->levels; ++l) {
        uint32_t v = p->vocab[l] ? p->vocab[l] : 1;
        z->v[l] = v;
        z->cdf[l] = (double*)malloc(sizeof(double) * v);
        double acc = 0;
        for (uint32_t k = 0; k < v; ++k) { acc += 1.0 / (double)(k + 1); z->cdf[l][k] = acc; }
        for (uint32_t k = 0; k < v; ++k) z->cdf[l][k] /= acc;
    }
}
static void zipf_free(zipf_t* z, uint32_t levels) { for (uint32_t l = 0; l < levels; ++l) free(z->cdf[l]); }
static uint32_t zipf_draw(const zipf_t* z, uint32_t l, rng_t* r) {
    double u = rng_u01(r);
    uint32_t lo = 0, hi = z->v[l] - 1;
    while (lo < hi) { uint32_t m = (lo + hi) / 2; if (z->cdf[l][m] < u) lo = m + 1; else hi = m; }
    return lo;
}

typedef struct { uint8_t* p; uint64_t n, cap; } out_t;
static int out_put(out_t* o, const char* s, size_t n) {
    if (o->n + n > o->cap) {
        uint64_t c = o->cap ? o->cap : 1 << 20;
        while (c < o->n + n) c *= 2;
        uint8_t* q = (uint8_t*)realloc(o->p, c);
        if (!q) return -1;
        o->p = q; o->cap = c;
    }
    memcpy(o->p + o->n, s, n); o->n += n;
    return 0;
}
static size_t fmt_word(char* dst, uint32_t level, uint32_t k) {
    /* "w<level>_<k>" */
    char tmp[32]; int n = 0;
    dst[0] = 'w';
    size_t o = 1;
    uint32_t x = level;
    do { tmp[n++] = (char)('0' + x % 10); x /= 10; } while (x);
    while (n) dst[o++] = tmp[--n];
    dst[o++] = '_';
    x = k;
    do { tmp[n++] = (char)('0' + x % 10); x /= 10; } while (x);
    while (n) dst[o++] = tmp[--n];
    return o;
}

/* 64-bit hash set for distinctness */
typedef struct { uint64_t* t; uint64_t cap, used; } hset_t;
static uint64_t fnv(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ULL; }
    h ^= h >> 32; h *= 0xD6E8FEB86659FD93ULL; h ^= h >> 32;
    return h ? h : 1;
}
static int hset_add(hset_t* s, uint64_t h) {  /* 1 if newly added */
    if ((s->used + 1) * 2 > s->cap) {
        uint64_t oc = s->cap, *ot = s->t;
        s->cap = oc ? oc * 2 : 1 << 16;
        s->t = (uint64_t*)calloc(s->cap, 8);
        for (uint64_t i = 0; i < oc; ++i) if (ot[i]) {
            uint64_t j = ot[i] & (s->cap - 1);
            while (s->t[j]) j = (j + 1) & (s->cap - 1);
            s->t[j] = ot[i];
        }
        free(ot);
    }
    uint64_t j = h & (s->cap - 1);
    while (s->t[j]) { if (s->t[j] == h) return 0; j = (j + 1) & (s->cap - 1); }
    s->t[j] = h; s->used++;
    return 1;
}

/* one filter into buf; returns length */
static size_t gen_filter(const wk_params* p, const zipf_t* z, rng_t* r, char* buf) {
    for (;;) {
        size_t o = 0;
        int shared = p->share_frac > 0 && rng_u01(r) < p->share_frac;
        if (shared) {
            memcpy(buf, "$share/g", 8); o = 8;
            char tmp[16]; int n = 0;
            uint32_t g = (uint32_t)(rng_next(r) % (p->share_groups ? p->share_groups : 4));
            do { tmp[n++] = (char)('0' + g % 10); g /= 10; } while (g);
            while (n) buf[o++] = tmp[--n];
            buf[o++] = '/';
        }
        size_t body = o;
        uint32_t len = 1 + (uint32_t)(rng_next(r) % p->levels);
        int sys = p->sys_frac > 0 && rng_u01(r) < p->sys_frac;
        int hash_last = rng_u01(r) < p->p_hash;
        int wild = 0;
        for (uint32_t l = 0; l < len; ++l) {
            if (l) buf[o++] = '/';
            if (l == 0 && sys) { memcpy(buf + o, "$SYS", 4); o += 4; continue; }
            if (l + 1 == len && hash_last) { buf[o++] = '#'; wild = 1; continue; }
            if (rng_u01(r) < p->p_plus) { buf[o++] = '+'; wild = 1; continue; }
            o += fmt_word(buf + o, l, zipf_draw(z, l, r));
        }
        (void)body;
        if (wild) return o;
    }
}

static size_t gen_topic(const wk_params* p, const zipf_t* z, rng_t* r, char* buf) {
    size_t o = 0;
    int sys = p->sys_frac > 0 && rng_u01(r) < p->sys_frac;
    for (uint32_t l = 0; l < p->levels; ++l) {
        if (l) buf[o++] = '/';
        if (l == 0 && sys) { memcpy(buf + o, "$SYS", 4); o += 4; continue; }
        o += fmt_word(buf + o, l, zipf_draw(z, l, r));
    }
    return o;
}

/* kind 0 = filters, 1 = topics.  Output arrays are malloc'ed; free with wk_free.
 * Returns 0 on success, -1 on bad params / allocation failure, -2 when
 * `distinct` could not find n distinct filters (space exhausted). */
int wk_generate(const wk_params* p, int kind, uint64_t n, uint64_t seed, int distinct, uint8_t** bytes,
                uint64_t** off, uint64_t* nbytes) {
    if (!p || p->levels == 0 || p->levels > WK_MAX_LEVELS || !bytes || !off || !nbytes) return -1;
    zipf_t z; zipf_init(&z, p);
    rng_t r; rng_seed(&r, seed);
    out_t o = {0};
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    hset_t hs = {0};
    char buf[64 * 32 + 64];
    int rc = 0;
    offs[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        size_t len;
        uint64_t tries = 0;
        for (;;) {
            len = kind == 0 ? gen_filter(p, &z, &r, buf) : gen_topic(p, &z, &r, buf);
            if (!(kind == 0 && distinct)) break;
            if (hset_add(&hs, fnv((const uint8_t*)buf, len))) break;
            if (++tries > 100000) { rc = -2; break; }
        }
        if (rc) break;
        if (out_put(&o, buf, len)) { rc = -1; break; }
        offs[i + 1] = o.n;
    }
    free(hs.t);
    zipf_free(&z, p->levels);
    if (rc) { free(o.p); free(offs); return rc; }
    out_put(&o, "\0\0\0\0\0\0\0\0", 8);  /* 8 B pad for aligned device reads */
    *bytes = o.p; *off = offs; *nbytes = offs[n];
    return 0;
}

void wk_free(void* p) { free(p); }
