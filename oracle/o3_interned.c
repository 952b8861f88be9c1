/*
 * o3_interned.c — TEST / MEASUREMENT INFRASTRUCTURE ONLY: the "optimized C++
 * variant (interned ids)" leg of the CPU baseline.  It is
 * never linked into libtopicmatch and never a fallback of the product path;
 * bench.py times it on the host beside O1, and tests check it against O1.
 *
 * Same algorithm as emqx_trie:match/1 (src/emqx_trie.erl:77-79, 121-145) and
 * O1, but with the data model a tuned CPU implementation would use instead of
 * the reference's ETS keys {trie_edge, NodeIdBinary, Word}: words interned to
 * u32 ids once per topic, nodes as dense u32 ids, and one open-addressing
 * table of 16 B edges keyed by (parent, word) — so every probe is two
 * integer compares instead of hashing a full-path binary.  Discovery order is
 * the reference's DFS ('match_#', then the word's subtree, then '+''s; at
 * the last level 'match_#' then the node's own filter); the output is its
 * reverse, as the reference prepends each discovery.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define O3_NONE 0xFFFFFFFFu
#define O3_PLUS 0xFFFFFFFEu
#define O3_HASH 0xFFFFFFFDu

typedef struct { uint64_t h; uint32_t id, len; uint64_t off; } wslot_t;   /* word dictionary */
typedef struct { uint32_t parent, word, child, pad; } eslot_t;              /* edge table      */

typedef struct o3 {
    wslot_t* dict; uint64_t dmask, dused;
    uint8_t* arena; uint64_t alen, acap;
    eslot_t* edges; uint64_t emask, eused;
    uint32_t* self_filter; uint32_t nodes, ncap;   /* filter index ending at node, O3_NONE */
    uint32_t filters;
} o3_t;

static uint64_t mix(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}
static uint64_t hbytes(const uint8_t* p, uint32_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ULL ^ n;
    for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ULL;
    return mix(h) | 1;
}

o3_t* o3_new(uint64_t hint) {
    o3_t* t = (o3_t*)calloc(1, sizeof(o3_t));
    uint64_t ec = 1024, dc = 1024;
    while (ec < hint * 6) ec <<= 1;
    t->edges = (eslot_t*)malloc(ec * sizeof(eslot_t));
    memset(t->edges, 0xFF, ec * sizeof(eslot_t));
    t->emask = ec - 1;
    t->dict = (wslot_t*)calloc(dc, sizeof(wslot_t));
    t->dmask = dc - 1;
    t->ncap = 1024;
    t->self_filter = (uint32_t*)malloc(t->ncap * 4);
    t->self_filter[0] = O3_NONE;
    t->nodes = 1;   /* root */
    return t;
}

void o3_free(o3_t* t) {
    if (!t) return;
    free(t->dict); free(t->arena); free(t->edges); free(t->self_filter); free(t);
}

static uint32_t word_find(const o3_t* t, const uint8_t* p, uint32_t n, uint64_t h) {
    for (uint64_t s = h & t->dmask;; s = (s + 1) & t->dmask) {
        const wslot_t* w = &t->dict[s];
        if (!w->h) return O3_NONE;
        if (w->h == h && w->len == n && memcmp(t->arena + w->off, p, n) == 0) return w->id;
    }
}
static uint32_t word_intern(o3_t* t, const uint8_t* p, uint32_t n) {
    if (n == 1 && p[0] == '+') return O3_PLUS;
    if (n == 1 && p[0] == '#') return O3_HASH;
    const uint64_t h = hbytes(p, n);
    uint32_t id = word_find(t, p, n, h);
    if (id != O3_NONE) return id;
    if ((t->dused + 1) * 2 > t->dmask + 1) {   /* grow the dictionary */
        uint64_t oc = t->dmask + 1, nc = oc * 2;
        wslot_t* old = t->dict;
        t->dict = (wslot_t*)calloc(nc, sizeof(wslot_t));
        t->dmask = nc - 1;
        for (uint64_t i = 0; i < oc; ++i)
            if (old[i].h) {
                uint64_t s = old[i].h & t->dmask;
                while (t->dict[s].h) s = (s + 1) & t->dmask;
                t->dict[s] = old[i];
            }
        free(old);
    }
    if (t->alen + n > t->acap) {
        t->acap = (t->alen + n) * 2 + 4096;
        t->arena = (uint8_t*)realloc(t->arena, t->acap);
    }
    memcpy(t->arena + t->alen, p, n);
    id = (uint32_t)t->dused++;
    uint64_t s = h & t->dmask;
    while (t->dict[s].h) s = (s + 1) & t->dmask;
    wslot_t w = {h, id, n, t->alen};
    t->dict[s] = w;
    t->alen += n;
    return id;
}

static uint32_t edge_find(const o3_t* t, uint32_t parent, uint32_t word) {
    for (uint64_t s = mix(((uint64_t)parent << 32) | word) & t->emask;; s = (s + 1) & t->emask) {
        const eslot_t* e = &t->edges[s];
        if (e->parent == O3_NONE) return O3_NONE;
        if (e->parent == parent && e->word == word) return e->child;
    }
}
static void edge_put(o3_t* t, uint32_t parent, uint32_t word, uint32_t child) {
    if ((t->eused + 1) * 2 > t->emask + 1) {
        uint64_t oc = t->emask + 1, nc = oc * 2;
        eslot_t* old = t->edges;
        t->edges = (eslot_t*)malloc(nc * sizeof(eslot_t));
        memset(t->edges, 0xFF, nc * sizeof(eslot_t));
        t->emask = nc - 1;
        for (uint64_t i = 0; i < oc; ++i)
            if (old[i].parent != O3_NONE) {
                uint64_t s = mix(((uint64_t)old[i].parent << 32) | old[i].word) & t->emask;
                while (t->edges[s].parent != O3_NONE) s = (s + 1) & t->emask;
                t->edges[s] = old[i];
            }
        free(old);
    }
    uint64_t s = mix(((uint64_t)parent << 32) | word) & t->emask;
    while (t->edges[s].parent != O3_NONE) s = (s + 1) & t->emask;
    eslot_t e = {parent, word, child, 0};
    t->edges[s] = e;
    t->eused++;
}

/* emqx_trie:insert/1 (src/emqx_trie.erl:62-73); filters get indices in first-insertion order */
void o3_insert(o3_t* t, const uint8_t* f, uint32_t len) {
    uint32_t v = 0, s = 0;
    for (uint32_t i = 0; i <= len; ++i) {
        if (i < len && f[i] != '/') continue;
        const uint32_t w = word_intern(t, f + s, i - s);
        uint32_t c = edge_find(t, v, w);
        if (c == O3_NONE) {
            if (t->nodes == t->ncap) {
                t->ncap *= 2;
                t->self_filter = (uint32_t*)realloc(t->self_filter, (size_t)t->ncap * 4);
            }
            c = t->nodes++;
            t->self_filter[c] = O3_NONE;
            edge_put(t, v, w, c);
        }
        v = c;
        s = i + 1;
    }
    if (t->self_filter[v] == O3_NONE) t->self_filter[v] = t->filters++;
}

void o3_insert_batch(o3_t* t, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) o3_insert(t, bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
}

typedef struct { uint32_t* ws; uint32_t wcap; uint32_t* acc; uint32_t n, cap; } o3_cur_t;

static void acc_push(o3_cur_t* c, uint32_t f) {
    if (c->n == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 256;
        c->acc = (uint32_t*)realloc(c->acc, (size_t)c->cap * 4);
    }
    c->acc[c->n++] = f;
}
/* 'match_#'/2 (src/emqx_trie.erl:140-145) */
static void match_hash(const o3_t* t, uint32_t v, o3_cur_t* c) {
    const uint32_t h = edge_find(t, v, O3_HASH);
    if (h != O3_NONE && t->self_filter[h] != O3_NONE) acc_push(c, t->self_filter[h]);
}
/* match_node/3 (src/emqx_trie.erl:127-136) */
static void match_node(const o3_t* t, uint32_t v, const uint32_t* ws, uint32_t nw, o3_cur_t* c) {
    if (nw == 0) {
        match_hash(t, v, c);
        if (t->self_filter[v] != O3_NONE) acc_push(c, t->self_filter[v]);
        return;
    }
    match_hash(t, v, c);
    const uint32_t w = ws[0];
    if (w != O3_NONE) {   /* a word no filter contains follows only '+' */
        const uint32_t x = edge_find(t, v, w);
        if (x != O3_NONE) match_node(t, x, ws + 1, nw - 1, c);
    }
    const uint32_t p = edge_find(t, v, O3_PLUS);
    if (p != O3_NONE) match_node(t, p, ws + 1, nw - 1, c);
}
/* match/1 with emqx_topic:words/1 and the '$' rule (src/emqx_trie.erl:121-122);
 * words are looked up, never interned, while matching */
static uint32_t match_one(const o3_t* t, o3_cur_t* c, const uint8_t* p, uint32_t len) {
    uint32_t nw = 0, s = 0;
    for (uint32_t i = 0; i <= len; ++i) {
        if (i < len && p[i] != '/') continue;
        if (nw == c->wcap) {
            c->wcap = c->wcap ? c->wcap * 2 : 64;
            c->ws = (uint32_t*)realloc(c->ws, (size_t)c->wcap * 4);
        }
        const uint32_t n = i - s;
        c->ws[nw++] = n == 1 && p[s] == '+' ? O3_PLUS : n == 1 && p[s] == '#' ? O3_HASH
                                                                                 : word_find(t, p + s, n, hbytes(p + s, n));
        s = i + 1;
    }
    c->n = 0;
    if (len > 0 && p[0] == '$') {
        const uint32_t x = c->ws[0] == O3_NONE ? O3_NONE : edge_find(t, 0, c->ws[0]);
        if (x != O3_NONE) match_node(t, x, c->ws + 1, nw - 1, c);
    } else {
        match_node(t, 0, c->ws, nw, c);
    }
    return c->n;
}

typedef struct {
    const o3_t* t; const uint8_t* bytes; const uint64_t* off;
    uint32_t lo, hi; uint32_t* counts; const uint64_t* out_off; uint32_t* ids; uint64_t matches;
} o3_job_t;

static void* o3_job(void* arg) {
    o3_job_t* j = (o3_job_t*)arg;
    o3_cur_t c = {0};
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        const uint32_t m = match_one(j->t, &c, j->bytes + j->off[i], (uint32_t)(j->off[i + 1] - j->off[i]));
        j->matches += m;
        if (j->counts) j->counts[i] = m;
        if (j->ids)
            for (uint32_t k = 0; k < m; ++k) j->ids[j->out_off[i] + k] = c.acc[m - 1 - k];   /* prepended */
    }
    free(c.ws);
    free(c.acc);
    return NULL;
}

/* n topics on `threads` pthreads; returns wall seconds.  counts / ids may be
 * NULL (ids need out_off, the CSR of counts). */
double o3_match_batch(const o3_t* t, const uint8_t* bytes, const uint64_t* off, uint32_t n, int threads,
                      uint32_t* counts, const uint64_t* out_off, uint32_t* ids, uint64_t* total_matches) {
    if (threads < 1) threads = 1;
    o3_job_t* jobs = (o3_job_t*)calloc((size_t)threads, sizeof(o3_job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int k = 0; k < threads; ++k) {
        o3_job_t j = {t, bytes, off, (uint32_t)((uint64_t)n * k / threads), (uint32_t)((uint64_t)n * (k + 1) / threads),
                      counts, out_off, ids, 0};
        jobs[k] = j;
    }
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int k = 1; k < threads; ++k) pthread_create(&th[k], NULL, o3_job, &jobs[k]);
    o3_job(&jobs[0]);
    for (int k = 1; k < threads; ++k) pthread_join(th[k], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    uint64_t m = 0;
    for (int k = 0; k < threads; ++k) m += jobs[k].matches;
    if (total_matches) *total_matches = m;
    free(jobs);
    free(th);
    return (double)(b.tv_sec - a.tv_sec) + (double)(b.tv_nsec - a.tv_nsec) * 1e-9;
}
