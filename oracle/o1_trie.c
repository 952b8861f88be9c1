/*
 * o1_trie.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement "O1" of the reference's subscription trie, kept faithful to
 * the reference's DATA MODEL, not just its results:
 *   - node ids are full path binaries (root is the atom `root`), built by
 *     emqx_topic:join/2 (src/emqx_topic.erl:126-134);
 *   - two keyed set tables exactly like the mnesia ram_copies / ETS tables of
 *     src/emqx_trie.erl:38-48: TRIE keyed by {trie_edge, NodeId, Word}
 *     (value: child NodeId) and TRIE_NODE keyed by NodeId
 *     (value: #trie_node{edge_count, topic}), include/emqx.hrl:93-110;
 *   - words carry Erlang term identity: the atoms '', '+', '#' are distinct
 *     from binaries (src/emqx_topic.erl:141-147).
 * Functions follow, line by line:
 *   o1_insert      emqx_trie:insert/1          src/emqx_trie.erl:62-73
 *   add_path       emqx_trie:add_path/1        src/emqx_trie.erl:104-117
 *   o1_match       emqx_trie:match/1           src/emqx_trie.erl:77-79
 *   match_node     match_node/2,3              src/emqx_trie.erl:121-136
 *   match_hash     'match_#'/2                 src/emqx_trie.erl:140-145
 *   o1_delete      emqx_trie:delete/1          src/emqx_trie.erl:88-96
 *   delete_path    delete_path/1               src/emqx_trie.erl:149-163
 *   o1_lookup      emqx_trie:lookup/1          src/emqx_trie.erl:83-84
 *   o2_topic_match emqx_topic:match/2          src/emqx_topic.erl:56-75
 * The match also counts E = the number of mnesia:read(?TRIE, ...) calls the
 * reference makes (emqx_trie.erl:132 and :141), the per-topic edge-lookup
 * count used for the roofline's algorithmic bytes.
 *
 * Pinned by the reference's own known-answer tests (test/emqx_trie_SUITE.erl,
 * test/emqx_topic_SUITE.erl, test/emqx_router_SUITE.erl,
 * test/emqx_client_SUITE.erl) transcribed as data under tests/golden/, and by
 * an independent pure-Python transcription (oracle/pytrie.py).  The Erlang
 * runtime is absent from this image, so the reference itself cannot be run.
 *
 * Also timed as the CPU baseline of bench.py ("kind": "port"), multithreaded
 * over read-only tables with pthreads.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- keys ---- */
/* A term key is a byte string: node ids are encoded 'R' (root) or
 * 'B' + u32 len + bytes; words 'E' (''), 'P' ('+'), 'H' ('#') or
 * 'B' + u32 len + bytes.  An edge key is node-key ++ word-key. */

typedef struct { uint8_t* p; size_t n, cap; } buf_t;

static void buf_reserve(buf_t* b, size_t extra) {
    if (b->n + extra <= b->cap) return;
    size_t c = b->cap ? b->cap : 256;
    while (c < b->n + extra) c *= 2;
    b->p = (uint8_t*)realloc(b->p, c);
    b->cap = c;
}
static void buf_put(buf_t* b, const void* p, size_t n) {
    buf_reserve(b, n);
    memcpy(b->p + b->n, p, n);
    b->n += n;
}
static void buf_u8(buf_t* b, uint8_t c) { buf_put(b, &c, 1); }
static void buf_u32(buf_t* b, uint32_t v) { buf_put(b, &v, 4); }

/* word term */
enum { W_BIN = 0, W_EMPTY = 1, W_PLUS = 2, W_HASH = 3 };
typedef struct { int kind; const uint8_t* p; uint32_t n; } word_t;

/* emqx_topic:word/1 (src/emqx_topic.erl:149-152) */
static word_t mkword(const uint8_t* p, uint32_t n) {
    word_t w = {W_BIN, p, n};
    if (n == 0) w.kind = W_EMPTY;
    else if (n == 1 && p[0] == '+') w.kind = W_PLUS;
    else if (n == 1 && p[0] == '#') w.kind = W_HASH;
    return w;
}

/* emqx_topic:words/1 (src/emqx_topic.erl:141-147): binary:split(T, "/", [global]) */
static uint32_t split_words(const uint8_t* t, uint32_t len, word_t** out, uint32_t* cap) {
    uint32_t k = 0, s = 0;
    for (uint32_t i = 0; i <= len; ++i) {
        if (i == len || t[i] == '/') {
            if (k == *cap) {
                *cap = *cap ? *cap * 2 : 16;
                *out = (word_t*)realloc(*out, *cap * sizeof(word_t));
            }
            (*out)[k++] = mkword(t + s, i - s);
            s = i + 1;
        }
    }
    return k;
}

/* node id: NULL ptr with is_root = root atom; else path bytes */
typedef struct { int is_root; const uint8_t* p; uint32_t n; } nid_t;

static void key_node(buf_t* k, nid_t id) {
    if (id.is_root) { buf_u8(k, 'R'); return; }
    buf_u8(k, 'B'); buf_u32(k, id.n); buf_put(k, id.p, id.n);
}
static void key_word(buf_t* k, word_t w) {
    switch (w.kind) {
        case W_EMPTY: buf_u8(k, 'E'); break;
        case W_PLUS: buf_u8(k, 'P'); break;
        case W_HASH: buf_u8(k, 'H'); break;
        default: buf_u8(k, 'B'); buf_u32(k, w.n); buf_put(k, w.p, w.n);
    }
}

/* emqx_topic:join/2 (src/emqx_topic.erl:126-134) of a topic's own words is a
 * prefix of the topic bytes (join inverts binary:split), so child node ids are
 * taken as prefixes: Node_i = Topic[0 .. len(w_0) + 1 + ... + len(w_i)). */

/* ------------------------------------------------------- ETS-like table ---- */
typedef struct {
    uint64_t h;      /* 0 empty, 1 tombstone */
    uint64_t koff;   /* key offset in arena */
    uint32_t klen;
    uint32_t a, b;   /* value words */
    uint64_t voff;   /* value bytes (child node id / topic) offset, or UINT64_MAX */
    uint32_t vlen;
    uint32_t fidx;   /* test annotation, not part of the reference model: the
                        sequence number given when `topic` was last set, so a
                        GPU engine fed the same inserts can be compared by id */
} slot_t;

typedef struct {
    slot_t* s;
    size_t cap, used, tomb;
    buf_t arena;
} table_t;

static uint64_t hbytes(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ULL;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t c; memcpy(&c, p + i, 8);
        h = (h ^ c) * 0x100000001b3ULL; h ^= h >> 31;
    }
    uint64_t c = 0; memcpy(&c, p + i, n - i);
    h = (h ^ c ^ (uint64_t)n << 56) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ULL; h ^= h >> 32;
    return h < 2 ? h + 2 : h;
}

static void tab_init(table_t* t, size_t cap) {
    size_t c = 64;
    while (c < cap) c *= 2;
    t->s = (slot_t*)calloc(c, sizeof(slot_t));
    t->cap = c; t->used = t->tomb = 0;
    memset(&t->arena, 0, sizeof(t->arena));
}
static void tab_free(table_t* t) { free(t->s); free(t->arena.p); memset(t, 0, sizeof(*t)); }

static slot_t* tab_find(const table_t* t, const uint8_t* k, uint32_t n) {
    uint64_t h = hbytes(k, n);
    size_t m = t->cap - 1;
    for (size_t i = h & m;; i = (i + 1) & m) {
        slot_t* s = &t->s[i];
        if (s->h == 0) return NULL;
        if (s->h == h && s->klen == n && memcmp(t->arena.p + s->koff, k, n) == 0) return s;
    }
}
static void tab_grow(table_t* t);
static slot_t* tab_put(table_t* t, const uint8_t* k, uint32_t n) {
    slot_t* s = tab_find(t, k, n);
    if (s) return s;
    if ((t->used + t->tomb + 1) * 10 > t->cap * 7) tab_grow(t);
    uint64_t h = hbytes(k, n);
    size_t m = t->cap - 1, i = h & m;
    while (t->s[i].h > 1) i = (i + 1) & m;
    if (t->s[i].h == 1) t->tomb--;
    s = &t->s[i];
    s->h = h; s->klen = n; s->koff = t->arena.n; s->a = s->b = 0; s->voff = UINT64_MAX; s->vlen = 0;
    buf_put(&t->arena, k, n);
    t->used++;
    return s;
}
static void tab_del(table_t* t, const uint8_t* k, uint32_t n) {
    slot_t* s = tab_find(t, k, n);
    if (!s) return;
    s->h = 1; t->used--; t->tomb++;
}
static void tab_grow(table_t* t) {
    slot_t* old = t->s;
    size_t oc = t->cap;
    size_t nc = t->used * 4 > oc ? oc * 2 : oc;   /* rehash in place if mostly tombstones */
    t->s = (slot_t*)calloc(nc, sizeof(slot_t));
    t->cap = nc; t->tomb = 0;
    size_t m = nc - 1;
    for (size_t j = 0; j < oc; ++j) {
        if (old[j].h < 2) continue;
        size_t i = old[j].h & m;
        while (t->s[i].h) i = (i + 1) & m;
        t->s[i] = old[j];
    }
    free(old);
}

/* --------------------------------------------------------------- trie ------ */
typedef struct o1 {
    table_t trie;       /* ?TRIE       {trie_edge{NodeId, Word}} -> Child */
    table_t trie_node;  /* ?TRIE_NODE  NodeId -> #trie_node{edge_count, topic} */
    /* value payloads (child ids, topics) live in this arena */
    buf_t vals;
    uint32_t next_fidx;
} o1_t;

/* scratch carried per call (per thread for match) */
typedef struct {
    buf_t k, j;
    word_t* w; uint32_t wcap;
} scratch_t;

static void scratch_free(scratch_t* s) { free(s->k.p); free(s->j.p); free(s->w); }

o1_t* o1_new(uint64_t hint) {
    o1_t* t = (o1_t*)calloc(1, sizeof(o1_t));
    tab_init(&t->trie, hint * 6);
    tab_init(&t->trie_node, hint * 6);
    return t;
}
void o1_free(o1_t* t) {
    if (!t) return;
    tab_free(&t->trie); tab_free(&t->trie_node); free(t->vals.p); free(t);
}

static slot_t* read_node(o1_t* t, scratch_t* sc, nid_t id) {
    sc->k.n = 0; key_node(&sc->k, id);
    return tab_find(&t->trie_node, sc->k.p, (uint32_t)sc->k.n);
}
/* write_trie_node/1 with topic: a = edge_count, b = topic set (topic == node id) */
static slot_t* write_node(o1_t* t, scratch_t* sc, nid_t id) {
    sc->k.n = 0; key_node(&sc->k, id);
    return tab_put(&t->trie_node, sc->k.p, (uint32_t)sc->k.n);
}

/* add_path({Node, Word, Child}) — src/emqx_trie.erl:104-117 */
static void add_path(o1_t* t, scratch_t* sc, nid_t node, word_t w, nid_t child) {
    slot_t* tn = read_node(t, sc, node);
    buf_t ek = {0};
    key_node(&ek, node); key_word(&ek, w);
    if (tn) {
        if (!tab_find(&t->trie, ek.p, (uint32_t)ek.n)) {            /* wread -> [] */
            tn->a += 1;                                            /* edge_count + 1 */
            slot_t* e = tab_put(&t->trie, ek.p, (uint32_t)ek.n);
            e->voff = t->vals.n; e->vlen = child.n; buf_put(&t->vals, child.p, child.n);
        }
    } else {
        tn = write_node(t, sc, node); tn->a = 1; tn->b = 0;        /* edge_count = 1 */
        slot_t* e = tab_put(&t->trie, ek.p, (uint32_t)ek.n);
        e->voff = t->vals.n; e->vlen = child.n; buf_put(&t->vals, child.p, child.n);
    }
    free(ek.p);
}

/* emqx_trie:insert/1 — src/emqx_trie.erl:62-73 */
void o1_insert(o1_t* t, const uint8_t* topic, uint32_t len) {
    scratch_t sc = {0};
    nid_t tid = {0, topic, len};
    slot_t* tn = read_node(t, &sc, tid);
    if (tn && tn->b) { scratch_free(&sc); return; }               /* topic = Topic -> ok */
    if (tn) { tn->b = 1; tn->fidx = t->next_fidx++; scratch_free(&sc); return; } /* set topic */
    /* lists:foreach(fun add_path/1, emqx_topic:triples(Topic)) — :117-124 */
    uint32_t nw = split_words(topic, len, &sc.w, &sc.wcap);
    nid_t parent = {1, NULL, 0};
    uint32_t plen = 0;  /* parent id = topic[0..plen) */
    for (uint32_t i = 0; i < nw; ++i) {
        /* child = join(parent, w_i): a prefix of Topic (join inverts split) */
        uint32_t clen = (i == 0) ? sc.w[0].n : plen + 1 + sc.w[i].n;
        nid_t child = {0, topic, clen};
        add_path(t, &sc, parent, sc.w[i], child);
        parent = child; plen = clen;
    }
    tn = write_node(t, &sc, tid);                                  /* last node, topic = Topic */
    tn->b = 1;                                                     /* edge_count stays as read */
    tn->fidx = t->next_fidx++;
    scratch_free(&sc);
}

/* delete_path/1 — src/emqx_trie.erl:149-163; returns 0 or -1 (mnesia:abort) */
static int delete_path(o1_t* t, scratch_t* sc, const uint8_t* topic, uint32_t nw) {
    /* triples reversed: level i = nw-1 .. 0 : {Node_i, W_i, Child_i} */
    for (int i = (int)nw - 1; i >= 0; --i) {
        uint32_t plen = 0;
        for (int j = 0; j < i; ++j) plen += sc->w[j].n + (j ? 1 : 0);
        nid_t node = {i == 0, topic, plen};
        buf_t ek = {0};
        key_node(&ek, node); key_word(&ek, sc->w[i]);
        tab_del(&t->trie, ek.p, (uint32_t)ek.n);                   /* mnesia:delete edge */
        free(ek.p);
        slot_t* tn = read_node(t, sc, node);
        if (!tn) return -1;                                        /* abort node_not_found */
        if (tn->a == 1 && !tn->b) {                                /* delete node, continue */
            sc->k.n = 0; key_node(&sc->k, node);
            tab_del(&t->trie_node, sc->k.p, (uint32_t)sc->k.n);
            continue;
        }
        tn->a -= 1;                                                /* edge_count = C-1 (or 0) */
        return 0;
    }
    return 0;
}

/* emqx_trie:delete/1 — src/emqx_trie.erl:88-96 */
int o1_delete(o1_t* t, const uint8_t* topic, uint32_t len) {
    scratch_t sc = {0};
    nid_t tid = {0, topic, len};
    slot_t* tn = read_node(t, &sc, tid);
    int rc = 0;
    if (tn && tn->a == 0) {
        sc.k.n = 0; key_node(&sc.k, tid);
        tab_del(&t->trie_node, sc.k.p, (uint32_t)sc.k.n);
        uint32_t nw = split_words(topic, len, &sc.w, &sc.wcap);
        rc = delete_path(t, &sc, topic, nw);
    } else if (tn) {
        tn->b = 0;                                                 /* topic = undefined */
    }
    scratch_free(&sc);
    return rc;
}

/* emqx_trie:lookup/1 — src/emqx_trie.erl:83-84.  1 found (fills), 0 [] */
int o1_lookup(o1_t* t, const uint8_t* id, uint32_t len, uint32_t* edge_count, int* has_topic) {
    scratch_t sc = {0};
    nid_t nid = {0, id, len};
    slot_t* tn = read_node(t, &sc, nid);
    int found = tn != NULL;
    if (tn) { *edge_count = tn->a; *has_topic = (int)tn->b; }
    scratch_free(&sc);
    return found;
}

/* ------------------------------------------------------------- match ------- */
typedef struct {
    /* discovery-order results (node ids with topic set); output = reversed */
    uint64_t* off; uint32_t* len; uint32_t* fidx; size_t n, cap;
    uint64_t edge_reads;
} acc_t;

static void acc_push(acc_t* a, uint64_t off, uint32_t len, uint32_t fidx) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 64;
        a->off = (uint64_t*)realloc(a->off, a->cap * 8);
        a->len = (uint32_t*)realloc(a->len, a->cap * 4);
        a->fidx = (uint32_t*)realloc(a->fidx, a->cap * 4);
    }
    a->off[a->n] = off; a->len[a->n] = len; a->fidx[a->n] = fidx; a->n++;
}

/* the trie_node key arena stores 'B' + u32 len + bytes; topic bytes = node id */
static void push_node_if_topic(const o1_t* t, const slot_t* tn, acc_t* acc) {
    (void)t;
    if (tn && tn->b) acc_push(acc, tn->koff + 5, tn->klen - 5, tn->fidx);
}

/* edge read: mnesia:read(?TRIE, #trie_edge{node_id, word}) -> child id slot */
static const slot_t* read_edge(const o1_t* t, scratch_t* sc, nid_t node, word_t w, acc_t* acc) {
    acc->edge_reads++;
    sc->k.n = 0; key_node(&sc->k, node); key_word(&sc->k, w);
    return tab_find(&t->trie, sc->k.p, (uint32_t)sc->k.n);
}

/* 'match_#'/2 — src/emqx_trie.erl:140-145 */
static void match_hash(const o1_t* t, scratch_t* sc, nid_t node, acc_t* acc) {
    word_t h = {W_HASH, NULL, 0};
    const slot_t* e = read_edge(t, sc, node, h, acc);
    if (e) {
        nid_t child = {0, t->vals.p + e->voff, e->vlen};
        sc->k.n = 0; key_node(&sc->k, child);
        push_node_if_topic(t, tab_find(&t->trie_node, sc->k.p, (uint32_t)sc->k.n), acc);
    }
}

/* match_node/3 — src/emqx_trie.erl:127-136 (ids of children are copied out
 * of the value arena because the scratch key buffer is reused) */
static void match_node(const o1_t* t, scratch_t* sc, nid_t node, const word_t* ws, uint32_t nw, acc_t* acc) {
    if (nw == 0) {
        /* mnesia:read(?TRIE_NODE, NodeId) ++ 'match_#'(NodeId, ResAcc) */
        match_hash(t, sc, node, acc);
        sc->k.n = 0; key_node(&sc->k, node);
        push_node_if_topic(t, tab_find(&t->trie_node, sc->k.p, (uint32_t)sc->k.n), acc);
        return;
    }
    match_hash(t, sc, node, acc);                                /* 'match_#'(NodeId, ResAcc) */
    word_t plus = {W_PLUS, NULL, 0};
    word_t fold[2] = {ws[0], plus};                              /* lists:foldl over [W, '+'] */
    for (int k = 0; k < 2; ++k) {
        const slot_t* e = read_edge(t, sc, node, fold[k], acc);
        if (e) {
            nid_t child = {0, t->vals.p + e->voff, e->vlen};
            match_node(t, sc, child, ws + 1, nw - 1, acc);
        }
    }
}

/* emqx_trie:match/1 — src/emqx_trie.erl:77-79 with match_node/2 :121-125 */
static void match_one(const o1_t* t, scratch_t* sc, const uint8_t* topic, uint32_t len, acc_t* acc) {
    uint32_t nw = split_words(topic, len, &sc->w, &sc->wcap);
    acc->n = 0;
    acc->edge_reads = 0;
    if (sc->w[0].kind == W_BIN && sc->w[0].n > 0 && sc->w[0].p[0] == '$') {
        /* match_node(root, [NodeId = <<$$, _/binary>>|Words]) -> match_node(NodeId, Words, []) */
        nid_t id = {0, sc->w[0].p, sc->w[0].n};
        match_node(t, sc, id, sc->w + 1, nw - 1, acc);
    } else {
        nid_t root = {1, NULL, 0};
        match_node(t, sc, root, sc->w, nw, acc);
    }
}

/* Single topic: writes up to cap result (offset,len) pairs referencing
 * o1_topic_bytes(); returns the match count (reference order). */
typedef struct { const o1_t* t; scratch_t sc; acc_t acc; } o1_cursor_t;

o1_cursor_t* o1_cursor_new(const o1_t* t) {
    o1_cursor_t* c = (o1_cursor_t*)calloc(1, sizeof(o1_cursor_t));
    c->t = t;
    return c;
}
void o1_cursor_free(o1_cursor_t* c) {
    if (!c) return;
    scratch_free(&c->sc); free(c->acc.off); free(c->acc.len); free(c->acc.fidx); free(c);
}
/* returns M; result i (0-based, reference order) is at o1_cursor_result */
uint32_t o1_match(o1_cursor_t* c, const uint8_t* topic, uint32_t len, uint64_t* edge_reads) {
    match_one(c->t, &c->sc, topic, len, &c->acc);
    if (edge_reads) *edge_reads = c->acc.edge_reads;
    return (uint32_t)c->acc.n;
}
const uint8_t* o1_cursor_result(const o1_cursor_t* c, uint32_t i, uint32_t* len) {
    size_t k = c->acc.n - 1 - i;  /* prepend order -> reversed */
    *len = c->acc.len[k];
    return c->t->trie_node.arena.p + c->acc.off[k];
}

/* ---------------------------------------------------- batch (threaded) ----- */
typedef struct {
    const o1_t* t;
    const uint8_t* bytes; const uint64_t* off;
    uint32_t lo, hi;
    uint32_t* counts;       /* may be NULL */
    uint64_t* edge_reads;   /* may be NULL */
    uint64_t matches, e_total, levels;
} job_t;

static void* job_run(void* arg) {
    job_t* j = (job_t*)arg;
    o1_cursor_t* c = o1_cursor_new(j->t);
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        uint64_t e = 0;
        uint32_t m = o1_match(c, j->bytes + j->off[i], (uint32_t)(j->off[i + 1] - j->off[i]), &e);
        if (j->counts) j->counts[i] = m;
        if (j->edge_reads) j->edge_reads[i] = e;
        j->matches += m; j->e_total += e;
    }
    o1_cursor_free(c);
    return NULL;
}

/* match n topics on `threads` pthreads (static contiguous partition); returns
 * wall seconds of the matching (tables are read-only during the run). */
double o1_match_batch(const o1_t* t, const uint8_t* bytes, const uint64_t* off, uint32_t n, int threads,
                      uint32_t* counts, uint64_t* edge_reads, uint64_t* total_matches, uint64_t* total_edge_reads) {
    if (threads < 1) threads = 1;
    job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int k = 0; k < threads; ++k) {
        jobs[k].t = t; jobs[k].bytes = bytes; jobs[k].off = off;
        jobs[k].lo = (uint32_t)((uint64_t)n * k / threads);
        jobs[k].hi = (uint32_t)((uint64_t)n * (k + 1) / threads);
        jobs[k].counts = counts; jobs[k].edge_reads = edge_reads;
    }
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int k = 1; k < threads; ++k) pthread_create(&th[k], NULL, job_run, &jobs[k]);
    job_run(&jobs[0]);
    for (int k = 1; k < threads; ++k) pthread_join(th[k], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    uint64_t m = 0, e = 0;
    for (int k = 0; k < threads; ++k) { m += jobs[k].matches; e += jobs[k].e_total; }
    if (total_matches) *total_matches = m;
    if (total_edge_reads) *total_edge_reads = e;
    free(jobs); free(th);
    return (double)(b.tv_sec - a.tv_sec) + (double)(b.tv_nsec - a.tv_nsec) * 1e-9;
}

/* CSR of insertion sequence numbers (reference order) for n topics, threaded.
 * Pass 1 (counts) must be run with ids == NULL to size; out_off has n+1. */
typedef struct {
    const o1_t* t; const uint8_t* bytes; const uint64_t* off;
    uint32_t lo, hi; uint32_t* counts; const uint64_t* out_off; uint32_t* ids;
} idjob_t;

static void* idjob_run(void* arg) {
    idjob_t* j = (idjob_t*)arg;
    o1_cursor_t* c = o1_cursor_new(j->t);
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        uint32_t m = o1_match(c, j->bytes + j->off[i], (uint32_t)(j->off[i + 1] - j->off[i]), NULL);
        if (j->counts) j->counts[i] = m;
        if (j->ids)
            for (uint32_t k = 0; k < m; ++k) j->ids[j->out_off[i] + k] = c->acc.fidx[c->acc.n - 1 - k];
    }
    o1_cursor_free(c);
    return NULL;
}

void o1_match_ids(const o1_t* t, const uint8_t* bytes, const uint64_t* off, uint32_t n, int threads,
                  uint32_t* counts, const uint64_t* out_off, uint32_t* ids) {
    if (threads < 1) threads = 1;
    idjob_t* jobs = (idjob_t*)calloc((size_t)threads, sizeof(idjob_t));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int k = 0; k < threads; ++k) {
        idjob_t j = {t, bytes, off, (uint32_t)((uint64_t)n * k / threads), (uint32_t)((uint64_t)n * (k + 1) / threads),
                     counts, out_off, ids};
        jobs[k] = j;
    }
    for (int k = 1; k < threads; ++k) pthread_create(&th[k], NULL, idjob_run, &jobs[k]);
    idjob_run(&jobs[0]);
    for (int k = 1; k < threads; ++k) pthread_join(th[k], NULL);
    free(jobs); free(th);
}

/* insert n filters (bulk of o1_insert) */
void o1_insert_batch(o1_t* t, const uint8_t* bytes, const uint64_t* off, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) o1_insert(t, bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
}

uint64_t o1_node_count(const o1_t* t) { return t->trie_node.used; }
uint64_t o1_edge_count(const o1_t* t) { return t->trie.used; }

/* ---------------------------------------------------------------- O2 ------ */
/* emqx_topic:match/2 — src/emqx_topic.erl:56-75 (binary/binary clause first) */
int o2_topic_match(const uint8_t* name, uint32_t nlen, const uint8_t* filt, uint32_t flen) {
    if (nlen > 0 && name[0] == '$' && flen > 0 && (filt[0] == '+' || filt[0] == '#')) return 0;
    word_t* nw = NULL; word_t* fw = NULL; uint32_t nc = 0, fc = 0;
    uint32_t nn = split_words(name, nlen, &nw, &nc);
    uint32_t fn = split_words(filt, flen, &fw, &fc);
    uint32_t i = 0, j = 0;
    int r;
    for (;;) {
        if (i == nn && j == fn) { r = 1; break; }                          /* match([], []) */
        if (i < nn && j < fn) {
            word_t a = nw[i], b = fw[j];
            int eq = a.kind == b.kind && (a.kind != W_BIN || (a.n == b.n && memcmp(a.p, b.p, a.n) == 0));
            if (eq) { ++i; ++j; continue; }                                /* [H|T1], [H|T2] */
            if (b.kind == W_PLUS) { ++i; ++j; continue; }                  /* [_|T1], ['+'|T2] */
        }
        if (j + 1 == fn && fw[j].kind == W_HASH) { r = 1; break; }          /* (_, ['#']) */
        r = 0; break;
    }
    free(nw); free(fw);
    return r;
}

/* brute force: indices of all filters matching each topic (set semantics,
 * ascending filter index); returns count, fills up to cap */
uint32_t o2_match(const uint8_t* fb, const uint64_t* fo, uint32_t nf, const uint8_t* topic, uint32_t len,
                  uint32_t* out, uint32_t cap) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < nf; ++i)
        if (o2_topic_match(topic, len, fb + fo[i], (uint32_t)(fo[i + 1] - fo[i]))) {
            if (k < cap) out[k] = i;
            ++k;
        }
    return k;
}
