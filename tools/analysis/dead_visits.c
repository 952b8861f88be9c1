/* dead_visits.c — analysis tool (not product code): over a filter set and a
 * topic batch, count the NFA walk's node visits (the reference's discovery
 * order, as tm_walk_queue walks) and how many of them lead to no match
 * ("dead"), split by how the node was reached, and how many a per-node
 * subtree summary could skip before loading the node:
 *   S1  "no filter in the subtree ends at depth n and no '#' filter below at
 *        depth <= n" (depth masks of filter ends and '#' parents)
 * Input: raw files of (u64 count, u64 offsets[count+1], bytes) for filters and
 * topics (tools/analysis/dead_visits.py writes them).  */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NONE 0xFFFFFFFFu
#define PLUS 0xFFFFFFFEu
#define HASH 0xFFFFFFFDu
typedef struct { uint64_t h; uint32_t id, len; uint64_t off; } ws_t;
typedef struct { uint32_t p, w, c, pad; } es_t;
static ws_t* dict; static uint64_t dmask, dused; static uint8_t* arena; static uint64_t alen, acap;
static es_t* edges; static uint64_t emask, eused;
static uint32_t *selff, nodes, ncap; static uint64_t *endm, *hashm; static uint8_t* depth;
static uint64_t mix(uint64_t k) { k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33; return k; }
static uint64_t hb(const uint8_t* p, uint32_t n) { uint64_t h = 1469598103934665603ULL ^ n; for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ULL; return mix(h) | 1; }
static uint32_t wfind(const uint8_t* p, uint32_t n, uint64_t h) {
    for (uint64_t s = h & dmask;; s = (s + 1) & dmask) { if (!dict[s].h) return NONE; if (dict[s].h == h && dict[s].len == n && !memcmp(arena + dict[s].off, p, n)) return dict[s].id; }
}
static uint32_t wid(const uint8_t* p, uint32_t n, int intern) {
    if (n == 1 && p[0] == '+') return PLUS; if (n == 1 && p[0] == '#') return HASH;
    uint64_t h = hb(p, n); uint32_t id = wfind(p, n, h); if (id != NONE || !intern) return id;
    if (alen + n > acap) { acap = (alen + n) * 2 + 4096; arena = realloc(arena, acap); }
    memcpy(arena + alen, p, n); id = (uint32_t)dused++;
    uint64_t s = h & dmask; while (dict[s].h) s = (s + 1) & dmask;
    dict[s].h = h; dict[s].id = id; dict[s].len = n; dict[s].off = alen; alen += n; return id;
}
static uint32_t efind(uint32_t p, uint32_t w) {
    for (uint64_t s = mix(((uint64_t)p << 32) | w) & emask;; s = (s + 1) & emask) { if (edges[s].p == NONE) return NONE; if (edges[s].p == p && edges[s].w == w) return edges[s].c; }
}
static void eput(uint32_t p, uint32_t w, uint32_t c) {
    uint64_t s = mix(((uint64_t)p << 32) | w) & emask; while (edges[s].p != NONE) s = (s + 1) & emask;
    edges[s].p = p; edges[s].w = w; edges[s].c = c; ++eused;
}
static uint32_t* par; static uint32_t* pword;
static void insert(const uint8_t* f, uint32_t len, uint32_t fid) {
    uint32_t v = 0, s = 0, d = 0;
    for (uint32_t i = 0; i <= len; ++i) {
        if (i < len && f[i] != '/') continue;
        uint32_t w = wid(f + s, i - s, 1), c = efind(v, w);
        if (c == NONE) { c = nodes++; selff[c] = NONE; endm[c] = hashm[c] = 0; depth[c] = (uint8_t)(d + 1); par[c] = v; pword[c] = w; eput(v, w, c); }
        v = c; s = i + 1; ++d;
    }
    if (selff[v] == NONE) selff[v] = fid;
}
/* walk statistics */
static uint64_t visits[2][2], pr1[2];   /* [reached by '+'?][dead?]; pruned by S1 */
static uint64_t matches;
static uint32_t W[256]; static uint32_t NW;
static uint64_t walk(uint32_t v, uint32_t r, int plus) {
    /* S1 check, as the parent would do before loading v (r = v's depth) */
    const uint32_t n = NW;
    int s1_dead = !((endm[v] >> n) & 1) && !(hashm[v] & ((n >= 63) ? ~0ull : ((2ull << n) - 1)));
    uint64_t m = 0;
    uint32_t h = efind(v, HASH);
    if (h != NONE && selff[h] != NONE) ++m;
    if (r == n) { if (selff[v] != NONE) ++m; }
    else {
        uint32_t w = W[r];
        if (w != NONE) { uint32_t c = efind(v, w); if (c != NONE) m += walk(c, r + 1, 0); }
        uint32_t p = efind(v, PLUS); if (p != NONE) m += walk(p, r + 1, 1);
    }
    visits[plus][m == 0]++;
    if (s1_dead) { pr1[plus]++; if (m) { fprintf(stderr, "S1 pruned a live node!\n"); exit(2); } }
    return m;
}
static uint8_t* readf(const char* fn, uint64_t* cnt, uint64_t** off) {
    FILE* f = fopen(fn, "rb"); if (!f) { perror(fn); exit(1); }
    fread(cnt, 8, 1, f); *off = malloc((*cnt + 1) * 8); fread(*off, 8, *cnt + 1, f);
    uint8_t* b = malloc((*off)[*cnt] + 8); fread(b, 1, (*off)[*cnt], f); fclose(f); return b;
}
int main(int argc, char** argv) {
    uint64_t nf, nt, *fo, *to; uint8_t* fb = readf(argv[1], &nf, &fo); uint8_t* tb = readf(argv[2], &nt, &to);
    uint64_t dc = 1 << 20; dict = calloc(dc, sizeof(ws_t)); dmask = dc - 1;
    uint64_t ec = 1; while (ec < nf * 8) ec <<= 1; edges = malloc(ec * sizeof(es_t)); memset(edges, 0xFF, ec * sizeof(es_t)); emask = ec - 1;
    ncap = (uint32_t)(nf * 4 + 16); selff = malloc(ncap * 4); endm = calloc(ncap, 8); hashm = calloc(ncap, 8); depth = calloc(ncap, 1);
    par = malloc(ncap * 4); pword = malloc(ncap * 4);
    selff[0] = NONE; nodes = 1; par[0] = NONE;
    for (uint64_t i = 0; i < nf; ++i) insert(fb + fo[i], (uint32_t)(fo[i + 1] - fo[i]), (uint32_t)i);
    /* subtree masks: children have larger ids than parents (created later) */
    for (int64_t v = nodes - 1; v >= 1; --v) {
        if (selff[v] != NONE) { if (pword[v] == HASH) hashm[par[v]] |= 1ull << (depth[v] - 1 < 63 ? depth[v] - 1 : 63); else endm[v] |= 1ull << (depth[v] < 63 ? depth[v] : 63); }
        endm[par[v]] |= endm[v]; hashm[par[v]] |= hashm[v];
    }
    for (uint64_t t = 0; t < nt; ++t) {
        const uint8_t* p = tb + to[t]; uint32_t len = (uint32_t)(to[t + 1] - to[t]); NW = 0; uint32_t s = 0;
        for (uint32_t i = 0; i <= len; ++i) { if (i < len && p[i] != '/') continue; W[NW++] = wid(p + s, i - s, 0); s = i + 1; }
        if (len && p[0] == '$') { uint32_t c = W[0] == NONE ? NONE : efind(0, W[0]); if (c != NONE) matches += walk(c, 1, 0); }
        else matches += walk(0, 0, 0);
    }
    double T = (double)nt;
    printf("{\"topics\": %llu, \"nodes\": %u, \"matches_per_topic\": %.2f, "
           "\"visits_per_topic\": %.2f, \"dead_literal\": %.2f, \"live_literal\": %.2f, \"dead_plus\": %.2f, \"live_plus\": %.2f, "
           "\"s1_prunable_literal\": %.2f, \"s1_prunable_plus\": %.2f}\n",
           (unsigned long long)nt, nodes, matches / T, (visits[0][0] + visits[0][1] + visits[1][0] + visits[1][1]) / T,
           visits[0][1] / T, visits[0][0] / T, visits[1][1] / T, visits[1][0] / T, pr1[0] / T, pr1[1] / T);
    return 0;
}
