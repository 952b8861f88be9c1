/*
 * emqx_trie_nif.c — Erlang NIF binding of libtopicmatch (include/topicmatch.h):
 * the reference-side drop-in for emqx_trie:match/1 and the trie deltas.
 * Built only where OTP's erl_nif.h is available (`make nif ERL_INCLUDE=...`);
 * this image has no Erlang runtime.  The Erlang wrapper that loads it is in
 * INTEGRATION.md.
 *
 *   emqx_trie_nif:open(Device | [Device])     -> {ok, Engine} | {error, Reason}
 *                                     (a list opens one engine across those GPUs: tm_open_devices)
 *   emqx_trie_nif:insert(Engine, Filter)      -> ok          emqx_trie:insert/1  (src/emqx_trie.erl:62-73)
 *   emqx_trie_nif:delete(Engine, Filter)      -> ok          emqx_trie:delete/1  (src/emqx_trie.erl:88-96)
 *   emqx_trie_nif:lookup(Engine, NodeId)      -> [] | [{EdgeCount, Topic | undefined}]
 *                                                           emqx_trie:lookup/1  (src/emqx_trie.erl:83-84)
 *   emqx_trie_nif:commit(Engine)              -> {ok, Epoch} (transaction commit -> HBM image)
 *   emqx_trie_nif:match(Engine, Topic)        -> [Filter]    emqx_trie:match/1   (src/emqx_trie.erl:77-79)
 *   emqx_trie_nif:match_many(Engine, [Topic]) -> [[Filter]]  one GPU batch for many publishes
 *   emqx_trie_nif:match_async(Engine, Topic)  -> Ref; later {Ref, [Filter]} | {Ref, {error, R}}
 *                                                           (micro-batched: tm_batcher_*, H5)
 *   emqx_trie_nif:route_add(Engine, Topic, DestBin) -> ok   emqx_router add_route (src/emqx_router.erl:153-163)
 *   emqx_trie_nif:route_del(Engine, Topic, DestBin) -> ok   emqx_router del_route (:165-187)
 *   emqx_trie_nif:route_write(Engine, Topic, DestBin) -> ok          emqx_route write event (bag only)
 *   emqx_trie_nif:route_delete_object(Engine, Topic, DestBin) -> ok  emqx_route delete_object event
 *                                   (bag only: node-down cleanup keeps the trie, emqx_router_helper.erl:156-160)
 *   emqx_trie_nif:match_routes_async(Engine, Topic) -> Ref; later {Ref, [{To, DestBin}]}
 *                                                           emqx_router:match_routes/1 (:116-118)
 *   emqx_trie_nif:dest_target(Engine, DestBin, node | group, Key) -> ok
 *                                   declares Dest's aggre target: the node atom's text, or the Group
 *   emqx_trie_nif:match_deliveries_async(Engine, Topic) -> Ref; later {Ref, [{To, Node | Group}]}
 *                                   emqx_broker:aggre(emqx_router:match_routes(Topic))
 *                                   (src/emqx_broker.erl:152, 194-206), route/2's input
 * DestBin is term_to_binary(Dest) (node() or {Group, node()}): opaque to the
 * engine, binary_to_term'd by the Erlang wrapper.
 *
 * Conventions: bad input -> badarg; engine errors ->
 * {error, Atom}; the engine handle is a resource; GPU calls run on dirty IO
 * schedulers so a batch never blocks a normal scheduler.  The engine
 * serialises its own calls, so the NIF holds no lock of its own: a match
 * builds its reply terms while other calls proceed, under a filter id lease
 * (tm_lease_begin) so a concurrent delete + insert never re-binds an id the
 * reply still has to turn into a binary.  The module supports
 * hot code upgrade (the resource type is taken over by the new version).
 * The Erlang side is in erlang/ (emqx_trie_nif.erl, emqx_trie_gpu.erl,
 * emqx_trie_gpu_feed.erl).
 */
#include <erl_nif.h>
#include <string.h>

#include "../../include/topicmatch.h"

static ErlNifResourceType* ENGINE_RT = NULL;

typedef struct {
    tm_engine* e;
    tm_batcher* filters_b;   /* micro-batcher for match_async (emqx_trie:match/1)          */
    tm_batcher* routes_b;    /* micro-batcher for match_routes_async (match_routes/1)      */
    tm_batcher* deliv_b;     /* micro-batcher for match_deliveries_async (aggre/1)         */
} engine_res;

/* one in-flight async request: where the reply goes */
typedef struct {
    ErlNifPid pid;
    ErlNifEnv* env;      /* process-independent env holding Ref and the reply */
    ERL_NIF_TERM ref;
    engine_res* r;       /* kept alive until the reply is sent */
    ERL_NIF_TERM topic;  /* copy of the topic (route source TM_ROUTE_TOPIC) */
    int mode;            /* 0 match/1, 1 match_routes/1, 2 aggre(match_routes/1) */
} async_req;

static ERL_NIF_TERM atom(ErlNifEnv* env, const char* name) {
    ERL_NIF_TERM a;
    if (enif_make_existing_atom(env, name, &a, ERL_NIF_LATIN1)) return a;
    return enif_make_atom(env, name);
}

static ERL_NIF_TERM error_tuple(ErlNifEnv* env, int code) {
    const char* why = "device";
    switch (code) {
        case TM_EINVAL: why = "einval"; break;
        case TM_ENOSPC: why = "enospc"; break;
        case TM_ENOMEM: why = "enomem"; break;
        case TM_ERANGE: why = "erange"; break;
        default: why = "edevice"; break;
    }
    return enif_make_tuple2(env, atom(env, "error"), atom(env, why));
}

static void engine_dtor(ErlNifEnv* env, void* obj) {
    (void)env;
    engine_res* r = (engine_res*)obj;
    if (r->filters_b) tm_batcher_close(r->filters_b);
    if (r->routes_b) tm_batcher_close(r->routes_b);
    if (r->deliv_b) tm_batcher_close(r->deliv_b);
    if (r->e) tm_close(r->e);
}

static int open_rt(ErlNifEnv* env, ErlNifResourceFlags flags) {
    ErlNifResourceType* rt = enif_open_resource_type(env, NULL, "tm_engine", engine_dtor, flags, NULL);
    if (!rt) return -1;
    ENGINE_RT = rt;
    return 0;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)info;
    return open_rt(env, ERL_NIF_RT_CREATE);
}

/* hot code upgrade: the new module version takes over the resource type, so
 * engines opened by the old version stay valid */
static int upgrade(ErlNifEnv* env, void** priv, void** old_priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)old_priv;
    (void)info;
    return open_rt(env, ERL_NIF_RT_CREATE | ERL_NIF_RT_TAKEOVER);
}

static int get_engine(ErlNifEnv* env, ERL_NIF_TERM t, engine_res** out) {
    return enif_get_resource(env, t, ENGINE_RT, (void**)out) && (*out)->e != NULL;
}

static ERL_NIF_TERM nif_open(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    int32_t devs[TM_MAX_REPLICAS];
    unsigned nd = 0;
    int dev;
    if (argc != 1) return enif_make_badarg(env);
    if (enif_get_int(env, argv[0], &dev)) {
        devs[nd++] = dev;
    } else {   /* [Device]: one engine over those GPUs */
        ERL_NIF_TERM head, tail = argv[0];
        if (!enif_is_list(env, tail)) return enif_make_badarg(env);
        while (enif_get_list_cell(env, tail, &head, &tail)) {
            if (nd == TM_MAX_REPLICAS || !enif_get_int(env, head, &dev)) return enif_make_badarg(env);
            devs[nd++] = dev;
        }
    }
    tm_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.device = nd ? devs[0] : -1;
    engine_res* r = (engine_res*)enif_alloc_resource(ENGINE_RT, sizeof(engine_res));
    r->e = NULL;
    r->filters_b = r->routes_b = r->deliv_b = NULL;
    int rc = tm_open_devices(&cfg, devs, nd, &r->e);
    if (rc == TM_OK) {
        /* batches sealed at 64K topics, once a lane is free and the oldest
         * topic has waited 40 us (eager), or 200 us after their first topic;
         * 4 batches in flight per GPU (steady state at 1M / 10M publishes/s:
         * p50 150-155 / 173-183 us, p99 219-225 / 281-306 us),
         * and the callbacks (term building + enif_send, the per-topic host
         * cost) shared with 8 threads */
        tm_batcher_config bc;
        memset(&bc, 0, sizeof(bc));
        bc.lanes_per_replica = 4;
        bc.callback_threads = 8;
        bc.flags = TM_BATCHER_EAGER;
        rc = tm_batcher_open(r->e, &bc, &r->filters_b);
        bc.flags = TM_BATCHER_ROUTES | TM_BATCHER_EAGER;
        if (rc == TM_OK) rc = tm_batcher_open(r->e, &bc, &r->routes_b);
        bc.flags = TM_BATCHER_DELIVERIES | TM_BATCHER_EAGER;
        if (rc == TM_OK) rc = tm_batcher_open(r->e, &bc, &r->deliv_b);
    }
    if (rc != TM_OK) {
        enif_release_resource(r);
        return error_tuple(env, rc);
    }
    ERL_NIF_TERM term = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, atom(env, "ok"), term);
}

static ERL_NIF_TERM nif_filter_op(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[], int is_insert) {
    engine_res* r;
    ErlNifBinary b;
    if (argc != 2 || !get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b))
        return enif_make_badarg(env);
    int rc = is_insert ? tm_insert(r->e, b.data, (uint32_t)b.size) : tm_delete(r->e, b.data, (uint32_t)b.size);
    return rc == TM_OK ? atom(env, "ok") : error_tuple(env, rc);
}

static ERL_NIF_TERM nif_insert(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return nif_filter_op(env, argc, argv, 1);
}
static ERL_NIF_TERM nif_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return nif_filter_op(env, argc, argv, 0);
}

/* n filter (or dest) ids -> n binaries, copied under the engine lock in one
 * call (safe beside subscribers that grow the engine's arenas).  The caller
 * holds a lease (tm_lease_begin) from before the match that produced the
 * ids, so a deleted filter's id still names its own bytes.  Returns the
 * gather's status; out[] is only valid on TM_OK. */
static int make_binaries(ErlNifEnv* env, tm_engine* e, const uint32_t* ids, uint32_t n, int dests,
                         ERL_NIF_TERM* out) {
    uint64_t* off = (uint64_t*)enif_alloc(sizeof(uint64_t) * (n + 1));
    uint64_t cap = (uint64_t)n * 48 + 64;
    uint8_t* buf = (uint8_t*)enif_alloc(cap);
    if (!off || !buf) {
        if (off) enif_free(off);
        if (buf) enif_free(buf);
        return TM_ENOMEM;
    }
    memset(off, 0, sizeof(uint64_t) * (n + 1));
    int rc = dests ? tm_dests_gather(e, ids, n, buf, cap, off) : tm_filters_gather(e, ids, n, buf, cap, off);
    if (rc == TM_ENOSPC) {
        cap = off[n];
        enif_free(buf);
        buf = (uint8_t*)enif_alloc(cap ? cap : 1);
        rc = buf ? (dests ? tm_dests_gather(e, ids, n, buf, cap, off) : tm_filters_gather(e, ids, n, buf, cap, off))
                 : TM_ENOMEM;
    }
    for (uint32_t k = 0; rc == TM_OK && k < n; ++k) {
        const size_t len = (size_t)(off[k + 1] - off[k]);
        unsigned char* d = enif_make_new_binary(env, len, &out[k]);
        if (len) memcpy(d, buf + off[k], len);
    }
    if (buf) enif_free(buf);
    enif_free(off);
    return rc;
}

static ERL_NIF_TERM nif_lookup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary b;
    if (argc != 2 || !get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b))
        return enif_make_badarg(env);
    tm_node_info info;
    int rc = tm_lookup(r->e, b.data, (uint32_t)b.size, &info);
    ERL_NIF_TERM res;
    if (rc == TM_ENOENT) {
        res = enif_make_list(env, 0);
    } else if (rc != TM_OK) {
        res = error_tuple(env, rc);
    } else {
        /* #trie_node.topic is the node id itself when set (emqx_trie.erl:67,
         * :72): the argument binary, with no second engine call that a
         * concurrent delete could race */
        ERL_NIF_TERM topic = info.filter_id == TM_NO_FILTER ? atom(env, "undefined") : argv[1];
        /* #trie_node{node_id, edge_count, topic, flags} (include/emqx.hrl:95-100):
         * the record as its tuple, flags never set by emqx_trie (undefined) */
        res = enif_make_list1(env, enif_make_tuple5(env, atom(env, "trie_node"), argv[1],
                                                    enif_make_uint(env, info.edge_count), topic,
                                                    atom(env, "undefined")));
    }
    return res;
}

static ERL_NIF_TERM nif_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    if (argc != 1 || !get_engine(env, argv[0], &r)) return enif_make_badarg(env);
    uint64_t epoch = 0;
    int rc = tm_commit(r->e, &epoch);
    if (rc != TM_OK) return error_tuple(env, rc);
    return enif_make_tuple2(env, atom(env, "ok"), enif_make_uint64(env, epoch));
}

/* match over a list of topic binaries -> list of lists (reference order) */
static ERL_NIF_TERM match_list(ErlNifEnv* env, engine_res* r, ERL_NIF_TERM list, unsigned n, int single) {
    ErlNifBinary* bins = (ErlNifBinary*)enif_alloc(sizeof(ErlNifBinary) * (n ? n : 1));
    uint64_t* off = (uint64_t*)enif_alloc(sizeof(uint64_t) * (n + 1));
    ERL_NIF_TERM head, tail = list;
    uint64_t total_bytes = 0;
    for (unsigned i = 0; i < n; ++i) {
        if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_inspect_binary(env, head, &bins[i])) {
            enif_free(bins);
            enif_free(off);
            return enif_make_badarg(env);
        }
        total_bytes += bins[i].size;
    }
    uint8_t* buf = (uint8_t*)enif_alloc(total_bytes + 8);
    off[0] = 0;
    for (unsigned i = 0; i < n; ++i) {
        memcpy(buf + off[i], bins[i].data, bins[i].size);
        off[i + 1] = off[i] + bins[i].size;
    }
    uint32_t* counts = (uint32_t*)enif_alloc(sizeof(uint32_t) * (n ? n : 1));
    uint64_t* out_off = (uint64_t*)enif_alloc(sizeof(uint64_t) * (n + 1));
    uint32_t* ids = NULL;
    uint64_t total = 0;
    uint64_t lease = 0;
    int rc = tm_lease_begin(r->e, &lease);   /* ids keep naming their filters until the gather below */
    /* the library sizes the id array at the exact total: one walk per batch */
    if (rc == TM_OK) rc = tm_match_batch_owned(r->e, buf, off, n, counts, out_off, &ids, &total);
    ERL_NIF_TERM res;
    if (rc == TM_OK) {
        ERL_NIF_TERM* rows = (ERL_NIF_TERM*)enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
        for (unsigned i = 0; i < n && rc == TM_OK; ++i) {
            uint32_t c = counts[i];
            ERL_NIF_TERM* cells = (ERL_NIF_TERM*)enif_alloc(sizeof(ERL_NIF_TERM) * (c ? c : 1));
            rc = make_binaries(env, r->e, ids + out_off[i], c, 0, cells);
            if (rc == TM_OK) rows[i] = enif_make_list_from_array(env, cells, c);
            enif_free(cells);
        }
        res = rc != TM_OK ? error_tuple(env, rc) : single ? rows[0] : enif_make_list_from_array(env, rows, n);
        enif_free(rows);
    } else {
        res = error_tuple(env, rc);
    }
    tm_lease_end(r->e, lease);
    tm_free(ids);
    enif_free(out_off);
    enif_free(counts);
    enif_free(buf);
    enif_free(off);
    enif_free(bins);
    return res;
}

static ERL_NIF_TERM nif_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    if (argc != 2 || !get_engine(env, argv[0], &r) || !enif_is_binary(env, argv[1])) return enif_make_badarg(env);
    return match_list(env, r, enif_make_list1(env, argv[1]), 1, 1);
}

static ERL_NIF_TERM nif_match_many(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    unsigned n;
    if (argc != 2 || !get_engine(env, argv[0], &r) || !enif_get_list_length(env, argv[1], &n))
        return enif_make_badarg(env);
    return match_list(env, r, argv[1], n, 0);
}

/* ---- async (micro-batched) match: the batcher's worker thread calls back ---- */
static void async_done(void* ctx, uint64_t ticket, int status, const uint32_t* ids, const uint32_t* dests,
                       uint32_t n) {
    (void)ticket;
    async_req* q = (async_req*)ctx;
    ErlNifEnv* env = q->env;
    ERL_NIF_TERM res;
    if (status != TM_OK) {
        res = error_tuple(env, status);
    } else {
        ERL_NIF_TERM* cells = (ERL_NIF_TERM*)enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
        ERL_NIF_TERM* db = dests ? (ERL_NIF_TERM*)enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1)) : NULL;
        if (dests && q->mode == 2) {
            /* targets: a node atom, or a $share group binary */
            for (uint32_t k = 0; k < n; ++k) {
                uint32_t kind = 0, len = 0;
                const uint8_t* p = tm_target_bytes(q->r->e, dests[k], &kind, &len);
                if (kind == TM_TARGET_NODE) {
                    db[k] = enif_make_atom_len(env, (const char*)p, len);
                } else {
                    unsigned char* o = enif_make_new_binary(env, len, &db[k]);
                    if (len) memcpy(o, p, len);
                }
            }
        }
        int grc = TM_OK;
        if (dests && q->mode != 2) grc = make_binaries(env, q->r->e, dests, n, 1, db);
        /* every filter binary of the list in ONE gather under the engine lock
         * (the literal topic's own routes, TM_ROUTE_TOPIC, reuse its term);
         * the batcher holds the batch's lease until this callback returns */
        uint32_t* fids = (uint32_t*)enif_alloc(sizeof(uint32_t) * (n ? n : 1));
        ERL_NIF_TERM* fb = (ERL_NIF_TERM*)enif_alloc(sizeof(ERL_NIF_TERM) * (n ? n : 1));
        uint32_t nf = 0;
        for (uint32_t k = 0; k < n; ++k)
            if (ids[k] != TM_ROUTE_TOPIC) fids[nf++] = ids[k];
        if (grc == TM_OK && nf) grc = make_binaries(env, q->r->e, fids, nf, 0, fb);
        if (grc == TM_OK) {
            for (uint32_t k = 0, j = 0; k < n; ++k) {
                ERL_NIF_TERM to = ids[k] == TM_ROUTE_TOPIC ? q->topic : fb[j++];
                cells[k] = dests ? enif_make_tuple2(env, to, db[k]) : to;
            }
            res = enif_make_list_from_array(env, cells, n);
        } else {
            res = error_tuple(env, grc);
        }
        enif_free(fb);
        enif_free(fids);
        if (db) enif_free(db);
        enif_free(cells);
    }
    enif_send(NULL, &q->pid, env, enif_make_tuple2(env, q->ref, res));
    enif_free_env(env);
    enif_release_resource(q->r);
    enif_free(q);
}

static ERL_NIF_TERM submit_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[], int mode) {
    engine_res* r;
    ErlNifBinary b;
    if (argc != 2 || !get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &b))
        return enif_make_badarg(env);
    async_req* q = (async_req*)enif_alloc(sizeof(async_req));
    if (!q) return error_tuple(env, TM_ENOMEM);
    q->env = enif_alloc_env();
    ERL_NIF_TERM ref = enif_make_ref(env);
    q->ref = enif_make_copy(q->env, ref);
    q->topic = enif_make_copy(q->env, argv[1]);
    q->r = r;
    q->mode = mode;
    enif_self(env, &q->pid);
    enif_keep_resource(r);
    tm_batcher* bt = mode == 2 ? r->deliv_b : mode == 1 ? r->routes_b : r->filters_b;
    int rc = tm_batcher_submit(bt, b.data, (uint32_t)b.size, async_done, q, NULL);
    if (rc != TM_OK) {
        enif_release_resource(r);
        enif_free_env(q->env);
        enif_free(q);
        return error_tuple(env, rc);
    }
    return ref;   /* the caller blocks in receive {Ref, Result} */
}

static ERL_NIF_TERM nif_match_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return submit_async(env, argc, argv, 0);
}
static ERL_NIF_TERM nif_match_routes_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return submit_async(env, argc, argv, 1);
}

static ERL_NIF_TERM nif_match_deliveries_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return submit_async(env, argc, argv, 2);
}

static ERL_NIF_TERM nif_dest_target(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    engine_res* r;
    ErlNifBinary d, k;
    if (argc != 4 || !get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &d) ||
        !enif_is_atom(env, argv[2]) || !enif_inspect_binary(env, argv[3], &k))
        return enif_make_badarg(env);
    uint32_t kind;
    if (enif_is_identical(argv[2], atom(env, "node"))) kind = TM_TARGET_NODE;
    else if (enif_is_identical(argv[2], atom(env, "group"))) kind = TM_TARGET_GROUP;
    else return enif_make_badarg(env);
    int rc = tm_dest_target(r->e, d.data, (uint32_t)d.size, kind, k.data, (uint32_t)k.size, NULL);
    return rc == TM_OK ? atom(env, "ok") : error_tuple(env, rc);
}

enum { ROUTE_ADD, ROUTE_DEL, ROUTE_WRITE, ROUTE_DELETE_OBJECT };
static ERL_NIF_TERM nif_route_op(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[], int op) {
    engine_res* r;
    ErlNifBinary t, d;
    if (argc != 3 || !get_engine(env, argv[0], &r) || !enif_inspect_binary(env, argv[1], &t) ||
        !enif_inspect_binary(env, argv[2], &d))
        return enif_make_badarg(env);
    const uint32_t tl = (uint32_t)t.size, dl = (uint32_t)d.size;
    int rc = op == ROUTE_ADD     ? tm_route_add(r->e, t.data, tl, d.data, dl)
           : op == ROUTE_DEL     ? tm_route_del(r->e, t.data, tl, d.data, dl)
           : op == ROUTE_WRITE   ? tm_route_write(r->e, t.data, tl, d.data, dl)
                                 : tm_route_delete_object(r->e, t.data, tl, d.data, dl);
    return rc == TM_OK ? atom(env, "ok") : error_tuple(env, rc);
}
static ERL_NIF_TERM nif_route_add(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return nif_route_op(env, argc, argv, ROUTE_ADD);
}
static ERL_NIF_TERM nif_route_del(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return nif_route_op(env, argc, argv, ROUTE_DEL);
}
/* the emqx_route table events of the delta feed: the bag only, never the trie */
static ERL_NIF_TERM nif_route_write(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return nif_route_op(env, argc, argv, ROUTE_WRITE);
}
static ERL_NIF_TERM nif_route_delete_object(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
    return nif_route_op(env, argc, argv, ROUTE_DELETE_OBJECT);
}

/* Deltas run on dirty CPU schedulers: they take the engine lock, which a
 * commit can hold while it waits for a batch pinned on the image it is about
 * to rewrite (milliseconds), longer than a normal scheduler slice. */
static ErlNifFunc funcs[] = {
    {"open", 1, nif_open, 0},
    {"insert", 2, nif_insert, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"delete", 2, nif_delete, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"lookup", 2, nif_lookup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"commit", 1, nif_commit, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"match", 2, nif_match, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"match_many", 2, nif_match_many, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"match_async", 2, nif_match_async, 0},                 /* returns at once: normal scheduler */
    {"match_routes_async", 2, nif_match_routes_async, 0},
    {"match_deliveries_async", 2, nif_match_deliveries_async, 0},
    {"dest_target", 4, nif_dest_target, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_add", 3, nif_route_add, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_del", 3, nif_route_del, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_write", 3, nif_route_write, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_delete_object", 3, nif_route_delete_object, ERL_NIF_DIRTY_JOB_CPU_BOUND},
};

ERL_NIF_INIT(emqx_trie_nif, funcs, load, NULL, upgrade, NULL)
