/*
 * topicmatch.h — C-ABI of libtopicmatch, the MI355X topic-routing engine that sits
 * behind EMQ X's publish path (emqx_trie:match/1, emqx_topic:words/1 + match/2,
 * emqx_router:match_routes/1).
 *
 * Every entry point replaces one reference interface; the citation is the Erlang
 * function (file:line in vus520/emqx @ 3.0-rc.3) whose semantics it reproduces.
 * No torch types, no C++ types: plain pointers, sizes and int status codes.
 * No exception ever crosses this boundary.
 *
 * Ownership: input buffers are borrowed for the duration of the call only.
 * Output buffers are caller-allocated. Filter bytes returned by
 * tm_filter_bytes() stay engine-owned and valid until that filter is deleted
 * and the next tm_commit().
 *
 * Threading: every call on one engine is serialised by the engine (single
 * writer; matches read a committed snapshot).  Different engines are
 * independent.  One engine may span several GPUs (tm_open_devices).
 */
#ifndef TOPICMATCH_H
#define TOPICMATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------- */
#define TM_OK        0
#define TM_EINVAL   -1   /* bad argument (NIF: enif_make_badarg)              */
#define TM_ENOSPC   -2   /* output buffer too small; *out_needed says how big */
#define TM_EDEVICE  -3   /* no GPU / HIP error / engine opened host-only      */
#define TM_ENOMEM   -4   /* host or device allocation failed                  */
#define TM_ENOENT   -5   /* tm_lookup: no such trie node                      */
#define TM_ERANGE   -6   /* image would exceed 2^29-1 nodes / 2^32 filters       */

#define TM_NO_FILTER 0xFFFFFFFFu

typedef struct tm_engine tm_engine;

/* mnesia(boot) analogue: src/emqx_trie.erl:38-48 creates the two ram_copies
 * tables; here the engine holds the host mirror and the HBM image. */
typedef struct tm_config {
    int32_t  device;          /* HIP device ordinal; -1 = host-only engine       */
    uint32_t reserved0;
    uint64_t filters_hint;    /* expected filter count (pre-sizes tables)        */
    uint64_t batch_topics;    /* workspace hint: topics per match batch          */
    uint64_t batch_bytes;     /* workspace hint: topic bytes per match batch     */
} tm_config;

/* #trie_node{node_id, edge_count, topic} — include/emqx.hrl:100-105 */
typedef struct tm_node_info {
    uint32_t edge_count;      /* distinct child words ('+', '#' included)        */
    uint32_t filter_id;       /* TM_NO_FILTER when topic = undefined             */
} tm_node_info;

/* batch statistics of the last match (for the roofline accounting) */
typedef struct tm_batch_stats {
    uint64_t topics;          /* n                                               */
    uint64_t levels;          /* sum n_t                                         */
    uint64_t visits;          /* trie nodes visited by the NFA walk (frontier)   */
    uint64_t edge_reads;      /* E = mnesia:read(?TRIE,...) calls the reference  */
                              /*     would make (emqx_trie.erl:132,141)          */
    uint64_t matches;         /* sum M_t                                         */
    uint64_t leaf_visits;     /* visits at the topic's last level (leaf half)    */
    uint64_t probe_loads;     /* 16 B edge-table slot loads (wide nodes, '#')    */
    uint64_t prunable_visits; /* visits the subtree summaries skip (the counting */
                              /* walk of stats mode skips none, so E is exact)   */
} tm_batch_stats;

/* engine lifetime ------------------------------------------------------------ */
int  tm_open(const tm_config* cfg, tm_engine** out);
/* One engine over several GPUs of the node (SURVEY §8(e) replicated mode):
 * the host trie is kept once and committed to a replica of the HBM image on
 * each of devices[0..n) (an ordinal may repeat: two replicas on one GPU).
 * Host-buffer batches (tm_match_batch, tm_match_routes_batch,
 * tm_match_deliveries_batch, the micro-batcher) are cut into one contiguous
 * slice per replica and run on all GPUs at once, with results identical to
 * one GPU; device-buffer calls run on the replica of the GPU holding the
 * batch.  This is how one BEAM process (emqx_broker:publish/1 on every
 * scheduler, src/emqx_broker.erl:148-157) drives the whole node through one
 * NIF handle.  cfg->device is ignored; n_devices = 0 opens a host-only
 * engine. */
#define TM_MAX_REPLICAS 64u
int  tm_open_devices(const tm_config* cfg, const int32_t* devices, uint32_t n_devices, tm_engine** out);
/* number of device replicas (0: host-only) */
int  tm_engine_replicas(tm_engine* e);
/* the replicas' HIP ordinals into out[0..cap); returns their number */
int  tm_engine_devices(tm_engine* e, int32_t* out, uint32_t cap);
void tm_close(tm_engine* e);
const char* tm_strerror(int code);
const char* tm_last_error(tm_engine* e);  /* text of the last failure on e */

/* emqx_trie:insert/1 — src/emqx_trie.erl:62-73 (+ add_path/1 :104-117).
 * Idempotent. Any byte string is accepted (the reference does not validate
 * inside the trie; validation happens at emqx_topic:validate/2). */
int tm_insert(tm_engine* e, const uint8_t* filter, uint32_t len);

/* Bulk form of tm_insert over n concatenated filters ([off[i], off[i+1])),
 * the router's batch add (src/emqx_router.erl:148-163 per route). Stops at
 * the first failure and returns its code. */
int tm_insert_batch(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n);

/* Sharded mode: the shard (0..n_shards-1) that owns a filter — by a hash of
 * its prefix through the second literal (non '+'/'#') level, so every filter
 * under one such prefix lives on one shard.  Any partition is correct (a
 * match is a per-filter predicate, match(T, F) = U_s match(T, F_s)); this one
 * keeps sub-tries disjoint below the prefix and spreads Zipf-heavy root words
 * and wildcard-led subtrees over all shards. */
uint32_t tm_shard_of(const uint8_t* filter, uint32_t len, uint32_t n_shards);

/* tm_shard_of over a packed batch: out[i] = shard of filter [off[i], off[i+1]). */
int tm_shard_of_batch(const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t n_shards, uint32_t* out);

/* tm_insert_batch restricted to the filters tm_shard_of assigns to `shard`. */
int tm_insert_batch_shard(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n,
                          uint32_t n_shards, uint32_t shard);

/* emqx_trie:delete/1 — src/emqx_trie.erl:88-96 (+ delete_path/1 :149-163).
 * Unknown filter = no-op (TM_OK). */
int tm_delete(tm_engine* e, const uint8_t* filter, uint32_t len);

/* Bulk form of tm_delete over n concatenated filters (the router's batch
 * delete, src/emqx_router.erl:243-250), applied in order. */
int tm_delete_batch(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n);

/* emqx_trie:lookup/1 — src/emqx_trie.erl:83-84.  node_id is the full path
 * binary (emqx_topic:join of the words).  TM_ENOENT when the node is absent. */
int tm_lookup(tm_engine* e, const uint8_t* node_id, uint32_t len, tm_node_info* out);

/* Filter id leases.  The ids a match returns name filters of the image
 * epoch it ran on; a caller that turns them into bytes later
 * (tm_filters_gather, the NIF's reply terms) holds a lease from before the
 * match until its last gather: a deleted filter's id is not reused while a
 * lease older than the deletion's commit is open, nor before both image
 * epochs have dropped it, and tm_filters_gather keeps returning its bytes
 * until then.  (The reference hands out the filter binaries themselves:
 * emqx_trie.erl:79.)  The micro-batcher leases each batch through its
 * callbacks. */
int  tm_lease_begin(tm_engine* e, uint64_t* lease);
void tm_lease_end(tm_engine* e, uint64_t lease);

/* Publish pending deltas to the HBM image (mnesia transaction commit,
 * src/emqx_router.erl:264-268).  tm_match_* commit implicitly. */
int tm_commit(tm_engine* e, uint64_t* epoch_out);

/* HIP device ordinal of the engine (-1: host-only) */
int tm_engine_device(tm_engine* e);

/* number of filters currently in the trie (nodes with topic =/= undefined) */
uint64_t tm_filter_count(tm_engine* e);
/* trie nodes / literal edges of the image (for sizing reports) */
uint64_t tm_node_count(tm_engine* e);
uint64_t tm_image_bytes(tm_engine* e);

/* filter id -> filter bytes (the #trie_node.topic binary).  The pointer is
 * into the engine's arena: valid until the next insert / delete on e (an
 * insert may grow the arena).  Threads that match while others subscribe
 * use tm_filters_gather. */
const uint8_t* tm_filter_bytes(tm_engine* e, uint32_t filter_id, uint32_t* len);

/* Copy the bytes of n filters (ids[i]) into buf, back to back, under the
 * engine lock: filter i is buf[off[i] .. off[i+1]) (off has n+1 entries).
 * TM_ENOSPC when they exceed cap (off[n] = the bytes needed); TM_EINVAL for
 * an unknown id.  tm_dests_gather does the same for route dest ids. */
int tm_filters_gather(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, uint64_t cap, uint64_t* off);
int tm_dests_gather(tm_engine* e, const uint32_t* ids, uint32_t n, uint8_t* buf, uint64_t cap, uint64_t* off);

/* emqx_trie:match/1 over a batch — src/emqx_trie.erl:77-79, 121-145, with
 * emqx_topic:words/1 (src/emqx_topic.erl:141-147) done on the device.
 * Topics are concatenated in topic_bytes; topic t is
 * [topic_off[t], topic_off[t+1]).  Output is CSR: the match list of topic t is
 * out_filter_id[out_off[t] .. out_off[t]+out_count[t]), in exactly the order
 * emqx_trie:match/1 returns it.  out_off has n+1 entries.
 * If the total exceeds out_cap: TM_ENOSPC, *out_needed = total, counts and
 * offsets are still filled.  Host buffers; the call synchronises. */
int tm_match_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off,
                   uint32_t n, uint32_t* out_count, uint64_t* out_off,
                   uint32_t* out_filter_id, uint64_t out_cap, uint64_t* out_needed);

/* tm_match_batch with the id array allocated by the library at the exact
 * total (*out_ids, released with tm_free; *out_total = its length): one walk
 * per batch whatever the fan-out, no caller-side capacity guess or retry.
 * The NIF's synchronous match/1 and match_many/2 use this. */
int  tm_match_batch_owned(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                          uint32_t* out_count, uint64_t* out_off, uint32_t** out_ids, uint64_t* out_total);
void tm_free(void* p);

/* Same, with every buffer device-resident (HBM) and stream-ordered on
 * `hip_stream` (a hipStream_t; NULL = the engine's stream).  Does not
 * synchronise.  *d_total (device) receives the match total; ids past out_cap
 * are dropped (the caller compares *d_total with out_cap).  d_topic_off must
 * have n+1 entries and topic_bytes = d_topic_off[n] - d_topic_off[0] (sizes
 * the engine's workspace without a device read).  Calls on one engine must
 * be issued on one stream.  This is the entry a pipelined batcher and the
 * bench use. */
int tm_match_batch_device(tm_engine* e, const uint8_t* d_topic_bytes, const uint64_t* d_topic_off,
                          uint32_t n, uint64_t topic_bytes, uint32_t* d_out_count,
                          uint64_t* d_out_off, uint32_t* d_out_filter_id, uint64_t out_cap,
                          uint64_t* d_total, void* hip_stream);

/* The same lists for a small batch in ONE kernel launch (tokenize, a wave per
 * topic, each list placed with one atomic): for latency-bound batches (the
 * micro-batcher's, up to a few tens of thousands of topics), where the four
 * launches and the scan of tm_match_batch_device cost more than the walk.
 * Each topic's list is contiguous and in emqx_trie:match/1 order at
 * d_out_off[t] .. + d_out_count[t], but topics' lists are laid out in
 * completion order (d_out_off is not an exclusive scan; there is no
 * d_out_off[n]).  *d_total = ids of all lists; when it exceeds out_cap, no
 * list past the capacity was written: run again with out_cap >= *d_total.
 * Same arguments and stream semantics as tm_match_batch_device. */
int tm_match_small_device(tm_engine* e, const uint8_t* d_topic_bytes, const uint64_t* d_topic_off,
                          uint32_t n, uint64_t topic_bytes, uint32_t* d_out_count,
                          uint64_t* d_out_off, uint32_t* d_out_filter_id, uint64_t out_cap,
                          uint64_t* d_total, void* hip_stream);

/* Sharded mode (the filter set partitioned over GPUs, see
 * emqx_amd/shard.py).  Same as tm_match_batch_device on this engine's shard,
 * plus d_out_key[i]: the order key of id i (2 bits per level for the branch
 * the reference's fold took — 'match_#' 0, topic word 1, '+' 2 — and an end
 * mark 1 for a node's own filter, packed from the top of a u64).  Each
 * topic's ids come in descending key order, which is emqx_trie:match/1's
 * order (emqx_trie.erl:127-145), so shards' lists merge by key.  One key
 * word covers topics of up to 31 levels; tm_match_batch_device_keys_w below
 * takes wider keys. */
int tm_match_batch_device_keys(tm_engine* e, const uint8_t* d_topic_bytes, const uint64_t* d_topic_off,
                               uint32_t n, uint64_t topic_bytes, uint32_t* d_out_count,
                               uint64_t* d_out_off, uint32_t* d_out_filter_id, uint64_t* d_out_key,
                               uint64_t out_cap, uint64_t* d_total, void* hip_stream);

/* Keys wider than one word, for topics of 32 levels or more (MQTT levels are
 * unlimited, src/emqx_mqtt_caps.erl:110): key_words u64 words per id (1 ..
 * TM_MAX_KEY_WORDS), word j of id i at d_out_key[j * out_cap + i]; topics of
 * up to 32 * key_words - 1 levels are keyed exactly.  The caller sizes
 * key_words from its topics' level counts; tm_key_levels reports the most
 * levels a keyed batch held, so a caller can verify the width it chose.
 * tm_match_batch_device_keys is key_words = 1. */
#define TM_MAX_KEY_WORDS 1024u
int tm_match_batch_device_keys_w(tm_engine* e, const uint8_t* d_topic_bytes, const uint64_t* d_topic_off,
                                 uint32_t n, uint64_t topic_bytes, uint32_t* d_out_count, uint64_t* d_out_off,
                                 uint32_t* d_out_filter_id, uint64_t* d_out_key, uint32_t key_words,
                                 uint64_t out_cap, uint64_t* d_total, void* hip_stream);
/* most levels of any topic in the engine's in-flight / last keyed batches
 * (synchronises on them) */
int tm_key_levels(tm_engine* e, uint32_t* max_levels);

/* Merge, on e's GPU, the keyed lists of n_shards (<= 8) shards for m topics
 * (after the all-to-all exchange): d_counts [n_shards][m]; shard s's ids and
 * keys start at d_src_base[s] (device u64 array) and are CSR-ordered by
 * topic.  Output: per-topic counts, offsets[m+1] and global filter ids
 * local_id * n_shards + s, in emqx_trie:match/1 order; *d_total is exact, ids
 * past out_cap are dropped.  Stream-ordered. */
int tm_shard_merge(tm_engine* e, uint32_t n_shards, uint32_t m, const uint32_t* d_counts,
                   const uint64_t* d_src_base, const uint32_t* d_ids, const uint64_t* d_keys,
                   uint32_t* d_out_count, uint64_t* d_out_off, uint32_t* d_out_gid, uint64_t out_cap,
                   uint64_t* d_total, void* hip_stream);
/* Same with keys of key_words words: word j of item g at d_keys[j * key_stride + g]. */
int tm_shard_merge_w(tm_engine* e, uint32_t n_shards, uint32_t m, const uint32_t* d_counts,
                     const uint64_t* d_src_base, const uint32_t* d_ids, const uint64_t* d_keys, uint32_t key_words,
                     uint64_t key_stride, uint32_t* d_out_count, uint64_t* d_out_off, uint32_t* d_out_gid,
                     uint64_t out_cap, uint64_t* d_total, void* hip_stream);

/* ---- sharded-mode exchange over RCCL (exchange.cpp) ---------
 * After the keyed walks, topic slice d (topics [n*d/S, n*(d+1)/S)) of every
 * shard's lists goes to rank d (an all-to-all: each id crosses xGMI once),
 * which merges them with tm_shard_merge_w.  A tm_comm is one rank's RCCL
 * communicator: tm_comm_init_rank for one rank per process (rank 0 makes the
 * id with tm_comm_unique_id and shares it, e.g. over torch.distributed),
 * tm_comm_init_all for all ranks of one process (ranks that share a GPU,
 * which RCCL refuses, exchange by device copies instead).  Receive buffers
 * belong to the comm and stay valid until its next exchange. */
#define TM_COMM_ID_BYTES 128
typedef struct tm_comm tm_comm;
typedef struct tm_exchange_in {
    uint32_t n;                 /* topics of the batch (the same batch on every rank)      */
    uint32_t key_words;         /* order key words per id                                   */
    const uint32_t* d_counts;   /* n: this shard's list lengths                            */
    const uint64_t* d_offs;     /* n + 1: CSR offsets                                      */
    const uint32_t* d_ids;      /* local filter ids                                        */
    const uint64_t* d_keys;     /* key_words planes, key_stride apart                      */
    uint64_t key_stride;
    void* hip_stream;           /* stream the lists were produced on (NULL: the comm's)    */
} tm_exchange_in;
typedef struct tm_exchange_out {
    uint32_t m;                 /* topics of this rank's slice                             */
    uint32_t reserved;
    uint64_t total;             /* ids received                                            */
    const uint32_t* d_counts;   /* [S][m], source-major                                    */
    const uint64_t* d_src_base; /* S: where source s's ids / keys start                    */
    const uint32_t* d_ids;      /* total                                                    */
    const uint64_t* d_keys;     /* key_words planes of `total`                             */
} tm_exchange_out;
int  tm_comm_unique_id(uint8_t id[TM_COMM_ID_BYTES]);
int  tm_comm_init_rank(const uint8_t id[TM_COMM_ID_BYTES], uint32_t nranks, uint32_t rank, int device,
                       tm_comm** out);
int  tm_comm_init_all(const int32_t* devices, uint32_t n, tm_comm** comms);
void tm_comm_destroy(tm_comm* c);
int  tm_comm_uses_rccl(tm_comm* c);   /* 1: RCCL, 0: device copies */
const char* tm_comm_last_error(tm_comm* c);
/* A rank's own part of every exchange (tm_shard_exchange, tm_route_exchange,
 * tm_route_return) through RCCL too -- ncclSend / ncclRecv to itself inside
 * the group, and the size all-to-alls over RCCL at one rank -- instead of a
 * device copy.  Slower; it exists so that a one-GPU box (one rank) executes
 * the RCCL code paths the multi-GPU ranks take.  TM_EINVAL without RCCL. */
int  tm_comm_set_self_rccl(tm_comm* c, int on);
/* one rank (RCCL communicator) of a multi-process exchange; stream-ordered
 * after two small host syncs that size the sends and receives */
int  tm_shard_exchange(tm_comm* c, const tm_exchange_in* in, tm_exchange_out* out);
/* all S ranks of one process at once (comms from tm_comm_init_all) */
int  tm_shard_exchange_group(tm_comm** comms, uint32_t S, const tm_exchange_in* ins, tm_exchange_out* outs);

/* ---- routed sharded mode (SURVEY §8(e) sharded, C4: filter capacity beyond
 * one GPU with per-topic work on ONE shard; exchange.cpp, route.hip) ---------
 * Topic T is owned by shard tm_route_of(T's first `depth` levels); filter F
 * lives on the shard of its first `depth` levels when those are all literal
 * (it can match only topics that begin with them), on EVERY shard otherwise
 * (a '+' / '#' among them).  The owner shard then holds every filter that can
 * match T, and its walk alone yields emqx_trie:match/1's complete list in
 * order (src/emqx_trie.erl:121-145): the relative order of two matching
 * filters is a property of the filters, so no merge is
 * needed, only a topic exchange.  Filters keep GLOBAL ids on every shard
 * (tm_insert_batch_ids), so every rank's lists name filters alike.
 *
 * tm_route_of: the owner shard (0 .. n_shards-1) of a publish topic, or of a
 * filter (is_filter = 1; TM_ROUTE_ALL when one of its first depth levels is
 * '+' or '#').  The key is the bytes of the first min(depth, levels) levels,
 * hashed exactly as the device does it. */
#define TM_ROUTE_ALL 0xFFFFFFFFu
uint32_t tm_route_of(const uint8_t* topic, uint32_t len, uint32_t n_shards, uint32_t depth, int is_filter);

/* emqx_trie:insert/1 of n filters under caller-chosen filter ids (ids[i],
 * unique, < 2^31 - 16): a sharded or routed engine holds its part of a global
 * filter set under the global ids, so its walks emit them directly.  An engine
 * filled this way must not also take tm_insert / tm_insert_batch (their ids
 * would collide).  TM_EINVAL when ids[i] names another live filter, when the
 * filter is present under another id, or when ids[i] was deleted from another
 * filter and batches in flight may still name it (it is reusable for another
 * filter after two commits and once the leases open at the delete end; the
 * same filter may take it back at once). */
int tm_insert_batch_ids(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n, const uint32_t* ids);

/* tm_insert_batch_ids of the filters tm_route_of places on `shard` (routed to
 * it, or to every shard), filter i of the batch under global id gid_base + i.
 * A filter repeated in the batch (or already present) keeps the id of its
 * first insertion: emqx_trie:insert/1 is idempotent (src/emqx_trie.erl:62-73),
 * so a list with repeats names each filter by its first index.  (tm_insert_
 * batch_ids, whose caller states every id, refuses a filter present under
 * another id with TM_EINVAL.) */
int tm_insert_batch_routed(tm_engine* e, const uint8_t* bytes, const uint64_t* off, uint32_t n, uint32_t n_shards,
                           uint32_t shard, uint32_t depth, uint32_t gid_base);

/* Topic exchange: every rank routes its own batch (HBM, stream-ordered) and
 * sends each topic to its owner; *out receives the topics this rank owns —
 * concatenated by source rank, in each source's order — as a batch for
 * tm_match_batch_device (bytes + n+1 offsets, comm-owned, valid until the
 * comm's next route call).  One host sync sizes the receives. */
typedef struct tm_route_in {
    uint32_t n;                 /* topics of this rank's batch                              */
    uint32_t depth;             /* routing depth (levels of the key)                        */
    uint64_t bytes;             /* d_off[n] - d_off[0] (sizes the sends without a device read) */
    const uint8_t* d_bytes;     /* topic bytes (+ 8 readable bytes past the end)            */
    const uint64_t* d_off;      /* n + 1 offsets                                            */
    void* hip_stream;           /* NULL: the comm's stream                                  */
} tm_route_in;
typedef struct tm_route_out {
    uint32_t m;                 /* topics this rank owns                                    */
    uint32_t reserved;
    uint64_t bytes;             /* their bytes                                              */
    const uint8_t* d_bytes;     /* m topics back to back (+ 8 padding bytes)                */
    const uint64_t* d_off;      /* m + 1 offsets                                            */
} tm_route_out;
int tm_route_exchange(tm_comm* c, const tm_route_in* in, tm_route_out* out);
int tm_route_exchange_group(tm_comm** comms, uint32_t S, const tm_route_in* ins, tm_route_out* outs);

/* The way back: the owner's lists of its m topics (CSR from
 * tm_match_batch_device on the batch tm_route_exchange delivered) return to
 * the ranks the topics came from; *res is each rank's own batch's lists in its
 * original topic order (counts n, offsets n+1, ids total; comm-owned, valid
 * until the comm's next route call). */
typedef struct tm_route_lists {
    const uint32_t* d_counts;   /* m                                                        */
    const uint64_t* d_offs;     /* m + 1                                                    */
    const uint32_t* d_ids;
    void* hip_stream;
} tm_route_lists;
typedef struct tm_route_result {
    uint32_t n;
    uint32_t reserved;
    uint64_t total;
    const uint32_t* d_counts;   /* n                                                        */
    const uint64_t* d_offs;     /* n + 1                                                    */
    const uint32_t* d_ids;      /* total                                                    */
} tm_route_result;
int tm_route_return(tm_comm* c, const tm_route_lists* lists, tm_route_result* res);
int tm_route_return_group(tm_comm** comms, uint32_t S, const tm_route_lists* lists, tm_route_result* res);

/* ---- routes: the emqx_route bag and emqx_router:match_routes/1 -------------
 * A route is (topic, dest) (#route{topic, dest}, include/emqx.hrl:84-87); dest
 * is opaque bytes (the NIF passes term_to_binary(node() | {Group, node()})),
 * interned to a dest id.  Routes of one topic keep insertion order (ETS bag). */

/* emqx_router add_route — handle_cast({add_route, Route}) src/emqx_router.erl:153-163
 * and add_trie_route/1 :226-231: an existing route is a no-op; a wildcard
 * topic (emqx_topic:wildcard/1) enters the trie (tm_insert) when it had no
 * route yet. */
int tm_route_add(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen);

/* Bulk tm_route_add: route i = (topic [topic_off[i], topic_off[i+1]),
 * dest [dest_off[i], dest_off[i+1])), applied in order. */
int tm_route_add_batch(tm_engine* e, const uint8_t* topics, const uint64_t* topic_off, const uint8_t* dests,
                       const uint64_t* dest_off, uint32_t n);

/* emqx_router del_route — handle_cast({del_route, Route}) :165-187,
 * del_trie_route/1 :252-260, del_direct_route/1 :240-241: removes the route;
 * a wildcard topic leaves the trie (tm_delete) with its last route.  An
 * absent route is a no-op.  (The emqx_subscriber check at :179 belongs to the
 * broker and stays with the caller.) */
int tm_route_del(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen);

/* Bulk tm_route_del, laid out as tm_route_add_batch, applied in order. */
int tm_route_del_batch(tm_engine* e, const uint8_t* topics, const uint64_t* topic_off, const uint8_t* dests,
                       const uint64_t* dest_off, uint32_t n);

/* The emqx_route table events the delta feed receives
 * (mnesia:subscribe({table, emqx_route, detailed}); erlang/emqx_trie_gpu_feed.erl):
 * the route bag ONLY, never the trie, whose membership the feed drives from
 * emqx_trie_node events alone (tm_insert / tm_delete).
 *   tm_route_write          = mnesia:write(emqx_route, #route{}) — add_trie_route/1
 *                             :231, add_direct_route/1 :223-224; an existing
 *                             route is a no-op, a new one goes last in its bag.
 *   tm_route_delete_object  = mnesia:delete_object(emqx_route, #route{}) —
 *                             del_trie_route/1 :255-258, del_direct_route/1
 *                             :240-241 and the node-down cleanup
 *                             emqx_router_helper:cleanup_routes/1
 *                             (src/emqx_router_helper.erl:156-160), which deletes
 *                             routes only: a stale filter stays in the trie and
 *                             emqx_trie:match/1 keeps returning it.  Absent: no-op.
 * A wildcard topic's routes join its trie filter whenever both exist, in either
 * order of arrival (match_routes/1 finds routes through the filter). */
int tm_route_write(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen);
int tm_route_delete_object(tm_engine* e, const uint8_t* topic, uint32_t tlen, const uint8_t* dest, uint32_t dlen);
/* Bulk tm_route_write (the feed's boot snapshot), laid out as tm_route_add_batch. */
int tm_route_write_batch(tm_engine* e, const uint8_t* topics, const uint64_t* topic_off, const uint8_t* dests,
                         const uint64_t* dest_off, uint32_t n);

/* get_routes/1 — :89-90: the dest ids of topic's routes in insertion order;
 * *out_n = their number (TM_ENOSPC when it exceeds cap). */
int tm_get_routes(tm_engine* e, const uint8_t* topic, uint32_t tlen, uint32_t* out_dest, uint32_t cap,
                  uint32_t* out_n);

/* number of routes (ets:info(emqx_route, size), emqx_router_helper.erl:148-154) */
uint64_t tm_route_count(tm_engine* e);

/* dest id -> dest bytes (engine-owned; valid until the next route add on e,
 * see tm_dests_gather) */
const uint8_t* tm_dest_bytes(tm_engine* e, uint32_t dest_id, uint32_t* len);

#define TM_ROUTE_TOPIC 0xFFFFFFFFu   /* route source: the publish topic itself */

/* emqx_router:match_routes/1 — src/emqx_router.erl:116-118 — over a batch:
 * routes of topic t are out_src/out_dest[out_off[t] .. +out_count[t]): first
 * get_routes(Topic) of the literal topic (out_src = TM_ROUTE_TOPIC), then,
 * for each filter emqx_trie:match/1 returns, in its order, that filter's
 * routes (out_src = filter id).  Host buffers, synchronous; TM_ENOSPC /
 * out_needed as tm_match_batch.  Trie walk and route expansion both run on
 * the GPU (routes.hip). */
int tm_match_routes_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                          uint32_t* out_count, uint64_t* out_off, uint32_t* out_src, uint32_t* out_dest,
                          uint64_t out_cap, uint64_t* out_needed);

/* Same with device buffers on hip_stream (reads the match total once to size
 * its workspace); *d_total = route total, routes past out_cap are dropped. */
int tm_match_routes_batch_device(tm_engine* e, const uint8_t* d_topic_bytes, const uint64_t* d_topic_off,
                                 uint32_t n, uint64_t topic_bytes, uint32_t* d_out_count, uint64_t* d_out_off,
                                 uint32_t* d_out_src, uint32_t* d_out_dest, uint64_t out_cap, uint64_t* d_total,
                                 void* hip_stream);

/* ---- emqx_broker:aggre/1 (emqx_amd/csrc/aggre.hip) -----------
 * publish/1 routes aggre(match_routes(Topic)) (src/emqx_broker.erl:152):
 * each #route{topic = To, dest} becomes {To, Node} for a node dest and
 * {To, Group} for a {Group, Node} dest; the fold prepends node entries and
 * lists:usort()s the whole accumulator at every group entry (:194-206).
 * Dest bytes are opaque to the engine, so the caller declares each dest's
 * target: kind TM_TARGET_NODE (key = the node atom's text) or
 * TM_TARGET_GROUP (key = the group binary).  An undeclared dest is a node
 * named by its dest bytes.  Sorting follows Erlang term order: To bytewise
 * (a proper prefix first), then node atoms before group binaries, each
 * bytewise. */
#define TM_TARGET_NODE  0u
#define TM_TARGET_GROUP 1u
int tm_dest_target(tm_engine* e, const uint8_t* dest, uint32_t dlen, uint32_t kind, const uint8_t* key,
                   uint32_t klen, uint32_t* target_out);
/* target id -> key bytes (engine-owned, stable; *kind = TM_TARGET_*) */
const uint8_t* tm_target_bytes(tm_engine* e, uint32_t target_id, uint32_t* kind, uint32_t* len);

/* aggre(emqx_router:match_routes(T)) per topic of a batch: entries of topic t
 * are out_to/out_target[out_off[t] .. +out_count[t]), out_to = TM_ROUTE_TOPIC
 * for the literal topic else the filter id (the To of the pair), out_target =
 * target id.  out_off are match_routes/1's offsets (aggre never lengthens a
 * list, so each list sits at its route offset and needs no compaction):
 * out_count[t] <= out_off[t+1] - out_off[t], and out_needed / *d_total is the
 * route total.  Host buffers, synchronous; TM_ENOSPC / out_needed as
 * tm_match_batch.  Walk, route expansion and aggre all run on the GPU. */
int tm_match_deliveries_batch(tm_engine* e, const uint8_t* topic_bytes, const uint64_t* topic_off, uint32_t n,
                              uint32_t* out_count, uint64_t* out_off, uint32_t* out_to, uint32_t* out_target,
                              uint64_t out_cap, uint64_t* out_needed);
/* Same with device buffers on hip_stream; *d_total = route total, entries at
 * or past out_cap are dropped. */
int tm_match_deliveries_batch_device(tm_engine* e, const uint8_t* d_topic_bytes, const uint64_t* d_topic_off,
                                     uint32_t n, uint64_t topic_bytes, uint32_t* d_out_count, uint64_t* d_out_off,
                                     uint32_t* d_out_to, uint32_t* d_out_target, uint64_t out_cap,
                                     uint64_t* d_total, void* hip_stream);

/* ---- publish micro-batcher (emqx_amd/csrc/batcher.cpp) -----
 * emqx_broker:publish/1 (src/emqx_broker.erl:148-157) matches one topic per
 * call in the publisher's process.  The NIF instead submits the topic here
 * and returns at once; a sealing thread closes a batch at max_topics /
 * max_bytes, or deadline_us after its first topic, and hands it to a free
 * lane: lanes_per_replica lanes per GPU of the engine, each with its own
 * thread and stream, so several batches are in flight on every GPU.  A lane
 * runs its batch (match/1, or match_routes/1 with TM_BATCHER_ROUTES, or
 * aggre(match_routes/1) with TM_BATCHER_DELIVERIES), reads back exactly the
 * results, and calls done() once per topic of the batch, in submission
 * order, from the lane's thread (or, with callback_threads, from the lane and
 * those threads, each part of the batch in submission order); different
 * batches complete independently
 * (a publisher waits for its own reply before publishing again).  The id /
 * dest arrays are valid only during the callback (the NIF copies them into a
 * term and enif_send()s it).  status != TM_OK: ids are null. */
#define TM_BATCHER_ROUTES 1u   /* results are match_routes/1 (src ids + dest ids) */
#define TM_BATCHER_DELIVERIES 2u   /* results are aggre(match_routes/1) (To ids + target ids) */
#define TM_BATCHER_CSR 8u   /* small match/1 batches through tm_match_batch_device (four launches and a
                              scan) instead of the one-launch tm_match_small_device (A/B) */
#define TM_BATCHER_EAGER 4u   /* seal as soon as a lane is free AND the oldest pending topic has waited
                                 eager_us or TM_BATCHER_EAGER_TOPICS are pending (deadline_us stays the
                                 upper bound): low load runs small batches early, high load batches up
                                 while lanes are busy, and no load makes batches of a handful of topics
                                 (a sealed batch costs ~100 us of host and PCIe latency, and tens of
                                 thousands of them a second crowd the host: the p99 of sealing at every
                                 free lane was 4 ms at 1M publishes/s) */
#define TM_BATCHER_EAGER_TOPICS 256u

typedef struct tm_batcher tm_batcher;
typedef struct tm_batcher_config {
    uint32_t max_topics;      /* seal at this many pending topics (0 = 65536); a seal takes every pending topic */
    uint32_t deadline_us;     /* seal this long after the first topic (0 = 200)  */
    uint64_t max_bytes;       /* seal at this many topic bytes (0 = 64 MiB)      */
    uint32_t flags;           /* TM_BATCHER_ROUTES | TM_BATCHER_DELIVERIES      */
    uint32_t lanes_per_replica; /* batches in flight per GPU (0 = 2)            */
    uint32_t callback_threads;  /* threads that share a batch's callbacks with its lane
                                   (parts of >= 8192 topics; 0 = the lane alone) */
    uint32_t eager_us;        /* TM_BATCHER_EAGER: least age of the oldest pending topic for a seal at a
                                 free lane (0 = 40; >= deadline_us: deadline sealing) */
} tm_batcher_config;
typedef struct tm_batcher_stats {
    uint64_t batches, topics, results, max_batch;
    uint64_t size_seals, deadline_seals, failed_batches;
    /* where a batch's time goes, summed over batches (ns): sealed -> its lane
     * starts, packing into pinned memory, the device path with both
     * read-backs, the callbacks; within the device path, the host time
     * spent enqueueing the copies and kernels and waiting on the stream */
    uint64_t wait_ns, pack_ns, device_ns, callback_ns;
    uint64_t launch_ns, sync_ns;
    /* the largest of each over single batches (ns) since the batcher opened
     * or the last read with TM_BATCHER_STATS_RESET_MAX: where a stall sat.
     * Only tm_batcher_get_stats2 writes these (a caller built against the
     * round-4 header, whose struct ends before them, keeps calling
     * tm_batcher_get_stats, which writes exactly that prefix) */
    uint64_t max_wait_ns, max_pack_ns, max_device_ns, max_callback_ns, max_sync_ns;
} tm_batcher_stats;
#define TM_BATCHER_STATS_V1_BYTES (13u * 8u)   /* the prefix tm_batcher_get_stats writes */
#define TM_BATCHER_STATS_RESET_MAX 1u          /* tm_batcher_get_stats2: zero the max_* fields after this read */
/* ids: filter ids (match/1), route sources (match_routes/1) or To ids
 * (deliveries); dests: route dest ids, target ids (deliveries) or null; n:
 * list length */
typedef void (*tm_batch_done_fn)(void* ctx, uint64_t ticket, int status, const uint32_t* ids,
                                 const uint32_t* dests, uint32_t n);

int  tm_batcher_open(tm_engine* e, const tm_batcher_config* cfg, tm_batcher** out);
int  tm_batcher_submit(tm_batcher* b, const uint8_t* topic, uint32_t len, tm_batch_done_fn done, void* ctx,
                       uint64_t* ticket_out);
/* seal the open batch and wait until every submitted topic has completed */
int  tm_batcher_flush(tm_batcher* b);
/* the counters up to sync_ns (TM_BATCHER_STATS_V1_BYTES bytes; max_* untouched) */
int  tm_batcher_get_stats(tm_batcher* b, tm_batcher_stats* out);
/* min(out_size, sizeof(tm_batcher_stats)) bytes of the stats (out_size <
 * TM_BATCHER_STATS_V1_BYTES: TM_EINVAL); flags TM_BATCHER_STATS_RESET_MAX
 * starts a new max_* window after the read (only the reader that owns the
 * window should pass it) */
int  tm_batcher_get_stats2(tm_batcher* b, tm_batcher_stats* out, uint32_t out_size, uint32_t flags);
/* flush, then stop the worker */
void tm_batcher_close(tm_batcher* b);

/* ---- batched ACL checks (emqx_amd/csrc/acl.hip) ---------------
 * The internal ACL module (src/emqx_acl_internal.erl) keeps the compiled
 * rules of etc/acl.conf and answers check_acl({Credentials, PubSub, Topic})
 * with the first matching rule of that access type (match/3, :63-87).  A
 * tm_acl holds the rules in order, built like emqx_access_rule:compile/1
 * (src/emqx_access_rule.erl:38-75):
 *   tm_acl_rule_begin(allow, access)   {allow|deny, Who, Access, Topics} / {allow|deny, all}
 *   tm_acl_who(kind, arg, len, prefix) Who: all | {client, C} | {user, U} | {client, all} |
 *                                      {user, all} | {ipaddr, "a.b.c.d[/n]"} (prefix = n, 0 = host);
 *                                      {'and' | 'or', [...]}: AND/OR, the conditions, END
 *   tm_acl_topic(eq, topic, len)       a topic filter, or {eq, Topic}; "%c"/"%u" levels make a
 *                                      pattern (feed_var/3, :136-149)
 *   tm_acl_rule_end()
 * tm_acl_check_batch evaluates n checks on the GPU: out_result[i] = 1 allow,
 * 0 deny, -1 nomatch (the module's ignore); out_rule[i] = index of the
 * matching rule (or 0xFFFFFFFF).  Credentials: client id / username bytes
 * with a defined flag (undefined = the atom), peer address 16 B per check
 * with family 4 / 6 (0 = no peername); peers may be NULL.  Topics are
 * matched as word lists (emqx_access_rule:match_topic/2: no '$' rule). */
#define TM_ACL_ALL        0u   /* {allow|deny, all}: matches any check */
#define TM_ACL_PUBLISH    1u
#define TM_ACL_SUBSCRIBE  2u
#define TM_ACL_PUBSUB     3u
#define TM_ACL_WHO_ALL        0u
#define TM_ACL_WHO_CLIENT     1u
#define TM_ACL_WHO_USER       2u
#define TM_ACL_WHO_CLIENT_ALL 3u
#define TM_ACL_WHO_USER_ALL   4u
#define TM_ACL_WHO_IPADDR     5u
#define TM_ACL_WHO_AND        6u
#define TM_ACL_WHO_OR         7u
#define TM_ACL_WHO_END        8u
typedef struct tm_acl tm_acl;
int  tm_acl_open(int device, tm_acl** out);
void tm_acl_close(tm_acl* a);
int  tm_acl_rule_begin(tm_acl* a, int allow, uint32_t access);
int  tm_acl_who(tm_acl* a, uint32_t kind, const uint8_t* arg, uint32_t len, uint32_t prefix);
int  tm_acl_topic(tm_acl* a, int eq, const uint8_t* topic, uint32_t len);
int  tm_acl_rule_end(tm_acl* a);
int  tm_acl_rule_count(tm_acl* a);
int  tm_acl_check_batch(tm_acl* a, uint32_t n, const uint8_t* access, const uint8_t* topics,
                        const uint64_t* topic_off, const uint8_t* client_ids, const uint64_t* client_off,
                        const uint8_t* client_defined, const uint8_t* usernames, const uint64_t* user_off,
                        const uint8_t* user_defined, const uint8_t* peers, const uint8_t* peer_family,
                        int8_t* out_result, uint32_t* out_rule);

/* Same with every buffer device-resident (HBM; byte offsets index topics /
 * client_ids / usernames directly), stream-ordered on hip_stream, no
 * synchronisation: the form a pipelined caller and the ACL bench use. */
int tm_acl_check_batch_device(tm_acl* a, uint32_t n, const uint8_t* d_access, const uint8_t* d_topics,
                              const uint64_t* d_topic_off, const uint8_t* d_client_ids, const uint64_t* d_client_off,
                              const uint8_t* d_client_defined, const uint8_t* d_usernames, const uint64_t* d_user_off,
                              const uint8_t* d_user_defined, const uint8_t* d_peers, const uint8_t* d_peer_family,
                              int8_t* d_out_result, uint32_t* d_out_rule, void* hip_stream);

/* ---- batched topic-rewrite rule selection (rewrite.hip) -------
 * emqx_mod_rewrite:match_rule/2 (src/emqx_mod_rewrite.erl:52-59) applies the
 * FIRST rule whose filter emqx_topic:match/2 accepts (the binary clause with
 * the '$' rule, src/emqx_topic.erl:56-61), then that rule's regex.  A
 * tm_rewrite holds the rules' filters in order (compile/1 order); the batch
 * calls return, per topic, the index of the first matching rule or
 * TM_NO_RULE.  The regex (re:run + re:replace of match_regx/3) stays with
 * the caller. */
#define TM_NO_RULE 0xFFFFFFFFu
typedef struct tm_rewrite tm_rewrite;
int  tm_rewrite_open(int device, tm_rewrite** out);
void tm_rewrite_close(tm_rewrite* r);
int  tm_rewrite_rule(tm_rewrite* r, const uint8_t* filter, uint32_t len);   /* appended as the next rule */
int  tm_rewrite_rule_count(tm_rewrite* r);
int  tm_rewrite_match_batch(tm_rewrite* r, const uint8_t* topics, const uint64_t* topic_off, uint32_t n,
                            uint32_t* out_rule);
/* device buffers (topic t = d_topics[d_topic_off[t] .. d_topic_off[t+1])), stream-ordered */
int  tm_rewrite_match_batch_device(tm_rewrite* r, const uint8_t* d_topics, const uint64_t* d_topic_off, uint32_t n,
                                   uint32_t* d_out_rule, void* hip_stream);

/* Engine knobs (the app-env analogue of SURVEY §5 config):
 *   "xcdq"     1 = per-XCD dequeue heads over contiguous ranges of the batch
 *              (default), 0 = one global head
 *   "walk_bpc" walk workgroups per CU, 0 = full occupancy (default)
 *   "hist"     1 = per-level visit/probe histogram in stats mode (diagnostic)
 *   "layout"   1 = renumber nodes in DFS preorder on commit once >= 1/4 of
 *              the live nodes are new (default), 0 = keep insertion order,
 *              2 = renumber on every commit
 *   "stage_k"  ids staged per topic before a fan-out re-walk (4..4096, % 4 == 0);
 *              setting it fixes K (turns "stage_auto" off)
 *   "stage_auto" 1 = grow K to the largest list of the previous walk, within
 *              a 16 GiB stage footprint (default), 0 = fixed K
 *   "split"    1 = walk reads separate inner / leaf half arrays (default),
 *              0 = interleaved 32 B records
 *   "blocks"   1 = a WIDE node's literal children in a block of its own
 *              (per-node open addressing, blocks in node order), 0 = the
 *              shared edge table (default; converted at the next commit)
 *   "block_load" blocks kept at load <= 1/value (2..16, default 4)
 *   "block_gc" garbage block slots before a compaction (default 2^20)
 *   "relayout" 1 = relayout the image at the next commit
 *   "hot_levels" depths laid out level by level first at relayout (0..16,
 *              default 4; 0 = DFS preorder throughout); forces a relayout
 *   "presort"  1 = walk each batch in the order of a key of its first words
 *              (device radix sort); 2 = the tail order: within each XCD
 *              range the topics whose words label the most trie nodes first
 *              (one radix pass), so the walk's last lanes finish on light
 *              topics (batches above wave_walk_max); 5 = the word-hash key
 *              within each XCD range (two radix passes); 6 = order 5 with
 *              each range's lightest topics last ("light_tail" per mille,
 *              default 60); 3 = by batch: 6 for heavy batches (lists mostly
 *              past the stage row), else 5 from "sort_min" topics on, 2
 *              below (default); 0 = arrival order; 4 = the tail order, then
 *              the word-hash key within a heat class (A/B)
 *   "sort_min" presort 3's smallest batch walked in range-local word-hash order
 *              (default 1500000)
 *   "sort_bits" the key bits presort 1 and 5 sort, one radix pass per 8
 *              (8..32, default 24; presort 5: the XCD range over the
 *              word-hash key's top sort_bits - 3 bits)
 *   "chunk_rows" 1 = a wave copies each taken chunk's 64 tokenized rows to
 *              LDS at once (default), 0 = each lane reads its topic's row
 *   "spill"    1 = ids past a stage row go to per-XCD spill chunks (default),
 *              0 = the copy-out re-walks such topics
 *   "wave_walk_max" batches of at most this many topics take the
 *              wave-per-topic level-synchronous walk (default 32768, 0 = never)
 *   "summaries" 1 = subtree summaries prune dead '+' / literal subtrees (default)
 *   "order"    relayout order bits (default 15: '+' child after its parent,
 *              '#' nodes last, heat order, heat from filter counts)
 *   "edge_load" edge tables kept at load <= 1/edge_load (2..16, default 4)
 *   "hot_edges" parents of depth < D probe a separate small table (0 = off)
 *   "slots"    per-batch workspace slots rotated over by consecutive batches
 *   "double_buffer" 1 = two image epochs per replica (commits never wait on
 *              walks; default), 0 = one
 *   "shape_keys" 1 = keyed batches of <= 31 levels walk unkeyed and key each
 *              id by its filter's shape (the shard engines set it), 0 = keyed
 *              walk (default)
 *   "route_gc" garbage dest entries before a route-pool compaction is considered
 *   "root_split" 1 = walk each topic as two queue items (the root's '+'
 *              subtree, the rest), 0 = one (default; slower at C3)
 *   "donate"   1 = once the queues are dry, lanes still walking hand pending
 *              '+' subtrees to idle lanes of their wave (ordered pieces of the
 *              topic's list), 0 = off (default; no gain at C3)
 *   "donate_busy" donate only while at most this many lanes of a wave walk
 *              (0..64, default 8); "donate_min" levels below a donated node
 *              (default 2); "donate_max" largest batch that donates
 * TM_EINVAL for unknown names / values. */
int tm_set_option(tm_engine* e, const char* name, int64_t value);

/* Pre-size every replica's match workspaces for batches of up to n_topics
 * topics of n_bytes topic bytes (optional).  Workspaces otherwise grow on
 * demand, and each growth frees and reallocates device memory, which waits
 * for the whole device: a stall of milliseconds in the middle of a stream of
 * batches.  tm_batcher_open reserves for its batches.  No reference
 * counterpart (an allocation hint, like tm_set_option). */
int tm_reserve(tm_engine* e, uint32_t n_topics, uint64_t n_bytes);

/* Counters of the last batch (visits, reference edge reads, matches).  Costs
 * one extra device pass; enable with tm_set_stats(e, 1) before the batch. */
int tm_set_stats(tm_engine* e, int enable);
int tm_last_stats(tm_engine* e, tm_batch_stats* out);

/* Per-kernel device times (ms), measured with hipEvents recorded around each
 * kernel stage on the stream the stage ran on; enable with tm_set_timing(e, 1).
 * Returns, per stage, the average over every batch since the previous call
 * (synchronising on those events).  names[i] point at static strings.
 * Returns the number of entries. */
int tm_set_timing(tm_engine* e, int enable);
int tm_last_kernel_times(tm_engine* e, const char** names, float* ms, int cap);

/* ---- pure topic algebra (no engine) ----------------------------------------
 * emqx_topic:match/2 (binary, binary) — src/emqx_topic.erl:56-75.  1 / 0. */
int tm_topic_match(const uint8_t* name, uint32_t nlen, const uint8_t* filt, uint32_t flen);
/* emqx_topic:wildcard/1 — src/emqx_topic.erl:41-50.  1 / 0. */
int tm_topic_wildcard(const uint8_t* topic, uint32_t len);
/* emqx_topic:parse/1 — src/emqx_topic.erl:180-200.  Strips "$queue/" and
 * "$share/<group>/".  On success *inner points into `topic`, *group into
 * `topic` (or NULL when not shared; "$queue" for $queue/).  TM_EINVAL on the
 * reference's {invalid_topic, _} errors. */
int tm_topic_parse(const uint8_t* topic, uint32_t len, const uint8_t** inner, uint32_t* inner_len,
                   const uint8_t** group, uint32_t* group_len);

/* library identity: "gfx950" build tag, for loaders that must fail loudly */
const char* tm_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* TOPICMATCH_H */
