// exchange.cpp — the sharded mode's exchange of keyed match lists
// (SURVEY §8(e), config C4), natively over RCCL.
//
// With the filter set partitioned over S GPUs, every shard walks the whole
// publish batch against its sub-trie with order keys
// (tm_match_batch_device_keys_w); then topic slice d of every shard's lists
// must reach rank d, which merges the S lists of each of its topics into
// emqx_trie:match/1 order (tm_shard_merge_w).  That is an all-to-all: every
// id crosses xGMI once (an all-gather would move S x the bytes for each rank
// to keep 1/S).  Per exchange:
//
//   1. tm_slice_sizes: ids and first id of each destination slice (device),
//      read back (S u64 pairs) to size the sends;
//   2. one RCCL group: counts of slice d -> rank d (u32 x m_d), and the
//      per-destination id counts (ncclAllToAll of one u64), read back to
//      size the receive buffers;
//   3. one RCCL group: ids, then each key plane, slice d -> rank d.
//
// Backends: RCCL (one communicator per rank: tm_comm_init_rank across
// processes, tm_comm_init_all for the GPUs of one process) or, for ranks of
// one process that share a GPU (which RCCL refuses: "Duplicate GPU"), plain
// device-to-device copies between the ranks' buffers (tm_comm_init_all
// chooses it then).  Both move the same bytes to the same places.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/topicmatch.h"
#include "kernels.h"

using namespace tmx;

namespace {

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool ensure(size_t need) {
        if (need <= bytes && p) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        const size_t want = std::max<size_t>(256, need + need / 4);
        if (hipMalloc(&p, want) != hipSuccess) return false;
        bytes = want;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

inline uint32_t slice_lo(uint32_t n, uint32_t S, uint32_t d) { return (uint32_t)((uint64_t)n * d / S); }


// The RCCL group this thread has open (ncclGroupStart .. ncclGroupEnd) and
// the communicators queued into it.  A failure between the two must not
// return with the group open (the next collective on these communicators
// would be queued into the broken group): fail() closes it and aborts those
// communicators, whose operations the peers can no longer complete; later
// exchanges on them report TM_EDEVICE.
thread_local int t_group_depth = 0;
thread_local std::vector<tm_comm*> t_group_comms;

int fail(tm_comm* c, const std::string& what, int code = TM_EDEVICE);
}  // namespace

struct tm_comm {
    int device = -1;
    uint32_t nranks = 1, rank = 0;
    ncclComm_t nccl = nullptr;    // RCCL backend (null: device copies within one process)
    bool aborted = false;         // aborted after a failure inside an RCCL group
    bool self_rccl = false;       // tm_comm_set_self_rccl: the rank's own part over RCCL too
    hipStream_t stream = nullptr;
    Buf sizes;                    // 2S u64: send counts per destination, then their first ids
    Buf rsizes;                   // S u64: ids to receive from each source
    Buf recv_counts, src_base, recv_ids, recv_keys;
    std::vector<uint64_t> h_send, h_recv, h_base;   // h_base: source of the async src_base upload
    std::string last_error;
    // routed mode (tm_route_exchange / tm_route_return): this rank's batch
    // in owner buckets, what it received, and the lists on their way back
    struct Route {
        uint32_t n = 0, m = 0;
        Buf owner, blk_cnt, blk_base, bucket, perm, slen, soff, scan_tmp, sbuf, cuts;
        std::vector<uint32_t> h_bucket;                 // S+1: topic base of each owner's bucket
        std::vector<uint64_t> h_cuts;                   // S+1: byte base of each bucket
        std::vector<uint64_t> h_sz, h_rsz;              // [topics, bytes] sent to / received from each peer
        std::vector<uint64_t> rt_base, rb_base;         // S+1: received topics / bytes by source
        Buf rlen, rbuf, roff, rscan;
        // return: the owner's id cut per source, ids coming back per owner
        Buf seg_idx, seg_cut, ret_sz, ret_rsz;
        std::vector<uint32_t> h_seg_idx;
        std::vector<uint64_t> h_seg_cut, h_ret;          // S+1 id cuts; S ids back from each owner
        Buf rcount, rids, rroff, out_count, out_off, out_ids, out_total, uscan;
        uint64_t total = 0;
    } rt;
};

namespace {
// abort the communicators of this thread's RCCL group (their peers can no
// longer complete the group's operations)
void abort_group(tm_comm* c, const std::string& what) {
    for (tm_comm* g : t_group_comms)
        if (g && g->nccl && !g->aborted) {
            (void)ncclCommAbort(g->nccl);
            g->nccl = nullptr;
            g->aborted = true;
            if (g != c) g->last_error = "aborted with its RCCL group: " + what;
        }
    t_group_comms.clear();
}

int fail(tm_comm* c, const std::string& what, int code) {
    if (c) c->last_error = what;
    if (t_group_depth > 0) {
        t_group_depth = 0;
        (void)ncclGroupEnd();
        abort_group(c, what);
    }
    return code;
}
#define XHIP(c, x)                                                                          \
    do {                                                                                    \
        hipError_t _e = (x);                                                                \
        if (_e != hipSuccess) return fail(c, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)
#define XNCCL(c, x)                                                                             \
    do {                                                                                        \
        ncclResult_t _r = (x);                                                                  \
        if (_r != ncclSuccess) return fail(c, std::string(#x) + ": " + ncclGetErrorString(_r)); \
    } while (0)

#define XGROUP_START(c, comms)                 \
    do {                                       \
        XNCCL(c, ncclGroupStart());            \
        ++t_group_depth;                       \
        t_group_comms = (comms);               \
    } while (0)
// ncclGroupEnd first, with the group state still set: when it fails, fail()
// aborts the group's communicators (the group is already closed, so fail()
// must not end it again: t_group_depth is cleared before the call)
#define XGROUP_END(c)                                                                    \
    do {                                                                                 \
        const ncclResult_t _g = ncclGroupEnd();                                          \
        if (_g != ncclSuccess) {                                                         \
            t_group_depth = 0;                                                           \
            abort_group(c, std::string("ncclGroupEnd: ") + ncclGetErrorString(_g));     \
            return fail(c, std::string("ncclGroupEnd: ") + ncclGetErrorString(_g));     \
        }                                                                                \
        t_group_depth = 0;                                                               \
        t_group_comms.clear();                                                           \
    } while (0)

hipStream_t stream_of(tm_comm* c, const tm_exchange_in& in) {
    return in.hip_stream ? (hipStream_t)in.hip_stream : c->stream;
}

// step 1 for one rank: send sizes / offsets to the host
int send_sizes(tm_comm* c, const tm_exchange_in& in) {
    const uint32_t S = c->nranks;
    hipStream_t st = stream_of(c, in);
    if (!c->sizes.ensure(2 * S * 8) || !c->rsizes.ensure(S * 8)) return fail(c, "hipMalloc", TM_ENOMEM);
    XHIP(c, launch_slice_sizes(in.d_offs, in.n, S, c->sizes.as<uint64_t>(), st));
    c->h_send.resize(2 * S);
    XHIP(c, hipMemcpyAsync(c->h_send.data(), c->sizes.p, 2 * S * 8, hipMemcpyDeviceToHost, st));
    XHIP(c, hipStreamSynchronize(st));
    return TM_OK;
}

// receive buffers for recv_items[s] from each source: counts, bases, ids, keys
int alloc_recv(tm_comm* c, const tm_exchange_in& in, tm_exchange_out& out) {
    const uint32_t S = c->nranks;
    const uint32_t m = slice_lo(in.n, S, c->rank + 1) - slice_lo(in.n, S, c->rank);
    std::vector<uint64_t>& base = c->h_base;   // outlives the async upload below
    base.assign(S, 0);
    uint64_t tot = 0;
    for (uint32_t s = 0; s < S; ++s) {
        base[s] = tot;
        tot += c->h_recv[s];
    }
    if (!c->recv_counts.ensure((size_t)S * m * 4 + 4) || !c->src_base.ensure(S * 8) ||
        !c->recv_ids.ensure(tot * 4 + 4) || !c->recv_keys.ensure(tot * 8 * in.key_words + 8))
        return fail(c, "hipMalloc", TM_ENOMEM);
    XHIP(c, hipMemcpyAsync(c->src_base.p, base.data(), S * 8, hipMemcpyHostToDevice, stream_of(c, in)));
    out.m = m;
    out.total = tot;
    out.d_counts = c->recv_counts.as<uint32_t>();
    out.d_src_base = c->src_base.as<uint64_t>();
    out.d_ids = c->recv_ids.as<uint32_t>();
    out.d_keys = c->recv_keys.as<uint64_t>();
    return TM_OK;
}

bool valid_in(const tm_exchange_in& in) {
    return in.d_offs && in.key_words >= 1 && in.key_words <= TM_MAX_KEY_WORDS && (in.n == 0 || in.d_counts);
}

// ---- routed mode ------------------------------------------------------------

hipStream_t route_stream(tm_comm* c, void* s) { return s ? (hipStream_t)s : c->stream; }

// step 1 (one rank): bucket the batch by owner, read the bucket cuts back
int route_plan(tm_comm* c, const tm_route_in& in) {
    const uint32_t S = c->nranks, n = in.n;
    tm_comm::Route& r = c->rt;
    hipStream_t st = route_stream(c, in.hip_stream);
    const uint64_t nbytes = n ? in.bytes : 0;
    const uint64_t nb = (n + 255) / 256;
    if (!r.owner.ensure(n + 8) || !r.blk_cnt.ensure((nb + 1) * S * 4) || !r.blk_base.ensure((nb + 1) * S * 4) ||
        !r.bucket.ensure((S + 1) * 4) || !r.perm.ensure((size_t)n * 4 + 4) || !r.slen.ensure((size_t)n * 4 + 4) ||
        !r.soff.ensure(((size_t)n + 1) * 8) || !r.scan_tmp.ensure(scan_tmp_elems(n) * 8 + 8) ||
        !r.sbuf.ensure(nbytes + 16) || !r.cuts.ensure((S + 1) * 8))
        return fail(c, "hipMalloc", TM_ENOMEM);
    RoutePlanBufs w{r.owner.as<uint8_t>(), r.blk_cnt.as<uint32_t>(), r.blk_base.as<uint32_t>(), r.bucket.as<uint32_t>(),
                    r.perm.as<uint32_t>(), r.slen.as<uint32_t>(), r.soff.as<uint64_t>(), r.scan_tmp.as<uint64_t>(),
                    r.sbuf.as<uint8_t>(), r.cuts.as<uint64_t>()};
    XHIP(c, launch_route_plan(in.d_bytes, in.d_off, n, in.depth, S, w, st));
    r.n = n;
    r.h_bucket.resize(S + 1);
    r.h_cuts.resize(S + 1);
    XHIP(c, hipMemcpyAsync(r.h_bucket.data(), r.bucket.p, (S + 1) * 4, hipMemcpyDeviceToHost, st));
    XHIP(c, hipMemcpyAsync(r.h_cuts.data(), r.cuts.p, (S + 1) * 8, hipMemcpyDeviceToHost, st));
    XHIP(c, hipStreamSynchronize(st));
    r.h_sz.assign(2 * S, 0);
    for (uint32_t p = 0; p < S; ++p) {
        r.h_sz[2 * p] = r.h_bucket[p + 1] - r.h_bucket[p];
        r.h_sz[2 * p + 1] = r.h_cuts[p + 1] - r.h_cuts[p];
    }
    return TM_OK;
}

// step 2 (one rank, after h_rsz is known): receive buffers
int route_alloc_recv(tm_comm* c) {
    const uint32_t S = c->nranks;
    tm_comm::Route& r = c->rt;
    r.rt_base.assign(S + 1, 0);
    r.rb_base.assign(S + 1, 0);
    for (uint32_t s = 0; s < S; ++s) {
        r.rt_base[s + 1] = r.rt_base[s] + r.h_rsz[2 * s];
        r.rb_base[s + 1] = r.rb_base[s] + r.h_rsz[2 * s + 1];
    }
    if (r.rt_base[S] > 0xFFFFFFF0ull) return fail(c, "routed batch past 2^32 topics", TM_ENOSPC);
    r.m = (uint32_t)r.rt_base[S];
    if (!r.rlen.ensure((size_t)r.m * 4 + 4) || !r.rbuf.ensure(r.rb_base[S] + 16) ||
        !r.roff.ensure(((size_t)r.m + 1) * 8) || !r.rscan.ensure(scan_tmp_elems(r.m) * 8 + 8))
        return fail(c, "hipMalloc", TM_ENOMEM);
    return TM_OK;
}

// step 3 (one rank, after the transfers): offsets of the received batch
int route_finish(tm_comm* c, hipStream_t st, tm_route_out* out) {
    tm_comm::Route& r = c->rt;
    XHIP(c, hipMemsetAsync(r.rbuf.as<uint8_t>() + r.rb_base[c->nranks], 0, 16, st));
    XHIP(c, launch_scan0(r.rlen.as<uint32_t>(), r.m, r.roff.as<uint64_t>(), r.roff.as<uint64_t>() + r.m,
                        r.rscan.as<uint64_t>(), st));
    out->m = r.m;
    out->reserved = 0;
    out->bytes = r.rb_base[c->nranks];
    out->d_bytes = r.rbuf.as<uint8_t>();
    out->d_off = r.roff.as<uint64_t>();
    return TM_OK;
}

// return step 1 (one rank): the owner's id cut at every source boundary
int return_cuts(tm_comm* c, const tm_route_lists& l) {
    const uint32_t S = c->nranks;
    tm_comm::Route& r = c->rt;
    hipStream_t st = route_stream(c, l.hip_stream);
    r.h_seg_idx.resize(S + 1);
    for (uint32_t s = 0; s <= S; ++s) r.h_seg_idx[s] = (uint32_t)r.rt_base[s];
    if (!r.seg_idx.ensure((S + 1) * 4) || !r.seg_cut.ensure((S + 1) * 8)) return fail(c, "hipMalloc", TM_ENOMEM);
    XHIP(c, hipMemcpyAsync(r.seg_idx.p, r.h_seg_idx.data(), (S + 1) * 4, hipMemcpyHostToDevice, st));
    XHIP(c, launch_gather_u64(l.d_offs, r.seg_idx.as<uint32_t>(), S + 1, r.seg_cut.as<uint64_t>(), st));
    r.h_seg_cut.resize(S + 1);
    XHIP(c, hipMemcpyAsync(r.h_seg_cut.data(), r.seg_cut.p, (S + 1) * 8, hipMemcpyDeviceToHost, st));
    XHIP(c, hipStreamSynchronize(st));
    return TM_OK;
}

// return step 2 (one rank, after h_ret is known): buffers of the lists coming back
int return_alloc(tm_comm* c) {
    tm_comm::Route& r = c->rt;
    uint64_t tot = 0;
    for (uint64_t x : r.h_ret) tot += x;
    r.total = tot;
    const uint32_t n = r.n;
    if (!r.rcount.ensure((size_t)n * 4 + 4) || !r.rids.ensure(tot * 4 + 4) || !r.rroff.ensure(((size_t)n + 1) * 8) ||
        !r.out_count.ensure((size_t)n * 4 + 4) || !r.out_off.ensure(((size_t)n + 1) * 8) ||
        !r.out_ids.ensure(tot * 4 + 4) || !r.out_total.ensure(8) || !r.uscan.ensure(scan_tmp_elems(n) * 8 + 8))
        return fail(c, "hipMalloc", TM_ENOMEM);
    return TM_OK;
}

// return step 3 (one rank): the lists in the batch's own topic order
int return_finish(tm_comm* c, hipStream_t st, tm_route_result* res) {
    tm_comm::Route& r = c->rt;
    XHIP(c, launch_scan0(r.rcount.as<uint32_t>(), r.n, r.rroff.as<uint64_t>(), r.rroff.as<uint64_t>() + r.n,
                        r.uscan.as<uint64_t>(), st));
    XHIP(c, launch_route_unpermute(r.rcount.as<uint32_t>(), r.rroff.as<uint64_t>(), r.rids.as<uint32_t>(),
                                   r.perm.as<uint32_t>(), r.n, r.out_count.as<uint32_t>(), r.out_off.as<uint64_t>(),
                                   r.out_ids.as<uint32_t>(), r.out_total.as<uint64_t>(), r.uscan.as<uint64_t>(), st));
    res->n = r.n;
    res->reserved = 0;
    res->total = r.total;
    res->d_counts = r.out_count.as<uint32_t>();
    res->d_offs = r.out_off.as<uint64_t>();
    res->d_ids = r.out_ids.as<uint32_t>();
    return TM_OK;
}

// one transfer of a routed exchange: bytes from rank src's buffer to rank dst's
struct Xfer {
    uint32_t src, dst;
    const void* sp;
    void* dp;
    size_t bytes;
};
// the transfers of ranks comms[0..k) of one process: an RCCL group over their
// communicators (a rank's own part a device copy), or device copies
int run_xfers(tm_comm** comms, uint32_t k, const std::vector<Xfer>& xs, const std::vector<hipStream_t>& st,
              bool rccl) {
    // comm of rank r among comms (single-rank callers pass their one comm)
    auto of = [&](uint32_t rank) -> int {
        for (uint32_t i = 0; i < k; ++i)
            if (comms[i]->rank == rank) return (int)i;
        return -1;
    };
    tm_comm* c0 = comms[0];
    if (rccl) XGROUP_START(c0, std::vector<tm_comm*>(comms, comms + k));
    for (const Xfer& x : xs) {
        if (!x.bytes) continue;
        const int is = of(x.src), id = of(x.dst);
        const bool self_copy = x.src == x.dst && !(rccl && is >= 0 && comms[is]->self_rccl);
        if (self_copy || !rccl) {   // a device copy (same rank, or ranks of one process without RCCL)
            if (is < 0 || id < 0) return fail(c0, "routed exchange: copy between ranks of different processes");
            XHIP(comms[id], hipMemcpyPeerAsync(x.dp, comms[id]->device, x.sp, comms[is]->device, x.bytes, st[id]));
            continue;
        }
        if (is >= 0) XNCCL(comms[is], ncclSend(x.sp, x.bytes, ncclUint8, (int)x.dst, comms[is]->nccl, st[is]));
        if (id >= 0) XNCCL(comms[id], ncclRecv(x.dp, x.bytes, ncclUint8, (int)x.src, comms[id]->nccl, st[id]));
    }
    if (rccl) XGROUP_END(c0);
    return TM_OK;
}

}  // namespace

extern "C" {

int tm_comm_unique_id(uint8_t id[TM_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == TM_COMM_ID_BYTES, "ncclUniqueId is 128 bytes");
    if (!id) return TM_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return TM_EDEVICE;
    std::memcpy(id, &u, sizeof(u));
    return TM_OK;
}

int tm_comm_init_rank(const uint8_t id[TM_COMM_ID_BYTES], uint32_t nranks, uint32_t rank, int device,
                      tm_comm** out) {
    if (!id || !out || nranks == 0 || rank >= nranks || nranks > 64) return TM_EINVAL;
    *out = nullptr;
    std::unique_ptr<tm_comm> c(new (std::nothrow) tm_comm());
    if (!c) return TM_ENOMEM;
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return TM_EDEVICE;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&c->nccl, (int)nranks, u, (int)rank) != ncclSuccess) {
        (void)hipStreamDestroy(c->stream);
        return TM_EDEVICE;
    }
    *out = c.release();
    return TM_OK;
}

int tm_comm_init_all(const int32_t* devices, uint32_t n, tm_comm** comms) {
    if (!devices || !comms || n == 0 || n > 64) return TM_EINVAL;
    bool distinct = true;
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = 0; j < i; ++j) distinct = distinct && devices[i] != devices[j];
    std::vector<ncclComm_t> nc(n, nullptr);
    if (distinct && n > 1 && ncclCommInitAll(nc.data(), (int)n, devices) != ncclSuccess) return TM_EDEVICE;
    for (uint32_t i = 0; i < n; ++i) {
        tm_comm* c = new (std::nothrow) tm_comm();
        if (!c || hipSetDevice(devices[i]) != hipSuccess ||
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
            delete c;
            for (uint32_t j = 0; j < i; ++j) tm_comm_destroy(comms[j]);
            for (uint32_t j = i; j < n; ++j)
                if (nc[j]) (void)ncclCommDestroy(nc[j]);
            return TM_EDEVICE;
        }
        c->device = devices[i];
        c->nranks = n;
        c->rank = i;
        c->nccl = distinct && n > 1 ? nc[i] : nullptr;   // shared GPU (or one rank): device copies
        comms[i] = c;
    }
    return TM_OK;
}

void tm_comm_destroy(tm_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    for (Buf* b : {&c->sizes, &c->rsizes, &c->recv_counts, &c->src_base, &c->recv_ids, &c->recv_keys}) b->release();
    tm_comm::Route& r = c->rt;
    for (Buf* b : {&r.owner, &r.blk_cnt, &r.blk_base, &r.bucket, &r.perm, &r.slen, &r.soff, &r.scan_tmp, &r.sbuf,
                   &r.cuts, &r.rlen, &r.rbuf, &r.roff, &r.rscan, &r.seg_idx, &r.seg_cut, &r.ret_sz, &r.ret_rsz,
                   &r.rcount, &r.rids, &r.rroff, &r.out_count, &r.out_off, &r.out_ids, &r.out_total, &r.uscan})
        b->release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int tm_comm_uses_rccl(tm_comm* c) { return c && c->nccl ? 1 : 0; }
int tm_comm_set_self_rccl(tm_comm* c, int on) {
    if (!c || !c->nccl) return TM_EINVAL;
    c->self_rccl = on != 0;
    return TM_OK;
}
const char* tm_comm_last_error(tm_comm* c) { return c ? c->last_error.c_str() : "null comm"; }

// one rank of a multi-process (or one-rank) RCCL exchange
int tm_shard_exchange(tm_comm* c, const tm_exchange_in* in, tm_exchange_out* out) {
    if (!c || !in || !out || !valid_in(*in)) return TM_EINVAL;
    if (c->aborted) return fail(c, "communicator aborted after a failed RCCL group");
    if (!c->nccl) return fail(c, "tm_shard_exchange needs an RCCL communicator (use tm_shard_exchange_group)",
                              TM_EINVAL);
    if (hipSetDevice(c->device) != hipSuccess) return TM_EDEVICE;
    const uint32_t S = c->nranks, me = c->rank, n = in->n;
    hipStream_t st = stream_of(c, *in);
    int rc = send_sizes(c, *in);
    if (rc != TM_OK) return rc;
    const uint32_t m = slice_lo(n, S, me + 1) - slice_lo(n, S, me);
    if (!c->recv_counts.ensure((size_t)S * m * 4 + 4)) return fail(c, "hipMalloc", TM_ENOMEM);
    // counts of slice p -> rank p, and the id count of each slice (all-to-all of one u64)
    XGROUP_START(c, std::vector<tm_comm*>{c});
    // (a rank's own slice is a device copy: RCCL's send to self is slower)
    for (uint32_t p = 0; p < S; ++p) {
        const uint32_t lo = slice_lo(n, S, p), mp = slice_lo(n, S, p + 1) - lo;
        if (p == me && !c->self_rccl) {
            XHIP(c, hipMemcpyAsync(c->recv_counts.as<uint32_t>() + (size_t)p * m, in->d_counts + lo, (size_t)mp * 4,
                                   hipMemcpyDeviceToDevice, st));
            continue;
        }
        XNCCL(c, ncclSend(in->d_counts + lo, mp, ncclUint32, (int)p, c->nccl, st));
        XNCCL(c, ncclRecv(c->recv_counts.as<uint32_t>() + (size_t)p * m, m, ncclUint32, (int)p, c->nccl, st));
    }
    XNCCL(c, ncclAllToAll(c->sizes.p, c->rsizes.p, 1, ncclUint64, c->nccl, st));
    XGROUP_END(c);
    c->h_recv.resize(S);
    XHIP(c, hipMemcpyAsync(c->h_recv.data(), c->rsizes.p, S * 8, hipMemcpyDeviceToHost, st));
    XHIP(c, hipStreamSynchronize(st));
    rc = alloc_recv(c, *in, *out);
    if (rc != TM_OK) return rc;
    // ids, then each key plane: slice p -> rank p
    XGROUP_START(c, std::vector<tm_comm*>{c});
    uint64_t base = 0;
    for (uint32_t p = 0; p < S; ++p) {
        const uint64_t items = c->h_send[p], from = c->h_send[S + p], ritems = c->h_recv[p];
        if (p == me && !c->self_rccl) {
            XHIP(c, hipMemcpyAsync(c->recv_ids.as<uint32_t>() + base, in->d_ids + from, items * 4,
                                   hipMemcpyDeviceToDevice, st));
            for (uint32_t j = 0; j < in->key_words; ++j)
                XHIP(c, hipMemcpyAsync(c->recv_keys.as<uint64_t>() + j * out->total + base,
                                       in->d_keys + j * in->key_stride + from, items * 8, hipMemcpyDeviceToDevice, st));
            base += ritems;
            continue;
        }
        XNCCL(c, ncclSend(in->d_ids + from, items, ncclUint32, (int)p, c->nccl, st));
        XNCCL(c, ncclRecv(c->recv_ids.as<uint32_t>() + base, ritems, ncclUint32, (int)p, c->nccl, st));
        for (uint32_t j = 0; j < in->key_words; ++j) {
            XNCCL(c, ncclSend(in->d_keys + j * in->key_stride + from, items, ncclUint64, (int)p, c->nccl, st));
            XNCCL(c, ncclRecv(c->recv_keys.as<uint64_t>() + j * out->total + base, ritems, ncclUint64, (int)p,
                              c->nccl, st));
        }
        base += ritems;
    }
    XGROUP_END(c);
    return TM_OK;
}

// every rank of one process at once: RCCL group calls across the ranks'
// communicators, or device copies when ranks share a GPU
int tm_shard_exchange_group(tm_comm** comms, uint32_t S, const tm_exchange_in* ins, tm_exchange_out* outs) {
    if (!comms || !ins || !outs || S == 0) return TM_EINVAL;
    for (uint32_t r = 0; r < S; ++r)
        if (!comms[r] || comms[r]->nranks != S || comms[r]->rank != r || !valid_in(ins[r]) || ins[r].n != ins[0].n ||
            ins[r].key_words != ins[0].key_words)
            return TM_EINVAL;
    // a group whose communicators were aborted stays failed: it must not fall
    // back to device copies (comm->nccl is null after an abort)
    for (uint32_t r = 0; r < S; ++r)
        if (comms[r]->aborted) return fail(comms[r], "communicator aborted after a failed RCCL group");
    const uint32_t n = ins[0].n;
    const bool rccl = comms[0]->nccl != nullptr;
    for (uint32_t r = 0; r < S; ++r) {   // sizes of every rank's sends, on the host
        if (hipSetDevice(comms[r]->device) != hipSuccess) return TM_EDEVICE;
        int rc = send_sizes(comms[r], ins[r]);
        if (rc != TM_OK) return rc;
    }
    for (uint32_t d = 0; d < S; ++d) {
        tm_comm* c = comms[d];
        c->h_recv.resize(S);
        for (uint32_t s = 0; s < S; ++s) c->h_recv[s] = comms[s]->h_send[d];
        if (hipSetDevice(c->device) != hipSuccess) return TM_EDEVICE;
        int rc = alloc_recv(c, ins[d], outs[d]);
        if (rc != TM_OK) return rc;
    }
    const std::vector<tm_comm*> group(comms, comms + S);
    if (rccl) XGROUP_START(comms[0], group);
    for (uint32_t d = 0; d < S; ++d) {
        tm_comm* c = comms[d];
        hipStream_t st = stream_of(c, ins[d]);
        if (hipSetDevice(c->device) != hipSuccess) return fail(c, "hipSetDevice");
        const uint32_t m = outs[d].m;
        uint64_t base = 0;
        for (uint32_t s = 0; s < S; ++s) {
            const tm_exchange_in& src = ins[s];
            const uint32_t lo = slice_lo(n, S, d);
            const uint64_t items = comms[s]->h_send[d], from = comms[s]->h_send[S + d];
            if (rccl) {   // rank d receives from s; rank s's send is issued in its own turn below
                XNCCL(c, ncclRecv(c->recv_counts.as<uint32_t>() + (size_t)s * m, m, ncclUint32, (int)s, c->nccl, st));
                XNCCL(c, ncclRecv(c->recv_ids.as<uint32_t>() + base, items, ncclUint32, (int)s, c->nccl, st));
                for (uint32_t j = 0; j < src.key_words; ++j)
                    XNCCL(c, ncclRecv(c->recv_keys.as<uint64_t>() + j * outs[d].total + base, items, ncclUint64,
                                      (int)s, c->nccl, st));
            } else {      // device copies (the ranks share a GPU, or S = 1)
                XHIP(c, hipMemcpyPeerAsync(c->recv_counts.as<uint32_t>() + (size_t)s * m, c->device, src.d_counts + lo,
                                           comms[s]->device, (size_t)m * 4, st));
                if (items) {
                    XHIP(c, hipMemcpyPeerAsync(c->recv_ids.as<uint32_t>() + base, c->device, src.d_ids + from,
                                               comms[s]->device, items * 4, st));
                    for (uint32_t j = 0; j < src.key_words; ++j)
                        XHIP(c, hipMemcpyPeerAsync(c->recv_keys.as<uint64_t>() + j * outs[d].total + base, c->device,
                                                   src.d_keys + j * src.key_stride + from, comms[s]->device, items * 8,
                                                   st));
                }
            }
            base += items;
        }
        if (rccl) {       // rank d's sends: slice p of its lists -> rank p
            const tm_exchange_in& in = ins[d];
            for (uint32_t p = 0; p < S; ++p) {
                const uint32_t lo = slice_lo(n, S, p), mp = slice_lo(n, S, p + 1) - lo;
                const uint64_t items = c->h_send[p], from = c->h_send[S + p];
                XNCCL(c, ncclSend(in.d_counts + lo, mp, ncclUint32, (int)p, c->nccl, st));
                XNCCL(c, ncclSend(in.d_ids + from, items, ncclUint32, (int)p, c->nccl, st));
                for (uint32_t j = 0; j < in.key_words; ++j)
                    XNCCL(c, ncclSend(in.d_keys + j * in.key_stride + from, items, ncclUint64, (int)p, c->nccl, st));
            }
        }
    }
    if (rccl) XGROUP_END(comms[0]);
    return TM_OK;
}

// ---- routed mode: the topic exchange ------------------------------------------
// One rank of a multi-process (or one-rank) exchange over RCCL.
int tm_route_exchange(tm_comm* c, const tm_route_in* in, tm_route_out* out) {
    if (!c || !in || !out || (in->n && (!in->d_bytes || !in->d_off)) || in->depth == 0) return TM_EINVAL;
    if (c->aborted) return fail(c, "communicator aborted after a failed RCCL group");
    const uint32_t S = c->nranks, me = c->rank;
    if (S > MAX_ROUTE_SHARDS) return TM_EINVAL;
    if (S > 1 && !c->nccl) return fail(c, "tm_route_exchange needs an RCCL communicator (use the _group form)", TM_EINVAL);
    if (hipSetDevice(c->device) != hipSuccess) return TM_EDEVICE;
    hipStream_t st = route_stream(c, in->hip_stream);
    int rc = route_plan(c, *in);
    if (rc != TM_OK) return rc;
    tm_comm::Route& r = c->rt;
    // [topics, bytes] per peer: an all-to-all of two u64
    if (!c->sizes.ensure(2 * S * 8) || !c->rsizes.ensure(2 * S * 8)) return fail(c, "hipMalloc", TM_ENOMEM);
    XHIP(c, hipMemcpyAsync(c->sizes.p, r.h_sz.data(), 2 * S * 8, hipMemcpyHostToDevice, st));
    const bool over_rccl = S > 1 || c->self_rccl;
    if (over_rccl) {
        XGROUP_START(c, std::vector<tm_comm*>{c});
        XNCCL(c, ncclAllToAll(c->sizes.p, c->rsizes.p, 2, ncclUint64, c->nccl, st));
        XGROUP_END(c);
    } else {
        XHIP(c, hipMemcpyAsync(c->rsizes.p, c->sizes.p, 16, hipMemcpyDeviceToDevice, st));
    }
    r.h_rsz.resize(2 * S);
    XHIP(c, hipMemcpyAsync(r.h_rsz.data(), c->rsizes.p, 2 * S * 8, hipMemcpyDeviceToHost, st));
    XHIP(c, hipStreamSynchronize(st));
    rc = route_alloc_recv(c);
    if (rc != TM_OK) return rc;
    std::vector<Xfer> run;
    for (uint32_t p = 0; p < S; ++p) {   // my bucket p -> rank p; rank p's bucket me -> me
        if (p == me) {
            run.push_back(Xfer{me, me, r.slen.as<uint32_t>() + r.h_bucket[me], r.rlen.as<uint32_t>() + r.rt_base[me],
                               r.h_sz[2 * me] * 4});
            run.push_back(Xfer{me, me, r.sbuf.as<uint8_t>() + r.h_cuts[me], r.rbuf.as<uint8_t>() + r.rb_base[me],
                               r.h_sz[2 * me + 1]});
            continue;
        }
        run.push_back(Xfer{me, p, r.slen.as<uint32_t>() + r.h_bucket[p], nullptr, r.h_sz[2 * p] * 4});
        run.push_back(Xfer{me, p, r.sbuf.as<uint8_t>() + r.h_cuts[p], nullptr, r.h_sz[2 * p + 1]});
        run.push_back(Xfer{p, me, nullptr, r.rlen.as<uint32_t>() + r.rt_base[p], r.h_rsz[2 * p] * 4});
        run.push_back(Xfer{p, me, nullptr, r.rbuf.as<uint8_t>() + r.rb_base[p], r.h_rsz[2 * p + 1]});
    }
    rc = run_xfers(&c, 1, run, {st}, over_rccl);
    if (rc != TM_OK) return rc;
    return route_finish(c, st, out);
}

// All S ranks of one process at once (comms from tm_comm_init_all): RCCL
// group calls across their communicators, or device copies when they share a GPU.
int tm_route_exchange_group(tm_comm** comms, uint32_t S, const tm_route_in* ins, tm_route_out* outs) {
    if (!comms || !ins || !outs || S == 0 || S > MAX_ROUTE_SHARDS) return TM_EINVAL;
    for (uint32_t r = 0; r < S; ++r) {
        if (!comms[r] || comms[r]->nranks != S || comms[r]->rank != r || ins[r].depth != ins[0].depth ||
            ins[r].depth == 0 || (ins[r].n && (!ins[r].d_bytes || !ins[r].d_off)))
            return TM_EINVAL;
        if (comms[r]->aborted) return fail(comms[r], "communicator aborted after a failed RCCL group");
    }
    const bool rccl = comms[0]->nccl != nullptr;
    std::vector<hipStream_t> st(S);
    for (uint32_t r = 0; r < S; ++r) {
        if (hipSetDevice(comms[r]->device) != hipSuccess) return TM_EDEVICE;
        st[r] = route_stream(comms[r], ins[r].hip_stream);
        int rc = route_plan(comms[r], ins[r]);
        if (rc != TM_OK) return rc;
    }
    for (uint32_t d = 0; d < S; ++d) {   // sizes are on every rank's host already
        tm_comm::Route& r = comms[d]->rt;
        r.h_rsz.resize(2 * S);
        for (uint32_t s = 0; s < S; ++s) {
            r.h_rsz[2 * s] = comms[s]->rt.h_sz[2 * d];
            r.h_rsz[2 * s + 1] = comms[s]->rt.h_sz[2 * d + 1];
        }
        if (hipSetDevice(comms[d]->device) != hipSuccess) return TM_EDEVICE;
        int rc = route_alloc_recv(comms[d]);
        if (rc != TM_OK) return rc;
    }
    std::vector<Xfer> xs;
    for (uint32_t s = 0; s < S; ++s)
        for (uint32_t d = 0; d < S; ++d) {
            tm_comm::Route &a = comms[s]->rt, &b = comms[d]->rt;
            xs.push_back(Xfer{s, d, a.slen.as<uint32_t>() + a.h_bucket[d], b.rlen.as<uint32_t>() + b.rt_base[s],
                              a.h_sz[2 * d] * 4});
            xs.push_back(Xfer{s, d, a.sbuf.as<uint8_t>() + a.h_cuts[d], b.rbuf.as<uint8_t>() + b.rb_base[s],
                              a.h_sz[2 * d + 1]});
        }
    int rc = run_xfers(comms, S, xs, st, rccl);
    if (rc != TM_OK) return rc;
    for (uint32_t d = 0; d < S; ++d) {
        if (hipSetDevice(comms[d]->device) != hipSuccess) return TM_EDEVICE;
        rc = route_finish(comms[d], st[d], &outs[d]);
        if (rc != TM_OK) return rc;
    }
    return TM_OK;
}

// ---- routed mode: the lists back to their sources ------------------------------
int tm_route_return(tm_comm* c, const tm_route_lists* l, tm_route_result* res) {
    if (!c || !l || !res || !l->d_offs || (c->rt.m && !l->d_counts)) return TM_EINVAL;
    if (c->aborted) return fail(c, "communicator aborted after a failed RCCL group");
    const uint32_t S = c->nranks, me = c->rank;
    if (S > 1 && !c->nccl) return fail(c, "tm_route_return needs an RCCL communicator (use the _group form)", TM_EINVAL);
    if (hipSetDevice(c->device) != hipSuccess) return TM_EDEVICE;
    hipStream_t st = route_stream(c, l->hip_stream);
    tm_comm::Route& r = c->rt;
    int rc = return_cuts(c, *l);
    if (rc != TM_OK) return rc;
    // ids per source -> all-to-all of one u64
    std::vector<uint64_t> send(S);
    for (uint32_t s = 0; s < S; ++s) send[s] = r.h_seg_cut[s + 1] - r.h_seg_cut[s];
    if (!r.ret_sz.ensure(S * 8) || !r.ret_rsz.ensure(S * 8)) return fail(c, "hipMalloc", TM_ENOMEM);
    XHIP(c, hipMemcpyAsync(r.ret_sz.p, send.data(), S * 8, hipMemcpyHostToDevice, st));
    const bool over_rccl = S > 1 || c->self_rccl;
    if (over_rccl) {
        XGROUP_START(c, std::vector<tm_comm*>{c});
        XNCCL(c, ncclAllToAll(r.ret_sz.p, r.ret_rsz.p, 1, ncclUint64, c->nccl, st));
        XGROUP_END(c);
    } else {
        XHIP(c, hipMemcpyAsync(r.ret_rsz.p, r.ret_sz.p, 8, hipMemcpyDeviceToDevice, st));
    }
    r.h_ret.resize(S);
    XHIP(c, hipMemcpyAsync(r.h_ret.data(), r.ret_rsz.p, S * 8, hipMemcpyDeviceToHost, st));
    XHIP(c, hipStreamSynchronize(st));
    rc = return_alloc(c);
    if (rc != TM_OK) return rc;
    std::vector<uint64_t> ret_base(S + 1, 0);
    for (uint32_t o = 0; o < S; ++o) ret_base[o + 1] = ret_base[o] + r.h_ret[o];
    std::vector<Xfer> xs;
    for (uint32_t p = 0; p < S; ++p) {
        // the counts and ids of the topics rank p sent me -> p
        const Xfer cnt_out{me, p, l->d_counts + r.rt_base[p], nullptr, (r.rt_base[p + 1] - r.rt_base[p]) * 4};
        const Xfer ids_out{me, p, l->d_ids + r.h_seg_cut[p], nullptr, send[p] * 4};
        // what owner p returns for my bucket p
        const Xfer cnt_in{p, me, nullptr, r.rcount.as<uint32_t>() + r.h_bucket[p], r.h_sz[2 * p] * 4};
        const Xfer ids_in{p, me, nullptr, r.rids.as<uint32_t>() + ret_base[p], r.h_ret[p] * 4};
        if (p == me) {
            xs.push_back(Xfer{me, me, cnt_out.sp, cnt_in.dp, cnt_out.bytes});
            xs.push_back(Xfer{me, me, ids_out.sp, ids_in.dp, ids_out.bytes});
        } else {
            xs.insert(xs.end(), {cnt_out, ids_out, cnt_in, ids_in});
        }
    }
    rc = run_xfers(&c, 1, xs, {st}, over_rccl);
    if (rc != TM_OK) return rc;
    return return_finish(c, st, res);
}

int tm_route_return_group(tm_comm** comms, uint32_t S, const tm_route_lists* ls, tm_route_result* res) {
    if (!comms || !ls || !res || S == 0 || S > MAX_ROUTE_SHARDS) return TM_EINVAL;
    for (uint32_t r = 0; r < S; ++r) {
        if (!comms[r] || comms[r]->nranks != S || comms[r]->rank != r || !ls[r].d_offs ||
            (comms[r]->rt.m && !ls[r].d_counts))
            return TM_EINVAL;
        if (comms[r]->aborted) return fail(comms[r], "communicator aborted after a failed RCCL group");
    }
    const bool rccl = comms[0]->nccl != nullptr;
    std::vector<hipStream_t> st(S);
    for (uint32_t r = 0; r < S; ++r) {
        if (hipSetDevice(comms[r]->device) != hipSuccess) return TM_EDEVICE;
        st[r] = route_stream(comms[r], ls[r].hip_stream);
        int rc = return_cuts(comms[r], ls[r]);
        if (rc != TM_OK) return rc;
    }
    for (uint32_t o = 0; o < S; ++o) {   // source o receives from every owner d its segment o
        tm_comm::Route& r = comms[o]->rt;
        r.h_ret.resize(S);
        for (uint32_t d = 0; d < S; ++d) r.h_ret[d] = comms[d]->rt.h_seg_cut[o + 1] - comms[d]->rt.h_seg_cut[o];
        if (hipSetDevice(comms[o]->device) != hipSuccess) return TM_EDEVICE;
        int rc = return_alloc(comms[o]);
        if (rc != TM_OK) return rc;
    }
    std::vector<Xfer> xs;
    for (uint32_t d = 0; d < S; ++d) {       // owner d
        tm_comm::Route& a = comms[d]->rt;
        for (uint32_t s = 0; s < S; ++s) {   // -> source s
            tm_comm::Route& b = comms[s]->rt;
            uint64_t ret_base = 0;
            for (uint32_t q = 0; q < d; ++q) ret_base += b.h_ret[q];
            xs.push_back(Xfer{d, s, ls[d].d_counts + a.rt_base[s], b.rcount.as<uint32_t>() + b.h_bucket[d],
                              (a.rt_base[s + 1] - a.rt_base[s]) * 4});
            xs.push_back(Xfer{d, s, ls[d].d_ids + a.h_seg_cut[s], b.rids.as<uint32_t>() + ret_base,
                              (a.h_seg_cut[s + 1] - a.h_seg_cut[s]) * 4});
        }
    }
    int rc = run_xfers(comms, S, xs, st, rccl);
    if (rc != TM_OK) return rc;
    for (uint32_t s = 0; s < S; ++s) {
        if (hipSetDevice(comms[s]->device) != hipSuccess) return TM_EDEVICE;
        rc = return_finish(comms[s], st[s], &res[s]);
        if (rc != TM_OK) return rc;
    }
    return TM_OK;
}

}  // extern "C"
