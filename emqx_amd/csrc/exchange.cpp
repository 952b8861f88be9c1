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
    hipStream_t stream = nullptr;
    Buf sizes;                    // 2S u64: send counts per destination, then their first ids
    Buf rsizes;                   // S u64: ids to receive from each source
    Buf recv_counts, src_base, recv_ids, recv_keys;
    std::vector<uint64_t> h_send, h_recv, h_base;   // h_base: source of the async src_base upload
    std::string last_error;
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
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int tm_comm_uses_rccl(tm_comm* c) { return c && c->nccl ? 1 : 0; }
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
        if (p == me) {
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
        if (p == me) {
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

}  // extern "C"
