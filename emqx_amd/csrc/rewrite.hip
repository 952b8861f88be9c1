// rewrite.hip — batched topic-rewrite rule selection on the device (SURVEY
// §8f-4, second caller of emqx_topic:match/2).
//
// emqx_mod_rewrite (src/emqx_mod_rewrite.erl:52-59) runs on every publish
// ('message.publish' hook) and subscribe:
//
//   match_rule(Topic, []) -> Topic;
//   match_rule(Topic, [{rewrite, Filter, MP, Dest} | Rules]) ->
//       case emqx_topic:match(Topic, Filter) of
//           true  -> match_regx(Topic, MP, Dest);
//           false -> match_rule(Topic, Rules)
//       end.
//
// The FIRST rule whose filter matches decides (a regex miss there leaves the
// topic unchanged; later rules are not tried), so the device part is: per
// topic, the index of the first rule with emqx_topic:match(Topic, Filter).
// The regex capture and substitution (re:run / re:replace) of that one rule
// stay with the caller.  match/2 here is the BINARY clause pair
// (src/emqx_topic.erl:56-61): a name starting with byte '$' never matches a
// filter starting with byte '+' or '#'; otherwise the word-list clauses
// (:62-75) on words/1 of both.
//
// One lane per topic; the rules (filters in one byte arena, a few KB) are
// read through the caches.
#include <hip/hip_runtime.h>

#include <mutex>
#include <new>
#include <vector>

#include "../../include/topicmatch.h"

namespace {

constexpr int RW_BLOCK = 256;

// next level [b, e) of bytes [pos, end); false when the list is exhausted
struct Cur {
    uint64_t pos, end;
    bool done;
};
__device__ __forceinline__ bool next_level(const uint8_t* s, Cur& c, uint64_t& b, uint64_t& e) {
    if (c.done) return false;
    uint64_t q = c.pos;
    while (q < c.end && s[q] != '/') ++q;
    b = c.pos;
    e = q;
    if (q < c.end) c.pos = q + 1;
    else c.done = true;
    return true;
}

// emqx_topic:match/2, binary/binary (src/emqx_topic.erl:56-75)
__device__ bool topic_match(const uint8_t* t, uint64_t tb, uint64_t te, const uint8_t* f, uint64_t fb,
                            uint64_t fe) {
    if (te > tb && t[tb] == '$' && fe > fb && (f[fb] == '+' || f[fb] == '#')) return false;
    Cur ct{tb, te, false}, cf{fb, fe, false};
    uint64_t ab = 0, ae = 0, bb = 0, be = 0;
    bool ha = next_level(t, ct, ab, ae), hb = next_level(f, cf, bb, be);
    for (;;) {
        if (!ha && !hb) return true;                                        // match([], [])
        if (ha && hb) {
            const uint64_t n = ae - ab;
            bool eq = n == be - bb;                                         // match([H|T1], [H|T2])
            for (uint64_t i = 0; eq && i < n; ++i) eq = t[ab + i] == f[bb + i];
            if (eq || (be - bb == 1 && f[bb] == '+')) {                     // match([_|T1], ['+'|T2])
                ha = next_level(t, ct, ab, ae);
                hb = next_level(f, cf, bb, be);
                continue;
            }
        }
        // match(_, ['#']): the filter's last word is '#'
        if (hb && be - bb == 1 && f[bb] == '#') {
            uint64_t x, y;
            return !next_level(f, cf, x, y);
        }
        return false;
    }
}

__global__ void __launch_bounds__(RW_BLOCK)
tm_rewrite_match(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ roff, uint32_t nrules,
                 const uint8_t* __restrict__ topics, const uint64_t* __restrict__ toff, uint32_t n,
                 uint32_t* __restrict__ out_rule) {
    const uint32_t i = blockIdx.x * RW_BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t tb = toff[i], te = toff[i + 1];   // topic i = topics[toff[i] .. toff[i+1])
    uint32_t which = TM_NO_RULE;
    for (uint32_t r = 0; r < nrules; ++r)
        if (topic_match(topics, tb, te, arena, roff[r], roff[r + 1])) {
            which = r;
            break;
        }
    out_rule[i] = which;
}

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    bool ensure(size_t need) {
        if (need <= bytes && p) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, need ? need : 16) != hipSuccess) return false;
        bytes = need ? need : 16;
        return true;
    }
    ~Buf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct tm_rewrite {
    std::mutex mu;
    int device = -1;
    hipStream_t stream = nullptr;
    std::vector<uint8_t> arena;
    std::vector<uint64_t> off{0};
    bool dirty = true;
    Buf d_arena, d_off;                 // the rules on the device
    Buf w_topics, w_toff, w_out;        // host-buffer batches: reused workspace
};

extern "C" {

int tm_rewrite_open(int device, tm_rewrite** out) {
    if (!out) return TM_EINVAL;
    *out = nullptr;
    tm_rewrite* r = new (std::nothrow) tm_rewrite();
    if (!r) return TM_ENOMEM;
    if (device >= 0) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev || hipSetDevice(device) != hipSuccess ||
            hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
            delete r;
            return TM_EDEVICE;
        }
    }
    r->device = device;
    *out = r;
    return TM_OK;
}

void tm_rewrite_close(tm_rewrite* r) {
    if (!r) return;
    if (r->stream) {
        (void)hipSetDevice(r->device);
        (void)hipStreamSynchronize(r->stream);
        (void)hipStreamDestroy(r->stream);
    }
    delete r;
}

int tm_rewrite_rule(tm_rewrite* r, const uint8_t* filter, uint32_t len) {
    if (!r || (len && !filter)) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(r->mu);
    r->arena.insert(r->arena.end(), filter, filter + len);
    r->off.push_back(r->arena.size());
    r->dirty = true;
    return TM_OK;
}

int tm_rewrite_rule_count(tm_rewrite* r) { return r ? (int)r->off.size() - 1 : 0; }

static int rewrite_launch(tm_rewrite* r, const uint8_t* d_topics, const uint64_t* d_off, uint32_t n,
                          uint32_t* d_out, hipStream_t st) {
    if (r->dirty) {
        if (!r->d_arena.ensure(r->arena.size()) || !r->d_off.ensure(r->off.size() * 8)) return TM_ENOMEM;
        if ((!r->arena.empty() && hipMemcpy(r->d_arena.p, r->arena.data(), r->arena.size(), hipMemcpyHostToDevice) !=
                                      hipSuccess) ||
            hipMemcpy(r->d_off.p, r->off.data(), r->off.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
            return TM_EDEVICE;
        r->dirty = false;
    }
    hipLaunchKernelGGL(tm_rewrite_match, dim3((n + RW_BLOCK - 1) / RW_BLOCK), dim3(RW_BLOCK), 0, st,
                       (const uint8_t*)r->d_arena.p, (const uint64_t*)r->d_off.p, (uint32_t)(r->off.size() - 1),
                       d_topics, d_off, n, d_out);
    return hipGetLastError() == hipSuccess ? TM_OK : TM_EDEVICE;
}

int tm_rewrite_match_batch_device(tm_rewrite* r, const uint8_t* d_topics, const uint64_t* d_off, uint32_t n,
                                  uint32_t* d_out_rule, void* hip_stream) {
    if (!r || (n && (!d_off || !d_out_rule))) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(r->mu);
    if (r->device < 0) return TM_EDEVICE;   // the rule scan runs on the GPU only
    if (n == 0) return TM_OK;
    if (hipSetDevice(r->device) != hipSuccess) return TM_EDEVICE;
    return rewrite_launch(r, d_topics, d_off, n, d_out_rule, hip_stream ? (hipStream_t)hip_stream : r->stream);
}

int tm_rewrite_match_batch(tm_rewrite* r, const uint8_t* topics, const uint64_t* topic_off, uint32_t n,
                           uint32_t* out_rule) {
    if (!r || (n && (!topic_off || !out_rule))) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(r->mu);
    if (r->device < 0) return TM_EDEVICE;
    if (n == 0) return TM_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (topic_off[i + 1] < topic_off[i]) return TM_EINVAL;
    const uint64_t nb = topic_off[n] - topic_off[0];
    if (nb && !topics) return TM_EINVAL;
    if (hipSetDevice(r->device) != hipSuccess) return TM_EDEVICE;
    if (!r->w_topics.ensure(nb + 8) || !r->w_toff.ensure((n + 1) * 8ull) || !r->w_out.ensure(n * 4ull))
        return TM_ENOMEM;
    hipStream_t st = r->stream;
    std::vector<uint64_t> rel(topic_off, topic_off + n + 1);
    for (auto& x : rel) x -= topic_off[0];
    if ((nb && hipMemcpyAsync(r->w_topics.p, topics + topic_off[0], nb, hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemcpyAsync(r->w_toff.p, rel.data(), (n + 1) * 8ull, hipMemcpyHostToDevice, st) != hipSuccess)
        return TM_EDEVICE;
    int rc = rewrite_launch(r, (const uint8_t*)r->w_topics.p, (const uint64_t*)r->w_toff.p, n, (uint32_t*)r->w_out.p,
                            st);
    if (rc != TM_OK) return rc;
    if (hipMemcpyAsync(out_rule, r->w_out.p, n * 4ull, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return TM_EDEVICE;
    return TM_OK;
}

}  // extern "C"
