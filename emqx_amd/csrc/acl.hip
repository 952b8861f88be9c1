// acl.hip — batched ACL checks on the device.
//
// The internal ACL module evaluates, per (credentials, publish|subscribe,
// topic), the compiled rules of that access type in order and returns the
// first match (emqx_acl_internal:check_acl/2 and match/3,
// src/emqx_acl_internal.erl:63-87, rules filtered by access at :47-61).  A
// rule matches when its "who" matches the credentials and one of its topic
// filters matches the topic (emqx_access_rule:match/3, :82-135):
//   plain filter   emqx_topic:match(words(Topic), Words)   (word lists: no '$' rule)
//   {eq, Topic}    words(Topic) == Words
//   pattern        feed_var/3 substitutes %c / %u (:136-149), then match/2
// Term identity is kept: the topic levels "", "+", "#" are the atoms '', '+',
// '#' (emqx_topic:words/1), a substituted client id or username is a binary
// even when its bytes are "+", so it never acts as a wildcard.
//
// One lane per check; rules, filters and words are a few KB, read through the
// caches.  Host side: a rule builder mirroring emqx_access_rule:compile/1.
#include <hip/hip_runtime.h>
#include <arpa/inet.h>

#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/topicmatch.h"

namespace {

// filter word kinds
enum : uint32_t { W_BIN = 0, W_EMPTY = 1, W_PLUS = 2, W_HASH = 3, W_PCT_C = 4, W_PCT_U = 5 };
// filter kinds
enum : uint32_t { F_PLAIN = 0, F_EQ = 1, F_PATTERN = 2 };
// who nodes (postfix)
enum : uint32_t { H_ALL = 0, H_CLIENT = 1, H_USER = 2, H_IPADDR = 3, H_AND = 4, H_OR = 5, H_FALSE = 6 };

struct AclWord {
    uint32_t kind, len;
    uint64_t off;       // bytes in the arena (W_BIN)
};
struct AclFilter {
    uint32_t kind, wbeg, wend, pad;
};
struct AclWho {
    uint32_t kind, n;   // n: child count (AND/OR), prefix bits (IPADDR), arg length (CLIENT/USER)
    uint32_t family, pad;
    uint64_t off;       // arg bytes (CLIENT/USER)
    uint8_t addr[16];   // IPADDR network (masked)
};
struct AclRule {
    int32_t allow;      // 1 allow, 0 deny
    uint32_t access;    // bit 0 publish, bit 1 subscribe
    uint32_t hbeg, hend, fbeg, fend;   // who nodes / filters; {A, all}: hbeg == hend && fbeg == fend, all = 1
    uint32_t all, pad;
};

struct AclView {
    const AclRule* rules;
    uint32_t nrules;
    const AclFilter* filters;
    const AclWord* words;
    const AclWho* who;
    const uint8_t* arena;
};

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// one level of a topic: [b, e)
struct Level {
    uint64_t b, e;
};
__device__ __forceinline__ bool next_level(const uint8_t* t, uint64_t end, uint64_t& pos, bool& done, Level& lv) {
    if (done) return false;
    uint64_t q = pos;
    while (q < end && t[q] != '/') ++q;
    lv.b = pos;
    lv.e = q;
    if (q < end) pos = q + 1;
    else done = true;
    return true;
}
__device__ __forceinline__ bool level_atomic(const uint8_t* t, const Level& lv) {   // '' / '+' / '#'
    const uint64_t n = lv.e - lv.b;
    return n == 0 || (n == 1 && (t[lv.b] == '+' || t[lv.b] == '#'));
}

// word equality as Erlang terms: topic level (atom or binary) vs filter word
__device__ bool word_eq(const AclView& v, const uint8_t* t, const Level& lv, const AclWord& w, const uint8_t* cid,
                        uint32_t cid_len, bool cid_def, const uint8_t* usr, uint32_t usr_len, bool usr_def) {
    const uint32_t n = (uint32_t)(lv.e - lv.b);
    const uint8_t* p = t + lv.b;
    switch (w.kind) {
        case W_EMPTY: return n == 0;
        case W_PLUS: return n == 1 && p[0] == '+';
        case W_HASH: return n == 1 && p[0] == '#';
        case W_BIN: return n == w.len && bytes_eq(p, v.arena + w.off, n);   // bytes never atomic
        default: {
            // feed_var: the credential (a binary), or the literal word when undefined
            const bool c = w.kind == W_PCT_C;
            const bool def = c ? cid_def : usr_def;
            const uint8_t* s = def ? (c ? cid : usr) : (const uint8_t*)(c ? "%c" : "%u");
            const uint32_t sl = def ? (c ? cid_len : usr_len) : 2u;
            return !level_atomic(t, lv) && n == sl && bytes_eq(p, s, n);
        }
    }
}

__device__ bool filter_match(const AclView& v, const AclFilter& f, const uint8_t* t, uint64_t tb, uint64_t te,
                             const uint8_t* cid, uint32_t cid_len, bool cid_def, const uint8_t* usr, uint32_t usr_len,
                             bool usr_def) {
    uint64_t pos = tb;
    bool done = false;
    Level lv;
    bool have = next_level(t, te, pos, done, lv);
    for (uint32_t j = f.wbeg;; ++j) {
        const bool f_end = j == f.wend;
        if (!have && f_end) return true;                                   // match([], [])
        if (f.kind == F_EQ) {                                             // Topic == Words
            if (!have || f_end || !word_eq(v, t, lv, v.words[j], cid, cid_len, cid_def, usr, usr_len, usr_def))
                return false;
        } else {
            if (f_end) return false;                                      // match([_|_], [])
            const AclWord& w = v.words[j];
            if (have && word_eq(v, t, lv, w, cid, cid_len, cid_def, usr, usr_len, usr_def)) {
                // match([H|T1], [H|T2])
            } else if (have && w.kind == W_PLUS) {
                // match([_|T1], ['+'|T2])
            } else {
                return w.kind == W_HASH && j + 1 == f.wend;               // match(_, ['#'])
            }
        }
        have = next_level(t, te, pos, done, lv);
    }
}

__device__ bool who_match(const AclView& v, uint32_t hb, uint32_t he, const uint8_t* cid, uint32_t cid_len,
                          bool cid_def, const uint8_t* usr, uint32_t usr_len, bool usr_def, uint32_t fam,
                          const uint8_t* ip) {
    uint32_t st = 0, depth = 0;   // bool stack as bits
    for (uint32_t k = hb; k < he; ++k) {
        const AclWho& h = v.who[k];
        bool r;
        switch (h.kind) {
            case H_ALL: r = true; break;
            case H_CLIENT: r = cid_def && cid_len == h.n && bytes_eq(cid, v.arena + h.off, h.n); break;
            case H_USER: r = usr_def && usr_len == h.n && bytes_eq(usr, v.arena + h.off, h.n); break;
            case H_IPADDR: {
                r = fam != 0 && fam == h.family;
                const uint32_t nb = h.family == 4 ? 4 : 16;
                for (uint32_t i = 0, bits = h.n; r && i < nb; ++i, bits = bits > 8 ? bits - 8 : 0) {
                    const uint8_t m = bits >= 8 ? 0xFF : (uint8_t)(0xFF00u >> bits);
                    r = (ip[i] & m) == h.addr[i];
                }
                break;
            }
            case H_AND:
            case H_OR: {
                const uint32_t mask = h.n >= 32 ? ~0u : ((1u << h.n) - 1u);
                const uint32_t kids = st & mask;
                st = h.n >= 32 ? 0 : st >> h.n;
                depth -= h.n;
                r = h.kind == H_AND ? kids == mask : kids != 0;
                break;
            }
            default: r = false;
        }
        st = (st << 1) | (r ? 1u : 0u);
        ++depth;
    }
    return depth > 0 && (st & 1u);
}

__global__ void __launch_bounds__(256)
tm_acl_check(AclView v, uint32_t n, const uint8_t* __restrict__ access, const uint8_t* __restrict__ topics,
             const uint64_t* __restrict__ toff, const uint8_t* __restrict__ cids, const uint64_t* __restrict__ coff,
             const uint8_t* __restrict__ cdef, const uint8_t* __restrict__ usrs, const uint64_t* __restrict__ uoff,
             const uint8_t* __restrict__ udef, const uint8_t* __restrict__ peers, const uint8_t* __restrict__ pfam,
             int8_t* __restrict__ out, uint32_t* __restrict__ out_rule) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t acc = access[i] == 1 ? 1u : 2u;   // publish / subscribe
    const uint8_t* cid = cids + coff[i];
    const uint32_t cid_len = (uint32_t)(coff[i + 1] - coff[i]);
    const bool cid_def = cdef[i] != 0;
    const uint8_t* usr = usrs + uoff[i];
    const uint32_t usr_len = (uint32_t)(uoff[i + 1] - uoff[i]);
    const bool usr_def = udef[i] != 0;
    const uint32_t fam = pfam ? pfam[i] : 0u;
    const uint8_t* ip = peers ? peers + 16ull * i : nullptr;
    int8_t res = -1;
    uint32_t which = 0xFFFFFFFFu;
    for (uint32_t r = 0; r < v.nrules; ++r) {
        const AclRule& R = v.rules[r];
        if (!(R.access & acc)) continue;                  // emqx_acl_internal filter/2
        bool m = R.all != 0;                              // {AllowDeny, all}
        if (!m && who_match(v, R.hbeg, R.hend, cid, cid_len, cid_def, usr, usr_len, usr_def, fam, ip)) {
            for (uint32_t f = R.fbeg; f < R.fend && !m; ++f)
                m = filter_match(v, v.filters[f], topics, toff[i], toff[i + 1], cid, cid_len, cid_def, usr, usr_len,
                                 usr_def);
        }
        if (m) {
            res = (int8_t)R.allow;
            which = r;
            break;
        }
    }
    out[i] = res;
    if (out_rule) out_rule[i] = which;
}

template <class T>
struct DVec {
    T* p = nullptr;
    size_t n = 0;
    bool put(const std::vector<T>& h) {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = h.size();
        if (h.empty()) return true;
        if (hipMalloc(&p, h.size() * sizeof(T)) != hipSuccess) return false;
        return hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
    }
    ~DVec() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct tm_acl {
    std::mutex mu;
    int device = -1;
    std::vector<AclRule> rules;
    std::vector<AclFilter> filters;
    std::vector<AclWord> words;
    std::vector<AclWho> who;
    std::vector<uint8_t> arena;
    bool open_rule = false, dirty = true;
    std::vector<uint32_t> groups;   // open AND/OR groups: index of the group's first child count slot
    std::vector<uint32_t> group_kind, group_count;
    DVec<AclRule> d_rules;
    DVec<AclFilter> d_filters;
    DVec<AclWord> d_words;
    DVec<AclWho> d_who;
    DVec<uint8_t> d_arena;

    uint64_t put_bytes(const uint8_t* p, uint32_t n) {
        const uint64_t off = arena.size();
        arena.insert(arena.end(), p, p + n);
        return off;
    }
    void bump_group() {
        if (!group_count.empty()) group_count.back()++;
    }
};

extern "C" {

int tm_acl_open(int device, tm_acl** out) {
    if (!out) return TM_EINVAL;
    tm_acl* a = new (std::nothrow) tm_acl();
    if (!a) return TM_ENOMEM;
    a->device = device;
    *out = a;
    return TM_OK;
}

void tm_acl_close(tm_acl* a) { delete a; }

int tm_acl_rule_begin(tm_acl* a, int allow, uint32_t access) {
    if (!a || a->open_rule || access > TM_ACL_PUBSUB) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    AclRule r{};
    r.allow = allow ? 1 : 0;
    r.all = access == TM_ACL_ALL ? 1u : 0u;
    r.access = access == TM_ACL_ALL || access == TM_ACL_PUBSUB ? 3u : access == TM_ACL_PUBLISH ? 1u : 2u;
    r.hbeg = r.hend = (uint32_t)a->who.size();
    r.fbeg = r.fend = (uint32_t)a->filters.size();
    a->rules.push_back(r);
    a->open_rule = true;
    a->dirty = true;
    return TM_OK;
}

int tm_acl_who(tm_acl* a, uint32_t kind, const uint8_t* arg, uint32_t len, uint32_t prefix) {
    if (!a || !a->open_rule || (len && !arg)) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    AclWho h{};
    switch (kind) {
        case TM_ACL_WHO_ALL:
        case TM_ACL_WHO_CLIENT_ALL:
        case TM_ACL_WHO_USER_ALL:
            h.kind = H_ALL;
            break;
        case TM_ACL_WHO_CLIENT:
        case TM_ACL_WHO_USER:
            h.kind = kind == TM_ACL_WHO_CLIENT ? H_CLIENT : H_USER;
            h.n = len;
            h.off = a->put_bytes(arg, len);
            break;
        case TM_ACL_WHO_IPADDR: {   // arg: "a.b.c.d" or IPv6 text; prefix: mask bits (0 = full)
            std::string s(reinterpret_cast<const char*>(arg), len);
            uint8_t buf[16] = {0};
            if (inet_pton(AF_INET, s.c_str(), buf) == 1) {
                h.family = 4;
                h.n = prefix ? prefix : 32;
                if (h.n > 32) return TM_EINVAL;
            } else if (inet_pton(AF_INET6, s.c_str(), buf) == 1) {
                h.family = 6;
                h.n = prefix ? prefix : 128;
                if (h.n > 128) return TM_EINVAL;
            } else {
                return TM_EINVAL;
            }
            h.kind = H_IPADDR;
            for (uint32_t i = 0, bits = h.n; i < 16; ++i, bits = bits > 8 ? bits - 8 : 0)
                h.addr[i] = buf[i] & (bits >= 8 ? 0xFF : (uint8_t)(0xFF00u >> bits));
            break;
        }
        case TM_ACL_WHO_AND:
        case TM_ACL_WHO_OR:   // open a group; its conditions follow, closed by TM_ACL_WHO_END
            a->bump_group();
            a->group_kind.push_back(kind);
            a->group_count.push_back(0);
            return TM_OK;
        case TM_ACL_WHO_END: {
            if (a->group_kind.empty()) return TM_EINVAL;
            h.kind = a->group_kind.back() == TM_ACL_WHO_AND ? H_AND : H_OR;
            h.n = a->group_count.back();
            if (h.n > 31) return TM_EINVAL;
            a->group_kind.pop_back();
            a->group_count.pop_back();
            a->who.push_back(h);
            a->rules.back().hend = (uint32_t)a->who.size();
            return TM_OK;
        }
        default:
            return TM_EINVAL;
    }
    a->bump_group();
    a->who.push_back(h);
    a->rules.back().hend = (uint32_t)a->who.size();
    return TM_OK;
}

int tm_acl_topic(tm_acl* a, int eq, const uint8_t* topic, uint32_t len) {
    if (!a || !a->open_rule || (len && !topic)) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    AclFilter f{};
    f.wbeg = (uint32_t)a->words.size();
    bool pattern = false;
    for (uint32_t s = 0, i = 0; i <= len; ++i) {   // emqx_topic:words/1
        if (i < len && topic[i] != '/') continue;
        AclWord w{};
        const uint32_t n = i - s;
        const uint8_t* p = topic + s;
        if (n == 0) w.kind = W_EMPTY;
        else if (n == 1 && p[0] == '+') w.kind = W_PLUS;
        else if (n == 1 && p[0] == '#') w.kind = W_HASH;
        else {
            w.kind = W_BIN;
            w.len = n;
            w.off = a->put_bytes(p, n);
            if (!eq && n == 2 && p[0] == '%' && (p[1] == 'c' || p[1] == 'u')) {   // 'pattern?'/1
                w.kind = p[1] == 'c' ? W_PCT_C : W_PCT_U;
                pattern = true;
            }
        }
        a->words.push_back(w);
        s = i + 1;
    }
    f.wend = (uint32_t)a->words.size();
    f.kind = eq ? F_EQ : pattern ? F_PATTERN : F_PLAIN;
    a->filters.push_back(f);
    a->rules.back().fend = (uint32_t)a->filters.size();
    return TM_OK;
}

int tm_acl_rule_end(tm_acl* a) {
    if (!a || !a->open_rule || !a->group_kind.empty()) return TM_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    AclRule& r = a->rules.back();
    if (!r.all && r.hbeg == r.hend) {   // no who: emqx_access_rule has none; treat as 'all'
        AclWho h{};
        h.kind = H_ALL;
        a->who.push_back(h);
        r.hend = (uint32_t)a->who.size();
    }
    a->open_rule = false;
    return TM_OK;
}

int tm_acl_rule_count(tm_acl* a) { return a ? (int)a->rules.size() : 0; }

int tm_acl_check_batch(tm_acl* a, uint32_t n, const uint8_t* access, const uint8_t* topics, const uint64_t* topic_off,
                       const uint8_t* client_ids, const uint64_t* client_off, const uint8_t* client_defined,
                       const uint8_t* usernames, const uint64_t* user_off, const uint8_t* user_defined,
                       const uint8_t* peers, const uint8_t* peer_family, int8_t* out_result, uint32_t* out_rule) {
    if (!a || a->open_rule || (n && (!access || !topics || !topic_off || !client_ids || !client_off ||
                                     !client_defined || !usernames || !user_off || !user_defined || !out_result)))
        return TM_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    if (a->device < 0) return TM_EDEVICE;   // the check runs on the GPU only
    if (n == 0) return TM_OK;
    if (hipSetDevice(a->device) != hipSuccess) return TM_EDEVICE;
    if (a->dirty) {
        if (!a->d_rules.put(a->rules) || !a->d_filters.put(a->filters) || !a->d_words.put(a->words) ||
            !a->d_who.put(a->who) || !a->d_arena.put(a->arena))
            return TM_ENOMEM;
        a->dirty = false;
    }
    // stage the batch (host buffers) on the device
    const uint64_t tb = topic_off[n] - topic_off[0], cb = client_off[n] - client_off[0],
                   ub = user_off[n] - user_off[0];
    std::vector<uint64_t> to(topic_off, topic_off + n + 1), co(client_off, client_off + n + 1),
        uo(user_off, user_off + n + 1);
    for (auto& x : to) x -= topic_off[0];
    for (auto& x : co) x -= client_off[0];
    for (auto& x : uo) x -= user_off[0];
    struct Buf {
        void* p = nullptr;
        ~Buf() {
            if (p) (void)hipFree(p);
        }
    } b_acc, b_t, b_to, b_c, b_co, b_cd, b_u, b_uo, b_ud, b_p, b_pf, b_out, b_rule;
    auto up = [](Buf& b, const void* src, size_t bytes) {
        if (hipMalloc(&b.p, bytes ? bytes : 1) != hipSuccess) return false;
        return !bytes || hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!up(b_acc, access, n) || !up(b_t, topics + topic_off[0], tb) || !up(b_to, to.data(), (n + 1) * 8) ||
        !up(b_c, client_ids + client_off[0], cb) || !up(b_co, co.data(), (n + 1) * 8) ||
        !up(b_cd, client_defined, n) || !up(b_u, usernames + user_off[0], ub) || !up(b_uo, uo.data(), (n + 1) * 8) ||
        !up(b_ud, user_defined, n) || (peers && !up(b_p, peers, 16ull * n)) ||
        (peer_family && !up(b_pf, peer_family, n)) || hipMalloc(&b_out.p, n) != hipSuccess ||
        (out_rule && hipMalloc(&b_rule.p, 4ull * n) != hipSuccess))
        return TM_ENOMEM;
    AclView v{a->d_rules.p, (uint32_t)a->rules.size(), a->d_filters.p, a->d_words.p, a->d_who.p, a->d_arena.p};
    hipLaunchKernelGGL(tm_acl_check, dim3((n + 255) / 256), dim3(256), 0, 0, v, n, (const uint8_t*)b_acc.p,
                       (const uint8_t*)b_t.p, (const uint64_t*)b_to.p, (const uint8_t*)b_c.p,
                       (const uint64_t*)b_co.p, (const uint8_t*)b_cd.p, (const uint8_t*)b_u.p,
                       (const uint64_t*)b_uo.p, (const uint8_t*)b_ud.p, (const uint8_t*)b_p.p,
                       (const uint8_t*)b_pf.p, (int8_t*)b_out.p, (uint32_t*)b_rule.p);
    if (hipGetLastError() != hipSuccess) return TM_EDEVICE;
    if (hipMemcpy(out_result, b_out.p, n, hipMemcpyDeviceToHost) != hipSuccess ||
        (out_rule && hipMemcpy(out_rule, b_rule.p, 4ull * n, hipMemcpyDeviceToHost) != hipSuccess))
        return TM_EDEVICE;
    return TM_OK;
}

int tm_acl_check_batch_device(tm_acl* a, uint32_t n, const uint8_t* d_access, const uint8_t* d_topics,
                              const uint64_t* d_topic_off, const uint8_t* d_client_ids, const uint64_t* d_client_off,
                              const uint8_t* d_client_defined, const uint8_t* d_usernames, const uint64_t* d_user_off,
                              const uint8_t* d_user_defined, const uint8_t* d_peers, const uint8_t* d_peer_family,
                              int8_t* d_out_result, uint32_t* d_out_rule, void* hip_stream) {
    if (!a || a->open_rule || (n && (!d_access || !d_topic_off || !d_client_off || !d_client_defined ||
                                     !d_user_off || !d_user_defined || !d_out_result)))
        return TM_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    if (a->device < 0) return TM_EDEVICE;
    if (n == 0) return TM_OK;
    if (hipSetDevice(a->device) != hipSuccess) return TM_EDEVICE;
    if (a->dirty) {
        if (!a->d_rules.put(a->rules) || !a->d_filters.put(a->filters) || !a->d_words.put(a->words) ||
            !a->d_who.put(a->who) || !a->d_arena.put(a->arena))
            return TM_ENOMEM;
        a->dirty = false;
    }
    AclView v{a->d_rules.p, (uint32_t)a->rules.size(), a->d_filters.p, a->d_words.p, a->d_who.p, a->d_arena.p};
    hipLaunchKernelGGL(tm_acl_check, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, v, n, d_access,
                       d_topics, d_topic_off, d_client_ids, d_client_off, d_client_defined, d_usernames, d_user_off,
                       d_user_defined, d_peers, d_peer_family, d_out_result, d_out_rule);
    return hipGetLastError() == hipSuccess ? TM_OK : TM_EDEVICE;
}

}  // extern "C"
