"""emqx_access_rule / emqx_acl_internal on the GPU: a rule set
compiled like emqx_access_rule:compile/1 (src/emqx_access_rule.erl:38-75),
checked in batches by the acl.hip kernel with emqx_acl_internal:match/3's
first-match semantics (src/emqx_acl_internal.erl:63-87).

Rule terms (the acl.conf shapes): ("allow"|"deny", "all") or
("allow"|"deny", who, "publish"|"subscribe"|"pubsub", topics), who = "all" |
("client", c | "all") | ("user", u | "all") | ("ipaddr", "a.b.c.d[/n]") |
("and"|"or", [who...]); topics = a topic or a list of topics / ("eq", topic).
Credentials: dicts with optional client_id, username (None = undefined) and
peername ((ip_text, port) or None)."""
import ctypes
import ipaddress

import numpy as np

from . import _lib as L

ACCESS = {"publish": 1, "subscribe": 2, "pubsub": 3}
WHO = {"all": 0, "client": 1, "user": 2, "client_all": 3, "user_all": 4, "ipaddr": 5, "and": 6, "or": 7, "end": 8}
RESULT = {1: "allow", 0: "deny", -1: "nomatch"}


def _b(x):
    return x.encode() if isinstance(x, str) else bytes(x)


class AclRules:
    def __init__(self, device=0):
        self.lib = L.load()
        h = ctypes.c_void_p()
        rc = self.lib.tm_acl_open(device, ctypes.byref(h))
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_acl_open")
        self.h = h

    def close(self):
        if self.h:
            self.lib.tm_acl_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc, what):
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, what)

    def _who(self, w):
        if w == "all":
            return self._ck(self.lib.tm_acl_who(self.h, WHO["all"], None, 0, 0), "who")
        kind, arg = w
        if kind in ("client", "user"):
            if arg == "all":
                return self._ck(self.lib.tm_acl_who(self.h, WHO[kind + "_all"], None, 0, 0), "who")
            a = _b(arg)
            return self._ck(self.lib.tm_acl_who(self.h, WHO[kind], a, len(a), 0), "who")
        if kind == "ipaddr":
            addr, _, bits = str(arg).partition("/")
            net = ipaddress.ip_network(str(arg), strict=False)
            a = addr.encode()
            return self._ck(self.lib.tm_acl_who(self.h, WHO["ipaddr"], a, len(a),
                                                int(bits) if bits else net.max_prefixlen), "who")
        if kind in ("and", "or"):
            self._ck(self.lib.tm_acl_who(self.h, WHO[kind], None, 0, 0), "who")
            for c in arg:
                self._who(c)
            return self._ck(self.lib.tm_acl_who(self.h, WHO["end"], None, 0, 0), "who")
        raise ValueError(w)

    def add(self, rule):
        """one rule, appended after the ones already loaded (file order)"""
        if len(rule) == 2 and rule[1] == "all":
            self._ck(self.lib.tm_acl_rule_begin(self.h, 1 if rule[0] == "allow" else 0, 0), "rule")
            return self._ck(self.lib.tm_acl_rule_end(self.h), "rule_end")
        a, who, access, topics = rule
        self._ck(self.lib.tm_acl_rule_begin(self.h, 1 if a == "allow" else 0, ACCESS[access]), "rule")
        self._who(who)
        if isinstance(topics, (str, bytes)):
            topics = [topics]
        for t in topics:
            eq = isinstance(t, (tuple, list)) and t[0] == "eq"
            tb = _b(t[1] if eq else t)
            self._ck(self.lib.tm_acl_topic(self.h, 1 if eq else 0, tb, len(tb)), "topic")
        return self._ck(self.lib.tm_acl_rule_end(self.h), "rule_end")

    def load(self, rules):
        for r in rules:
            self.add(r)
        return self

    @staticmethod
    def pack(creds, pubsubs, topics):
        """the batch as the C-ABI's arrays (name -> numpy array), in
        tm_acl_check_batch's argument order"""
        n = len(topics)

        def strs(items):
            bs = [_b(x) for x in items]
            off = np.zeros(n + 1, dtype=np.uint64)
            if n:
                off[1:] = np.cumsum([len(x) for x in bs])
            return np.frombuffer(b"".join(bs) + b"\0" * 8, dtype=np.uint8).copy(), off
        tb, to = strs(topics)
        cb, co = strs([c.get("client_id") or b"" for c in creds])
        ub, uo = strs([c.get("username") or b"" for c in creds])
        cd = np.array([c.get("client_id") is not None for c in creds], dtype=np.uint8)
        ud = np.array([c.get("username") is not None for c in creds], dtype=np.uint8)
        peers = np.zeros((max(n, 1), 16), dtype=np.uint8)
        fam = np.zeros(max(n, 1), dtype=np.uint8)
        for i, c in enumerate(creds):
            p = c.get("peername")
            if p:
                ip = ipaddress.ip_address(p[0])
                raw = ip.packed
                peers[i, :len(raw)] = np.frombuffer(raw, dtype=np.uint8)
                fam[i] = 4 if ip.version == 4 else 6
        acc = np.array([1 if p == "publish" else 2 for p in pubsubs], dtype=np.uint8)
        return {"access": acc, "topics": tb, "topic_off": to, "client_ids": cb, "client_off": co,
                "client_defined": cd, "usernames": ub, "user_off": uo, "user_defined": ud, "peers": peers,
                "peer_family": fam}

    ARGS = ("access", "topics", "topic_off", "client_ids", "client_off", "client_defined", "usernames", "user_off",
            "user_defined", "peers", "peer_family")

    def check_packed(self, n, arrs):
        """host arrays from pack() -> (result int8[n], rule u32[n])"""
        out = np.zeros(max(n, 1), dtype=np.int8)
        rule = np.zeros(max(n, 1), dtype=np.uint32)
        P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        self._ck(self.lib.tm_acl_check_batch(self.h, n, *[P(arrs[k]) for k in self.ARGS], P(out), P(rule)),
                 "tm_acl_check_batch")
        return out[:n], rule[:n]

    def check_device(self, n, d, d_out, d_rule, stream=None):
        """device tensors (the pack() names) -> d_out / d_rule, stream-ordered
        (tm_acl_check_batch_device)"""
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        st = None
        if stream is not None:
            st = ctypes.c_void_p(L.stream_handle(stream))
        self._ck(self.lib.tm_acl_check_batch_device(self.h, n, *[P(d[k]) for k in self.ARGS], P(d_out), P(d_rule),
                                                    st), "tm_acl_check_batch_device")

    def check_many(self, creds, pubsubs, topics):
        """-> [(allow|deny|nomatch, rule index or None)] per check (GPU)"""
        n = len(topics)
        out, rule = self.check_packed(n, self.pack(creds, pubsubs, topics))
        return [(RESULT[int(out[i])], None if rule[i] == 0xFFFFFFFF else int(rule[i])) for i in range(n)]
