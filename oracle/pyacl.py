"""TEST INFRASTRUCTURE ONLY — literal Python transcription of the reference's
ACL rule matching, the checker of the batched ACL kernel (emqx_amd/csrc/acl.hip).
Never imported by the product package.

    emqx_access_rule:compile/1, compile/2   src/emqx_access_rule.erl:38-80
    emqx_access_rule:match/3                 :82-92
    match_who/2                              :94-119
    match_topics/3, match_topic/2            :121-134
    feed_var/2,3                             :136-149
    emqx_acl_internal filter/2, match/3      src/emqx_acl_internal.erl:47-61, 79-87
    esockd_cidr:parse/2, match/2             esockd v5.4.2 (not vendored; restated:
                                             a CIDR is the address range Start..End)

Terms: who = "all" | ("client", b | "all") | ("user", b | "all") |
("ipaddr", "a.b.c.d[/n]") | ("and" | "or", [who]); rule = (A, "all") |
(A, who, "publish" | "subscribe" | "pubsub", topics) with topics a str/bytes or
a list of (bytes | ("eq", bytes)); credentials = dict with optional keys
client_id, username (None = undefined) and peername ((ip_bytes, port) or None).
"""
import ipaddress

from .pytrie import EMPTY, HASH, PLUS, _Atom, words


def _b(x):
    return x.encode() if isinstance(x, str) else bytes(x)


# ---- esockd_cidr (restated) --------------------------------------------------
def cidr_parse(s: str):
    net = ipaddress.ip_network(s, strict=False)
    return (int(net.network_address), int(net.broadcast_address), net.version)


def cidr_match(ip: bytes, cidr) -> bool:
    start, end, ver = cidr
    if (len(ip) == 4) != (ver == 4):
        return False
    v = int.from_bytes(ip, "big")
    return start <= v <= end


# ---- emqx_access_rule:compile ---------------------------------------------------
class Pattern:
    def __init__(self, ws):
        self.words = ws

    def __eq__(self, o):
        return isinstance(o, Pattern) and _weq_list(self.words, o.words)


def _weq(a, b):
    return a is b if isinstance(a, _Atom) or isinstance(b, _Atom) else a == b


def _weq_list(a, b):
    return len(a) == len(b) and all(_weq(x, y) for x, y in zip(a, b))


def compile_who(who):
    if who == "all":
        return "all"
    kind, arg = who
    if kind == "ipaddr":
        return ("ipaddr", cidr_parse(arg))
    if kind in ("client", "user"):
        return (kind, "all" if arg == "all" else _b(arg))
    if kind in ("and", "or"):
        return (kind, [compile_who(c) for c in arg])
    raise ValueError(who)


def compile_topic(t):
    if isinstance(t, tuple) and t[0] == "eq":
        return ("eq", words(_b(t[1])))
    ws = words(_b(t))
    if b"%u" in [w for w in ws if not isinstance(w, _Atom)] or b"%c" in [w for w in ws if not isinstance(w, _Atom)]:
        return Pattern(ws)                            # 'pattern?'/1
    return ws


def compile_rule(rule):
    if len(rule) == 2 and rule[1] == "all":
        return (rule[0], "all")
    a, who, access, topics = rule
    if isinstance(topics, (str, bytes)):
        topics = [topics]
    return (a, compile_who(who), access, [compile_topic(t) for t in topics])


# ---- emqx_access_rule:match -----------------------------------------------------
def match_who(cred, who) -> bool:
    if who == "all" or who == ("user", "all") or who == ("client", "all"):
        return True
    kind, arg = who
    if kind == "client":
        return "client_id" in cred and cred["client_id"] is not None and cred["client_id"] == arg
    if kind == "user":
        return "username" in cred and cred["username"] is not None and cred["username"] == arg
    if kind == "ipaddr":
        if "peername" not in cred:
            return False                              # match_who(_, _) -> false
        if cred["peername"] is None:
            return False                              # #{peername := undefined}
        return cidr_match(cred["peername"][0], arg)
    if kind == "and":
        allow = True
        for c in arg:                                 # lists:foldl, andalso
            allow = match_who(cred, c) and allow
        return allow
    if kind == "or":
        allow = False
        for c in arg:
            allow = match_who(cred, c) or allow
        return allow
    return False


def feed_var(cred, pattern):
    out = []
    for w in pattern:
        if w == b"%c" and not isinstance(w, _Atom):
            cid = cred.get("client_id")
            out.append(b"%c" if cid is None else cid)
        elif w == b"%u" and not isinstance(w, _Atom):
            u = cred.get("username")
            out.append(b"%u" if u is None else u)
        else:
            out.append(w)
    return out


def match_words(name, filt) -> bool:
    """emqx_topic:match/2 on word lists (no '$' clause), clause by clause"""
    if not name and not filt:
        return True
    if name and filt and _weq(name[0], filt[0]):
        return match_words(name[1:], filt[1:])
    if name and filt and filt[0] is PLUS:
        return match_words(name[1:], filt[1:])
    if len(filt) == 1 and filt[0] is HASH:
        return True
    return False


def match_topic(topic_words, filt) -> bool:
    if isinstance(filt, tuple) and filt[0] == "eq":
        return _weq_list(topic_words, filt[1])
    return match_words(topic_words, filt)


def match_topics(cred, topic: bytes, filters) -> bool:
    for f in filters:
        if isinstance(f, Pattern):
            if match_topic(words(topic), feed_var(cred, f.words)):
                return True
        elif match_topic(words(topic), f):
            return True
    return False


def match(cred, topic: bytes, rule):
    """-> ("matched", allow|deny) | "nomatch" """
    if len(rule) == 2 and rule[1] == "all":
        return ("matched", rule[0])
    a, who, _access, filters = rule
    if match_who(cred, who) and match_topics(cred, topic, filters):
        return ("matched", a)
    return "nomatch"


# ---- emqx_acl_internal -------------------------------------------------------------
def access_filter(pubsub, rule) -> bool:
    if len(rule) == 2 and rule[1] == "all":
        return True
    access = rule[2]
    return access == "pubsub" or access == pubsub


def check_acl(rules, cred, pubsub, topic: bytes):
    """compiled rules, in order -> ("allow" | "deny" | "nomatch", rule index)"""
    for i, r in enumerate(rules):
        if not access_filter(pubsub, r):
            continue
        m = match(cred, topic, r)
        if m != "nomatch":
            return m[1], i
    return "nomatch", None


__all__ = ["compile_rule", "match", "check_acl", "match_words", "feed_var", "EMPTY"]
