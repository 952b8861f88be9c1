"""emqx_topic — the reference's topic algebra (src/emqx_topic.erl), same names,
argument meaning and error behaviour.

Words follow the Erlang term model: the levels "", "+" and "#" become the
atoms EMPTY, PLUS, HASH (src/emqx_topic.erl:149-152); other levels stay bytes.
match/2, wildcard/1 and parse/1,2 run in libtopicmatch (the same C code the
engine uses); the rest are small pure functions.
"""
import ctypes

from . import _lib as L

MAX_TOPIC_LEN = 4096   # src/emqx_topic.erl:35


class Atom(str):
    """An Erlang atom among words ('' / '+' / '#')."""
    def __repr__(self):
        return "'%s'" % str.__str__(self)


EMPTY, PLUS, HASH = Atom(""), Atom("+"), Atom("#")


class TopicError(ValueError):
    """error(Reason) of the reference (empty_topic, topic_too_long,
    'topic_invalid_#', topic_invalid_char, {invalid_topic, T})."""


def _b(t):
    return t.encode() if isinstance(t, str) and not isinstance(t, Atom) else t


def word(w: bytes):
    """word/1 — src/emqx_topic.erl:149-152"""
    if w == b"":
        return EMPTY
    if w == b"+":
        return PLUS
    if w == b"#":
        return HASH
    return w


def words(topic):
    """words/1 — src/emqx_topic.erl:141-147"""
    return [word(w) for w in _b(topic).split(b"/")]


def levels(topic) -> int:
    """levels/1 — src/emqx_topic.erl:136-137"""
    return len(words(topic))


def wildcard(topic) -> bool:
    """wildcard/1 — src/emqx_topic.erl:41-50"""
    if isinstance(topic, list):
        return any(w is PLUS or w is HASH for w in topic)
    t = _b(topic)
    return L.load().tm_topic_wildcard(t, len(t)) == 1


def _bin(w):
    """bin/1 — src/emqx_topic.erl:131-134"""
    if w is EMPTY:
        return b""
    if w is PLUS:
        return b"+"
    if w is HASH:
        return b"#"
    return _b(w)


def match(name, filt) -> bool:
    """match/2 — src/emqx_topic.erl:56-75 (binaries: through libtopicmatch;
    word lists: the list clauses, which skip the '$' rule)"""
    if isinstance(name, list) or isinstance(filt, list):
        n = name if isinstance(name, list) else words(name)
        f = filt if isinstance(filt, list) else words(filt)
        return _match_words(n, f)
    n, f = _b(name), _b(filt)
    return L.load().tm_topic_match(n, len(n), f, len(f)) == 1


def _weq(a, b):
    if isinstance(a, Atom) or isinstance(b, Atom):
        return a is b
    return a == b


def _match_words(n, f):
    while True:
        if not n and not f:
            return True
        if n and f and _weq(n[0], f[0]):
            n, f = n[1:], f[1:]
            continue
        if n and f and f[0] is PLUS:
            n, f = n[1:], f[1:]
            continue
        return len(f) == 1 and f[0] is HASH


def triples(topic):
    """triples/1 — src/emqx_topic.erl:117-124 -> [(parent, word, node)],
    parent of the first triple is the atom 'root' (None here)"""
    out, parent = [], None
    for w in words(topic):
        node = _bin(w) if parent is None else parent + b"/" + _bin(w)
        out.append((parent, w, node))
        parent = node
    return out


def join(ws) -> bytes:
    """join/1 — src/emqx_topic.erl:165-178"""
    return b"/".join(_bin(w) for w in ws)


def _validate3(w: bytes):
    """validate3/1 — src/emqx_topic.erl:107-113 (utf8 walk)"""
    try:
        s = w.decode("utf-8")
    except UnicodeDecodeError:
        # the reference's <<C/utf8, ...>> clause fails to match -> function_clause
        raise TopicError("function_clause")
    for c in s:
        if c in ("#", "+", "\x00"):
            raise TopicError("topic_invalid_char")
    return True


def _validate2(ws):
    """validate2/1 — src/emqx_topic.erl:94-105"""
    for i, w in enumerate(ws):
        if w is HASH:
            if i != len(ws) - 1:
                raise TopicError("topic_invalid_#")
            return True
        if w is EMPTY or w is PLUS:
            continue
        _validate3(w)
    return True


def validate(arg, topic=None) -> bool:
    """validate/1,2 — src/emqx_topic.erl:79-92.  validate(topic) is a filter
    check; validate(('name'|'filter', topic)) or validate(kind, topic)."""
    if topic is None:
        if isinstance(arg, tuple):
            kind, topic = arg
        else:
            kind, topic = "filter", arg
    else:
        kind = arg
    t = _b(topic)
    if t == b"":
        raise TopicError("empty_topic")
    if len(t) > MAX_TOPIC_LEN:
        raise TopicError("topic_too_long")
    ws = words(t)
    if kind == "filter":
        return _validate2(ws)
    if kind == "name":
        return _validate2(ws) and not wildcard(ws)
    raise TopicError("function_clause")


def parse(topic, options=None):
    """parse/1,2 — src/emqx_topic.erl:180-200 -> (inner_topic, options)"""
    options = dict(options or {})
    t = _b(topic)
    if "share" in options and (t.startswith(b"$queue/") or t.startswith(b"$share/")):
        raise TopicError(("invalid_topic", t))
    inner, ilen = ctypes.c_void_p(), ctypes.c_uint32()
    grp, glen = ctypes.c_void_p(), ctypes.c_uint32()
    rc = L.load().tm_topic_parse(t, len(t), ctypes.byref(inner), ctypes.byref(ilen), ctypes.byref(grp),
                                 ctypes.byref(glen))
    if rc != L.TM_OK:
        raise TopicError(("invalid_topic", t))
    inner_b = ctypes.string_at(inner.value, ilen.value) if ilen.value else b""
    if grp.value:
        options["share"] = ctypes.string_at(grp.value, glen.value) if glen.value else b""
    return inner_b, options


def feed_var(var, val, topic) -> bytes:
    """feed_var/3 — src/emqx_topic.erl:156-163"""
    var, val = _b(var), _b(val)
    return join([val if (not isinstance(w, Atom) and w == var) else w for w in words(topic)])


def systop(name, node=b"emqx@127.0.0.1") -> bytes:
    """systop/1 — src/emqx_topic.erl:150-153 ($SYS/brokers/<node>/<name>)"""
    return b"$SYS/brokers/" + _b(node) + b"/" + _b(name)
