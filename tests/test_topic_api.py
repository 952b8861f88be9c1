"""emqx_amd.emqx_topic (the reference's topic algebra API) against the
reference's known answers (tests/golden/kat_topic.json) and the pytrie
transcription.  CPU only: these are pure functions of libtopicmatch."""
import random

import pytest

from emqx_amd import emqx_topic as T
from oracle import pytrie


def w(x):
    if isinstance(x, dict):
        return {"": T.EMPTY, "+": T.PLUS, "#": T.HASH}[x["atom"]]
    return x.encode()


def test_match_kat(golden):
    for name, filt, exp in golden["kat_topic"]["match"]:
        assert T.match(name.encode(), filt.encode()) == exp, (name, filt)


def test_wildcard_kat(golden):
    for t, exp in golden["kat_topic"]["wildcard"]:
        assert T.wildcard(t.encode()) == exp


def test_words_kat(golden):
    for t, exp in golden["kat_topic"]["words"]:
        got = T.words(t.encode())
        want = [w(x) for x in exp]
        assert len(got) == len(want)
        for g, x in zip(got, want):
            if isinstance(x, T.Atom):
                assert g is x
            else:
                assert g == x


def test_triples_levels_join_kat(golden):
    kt = golden["kat_topic"]
    for t, exp in kt["triples"]:
        got = [(None if p is None else p.decode(), x.decode(), n.decode()) for p, x, n in T.triples(t.encode())]
        assert got == [tuple(e) for e in exp]
    for t, n in kt["levels"]:
        assert T.levels(t.encode()) == n
    for ws, exp in kt["join"]:
        assert T.join([w(x) for x in ws]) == exp.encode()
    for t in kt["join_words_roundtrip"]:
        assert T.join(T.words(t.encode())) == t.encode()


def test_validate_kat(golden):
    for (kind, t), exp in golden["kat_topic"]["validate"]:
        if exp == "error":
            with pytest.raises(T.TopicError):
                T.validate((kind, t.encode()))
        else:
            assert T.validate((kind, t.encode())) == exp, (kind, t)
    long_topic = b"".join(b"%d/" % i for i in range(10001))
    with pytest.raises(T.TopicError):
        T.validate(("name", long_topic))


def test_parse_kat(golden):
    for t, inner, grp in golden["kat_topic"]["parse"]:
        got, opts = T.parse(t.encode())
        assert got == inner.encode()
        assert opts.get("share") == (None if grp is None else grp.encode())
    for bad in [b"$share/x", b"$share/", b"$share/g+/t", b"$queue/$share/g/t", b"$queue/$queue/t"]:
        with pytest.raises(T.TopicError):
            T.parse(bad)
    with pytest.raises(T.TopicError):
        T.parse(b"$queue/t", {"share": b"g"})


def test_feed_var_kat(golden):
    for var, val, topic, exp in golden["kat_topic"]["feed_var"]:
        assert T.feed_var(var, val, topic) == exp.encode()


def test_match_vs_pytrie_random():
    rng = random.Random(99)
    alpha = ["a", "b", "", "+", "#", "$x", "$SYS"]
    for _ in range(4000):
        name = "/".join(rng.choice(["a", "b", "", "$x", "c"]) for _ in range(rng.randint(1, 4)))
        filt = "/".join(rng.choice(alpha) for _ in range(rng.randint(1, 4)))
        exp = pytrie.match(name.encode(), filt.encode())
        assert T.match(name.encode(), filt.encode()) == exp, (name, filt)
        # word-list form skips the '$' rule like the reference's list clauses
        assert T.match(T.words(name), T.words(filt)) == pytrie.match(pytrie.words(name.encode()),
                                                                       pytrie.words(filt.encode()))


def test_parse_vs_pytrie_random():
    rng = random.Random(5)
    parts = ["$share", "$queue", "g", "", "a", "+", "#", "$local"]
    for _ in range(3000):
        t = "/".join(rng.choice(parts) for _ in range(rng.randint(1, 5))).encode()
        try:
            exp = pytrie.parse(t)
        except pytrie.InvalidTopic:
            exp = "error"
        try:
            got = T.parse(t)
        except T.TopicError:
            got = "error"
        assert got == exp, t
