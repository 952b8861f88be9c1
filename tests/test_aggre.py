"""emqx_broker:aggre/1 (src/emqx_broker.erl:194-206) without a GPU: the
oracle's clause-by-clause transcription on hand-worked cases, the closed form
aggre.hip implements checked against the literal fold on random route lists,
and the engine's target registry (tm_dest_target / tm_target_bytes) on a
host-only engine.  The reference's suites hold no aggre/1 vectors, so the
hand cases are worked from the Erlang source (parity of this row rests on the
transcription)."""
import random

import pytest

from emqx_amd import Engine
from emqx_amd.emqx_router import Router
from oracle import pytrie
from oracle.pytrie import _x_term, aggre

N1, N2 = b"n1", b"n2"
G = lambda g, n=b"n1": (g, n)   # noqa: E731  {Group, Node}


def test_aggre_clauses():
    assert aggre([]) == []
    assert aggre([(b"t", N1)]) == [(b"t", (0, N1))]
    assert aggre([(b"t", G(b"g"))]) == [(b"t", (1, b"g"))]
    # node routes only: the fold prepends, no dedup
    assert aggre([(b"a", N1), (b"b", N2), (b"a", N1)]) == [(b"a", (0, N1)), (b"b", (0, N2)), (b"a", (0, N1))]
    # a group route usorts the whole accumulator, later node routes are prepended
    assert aggre([(b"b", N2), (b"a", G(b"g")), (b"c", N1)]) == [(b"c", (0, N1)), (b"a", (1, b"g")), (b"b", (0, N2))]
    # two members of one group on different nodes collapse to one {To, Group}
    assert aggre([(b"x", G(b"g", N1)), (b"x", G(b"g", N2))]) == [(b"x", (1, b"g"))]
    # duplicates before the last group route are removed with it
    assert aggre([(b"a", N1), (b"a", N1), (b"z", G(b"g"))]) == [(b"a", (0, N1)), (b"z", (1, b"g"))]
    # term order: To first (a proper prefix first), then atom < binary
    assert aggre([(b"ab", N1), (b"a", G(b"g")), (b"a", N2), (b"a", G(b"a"))]) == \
        [(b"a", (0, N2)), (b"a", (1, b"a")), (b"a", (1, b"g")), (b"ab", (0, N1))]
    # an atom and a binary with the same text stay distinct
    assert aggre([(b"t", b"g"), (b"t", G(b"g"))]) == [(b"t", (0, b"g")), (b"t", (1, b"g"))]


def closed_form(routes):
    """aggre.hip's formulation: j = last group route; tail r_{m-1}..r_{j+1}
    reversed, then the rank-by-counting usort of r_0..r_j"""
    keys = [(to, _x_term(d)) for to, d in routes]
    grp = [i for i, (_, d) in enumerate(routes) if isinstance(d, tuple)]
    if not grp:
        return keys[::-1]
    j = grp[-1]
    head, tail = keys[: j + 1], keys[j + 1:][::-1]
    first = [k for i, k in enumerate(head) if k not in head[:i]]
    out = [None] * len(first)
    for k in first:
        out[sum(1 for x in first if x < k)] = k
    return tail + out


def test_closed_form_equals_fold():
    rng = random.Random(3)
    tos = [b"", b"a", b"a/b", b"a/+", b"#", b"ab", b"\xff"]
    dests = [N1, N2, b"n10", G(b"g1"), G(b"g1", N2), G(b"g2"), G(b""), b"g1"]
    for _ in range(3000):
        routes = [(rng.choice(tos), rng.choice(dests)) for _ in range(rng.randint(0, 12))]
        assert closed_form(routes) == aggre(routes), routes


def test_target_registry_host_only():
    e = Engine(device=-1)
    t1 = e.dest_target(b"\x02n1", Engine.TARGET_NODE, b"n1")
    t2 = e.dest_target(b"\x01g\x00n1", Engine.TARGET_GROUP, b"g")
    assert t1 != t2
    assert e.target_bytes(t1) == (0, b"n1") and e.target_bytes(t2) == (1, b"g")
    assert e.dest_target(b"\x01g\x00n2", Engine.TARGET_GROUP, b"g") == t2      # same group, same target
    assert e.dest_target(b"\x02g", Engine.TARGET_NODE, b"g") not in (t1, t2)   # atom 'g' =/= <<"g">>
    with pytest.raises(Exception):
        e.dest_target(b"x", 7, b"x")
    with pytest.raises(KeyError):
        e.target_bytes(999)
    r = Router(e, node="n1")
    r.add_route(b"a/+", ("g", "n2"))
    # matching needs the GPU: a host-only engine refuses loudly
    with pytest.raises(Exception):
        r.match_deliveries(b"a/b")
    e.close()


def test_routetable_match_deliveries():
    o = pytrie.RouteTable()
    o.add_route(b"a/+", "n1")
    o.add_route(b"a/+", ("g", "n2"))
    o.add_route(b"a/#", "n2")
    o.add_route(b"a/b", "n3")
    assert o.match_routes(b"a/b") == [(b"a/b", "n3"), (b"a/+", "n1"), (b"a/+", ("g", "n2")), (b"a/#", "n2")]
    assert o.match_deliveries(b"a/b") == [(b"a/#", (0, b"n2")), (b"a/+", (0, b"n1")), (b"a/+", (1, b"g")),
                                          (b"a/b", (0, b"n3"))]


def _golden():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "aggre_vectors.json")))


def _dest(d):
    return (d[1], d[2]) if d[0] == "group" else d[1]


def test_oracle_matches_aggre_golden():
    """the committed fixture (tests/golden/make_aggre_golden.py) replays"""
    n = 0
    for case in _golden()["cases"]:
        o = pytrie.RouteTable()
        for op, t, d in case["ops"]:
            (o.add_route if op == "add" else o.del_route)(bytes.fromhex(t), _dest(d))
        for tp, want in zip(case["topics"] + case["ood_topics"], case["deliveries"] + case["ood_deliveries"]):
            got = [[to.hex(), x[0], x[1].hex()] for to, x in o.match_deliveries(bytes.fromhex(tp))]
            assert got == want, tp
            n += len(want)
        assert all(b"+" not in bytes.fromhex(tp).split(b"/") and b"#" not in bytes.fromhex(tp).split(b"/")
                   for tp in case["topics"])
    assert n > 100
    assert _golden()["source"].startswith("ORACLE-DERIVED")
