"""The oracle against the reference's golden vectors (CPU only).

O1 (oracle/o1_trie.c) and pytrie (oracle/pytrie.py) are two independent
restatements of emqx_trie; both must reproduce every known-answer test of the
reference suites (tests/golden/kat_*.json) and agree with each other and with
brute-force emqx_topic:match/2 (O2) on randomized tries.
"""
import os
import random

import pytest

from oracle import O1, o2_topic_match, pytrie

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

L1 = "latin-1"


def b(x):
    return x.encode(L1)


def run_kat_trie(kat, impl):
    for op, arg in kat["ops"]:
        getattr(impl, op)(b(arg))
    for chk in kat["checks"]:
        kind, arg, exp = chk
        if kind == "lookup":
            got = [[ec, None if t is None else t.decode(L1)] for ec, t in impl.lookup(b(arg))]
            assert got == exp, (kat["name"], arg, got, exp)
        elif kind == "match":
            got = [t.decode(L1) for t in impl.match(b(arg))]
            assert got == exp, (kat["name"], arg, got, exp)
        elif kind == "match_len":
            assert len(impl.match(b(arg))) == exp


@pytest.mark.parametrize("impl", ["o1", "pytrie"])
def test_kat_trie(golden, impl):
    for kat in golden["kat_trie"]:
        t = O1() if impl == "o1" else pytrie.Trie()
        run_kat_trie(kat, t)


def test_kat_topic_match(golden):
    for name, filt, exp in golden["kat_topic"]["match"]:
        assert o2_topic_match(b(name), b(filt)) == exp, (name, filt)
        assert pytrie.match(b(name), b(filt)) == exp, (name, filt)


def test_kat_client_sets(golden):
    for case in golden["kat_client"]["cases"]:
        t = O1()
        for f in case["subs"]:
            t.insert(b(f))
        assert sorted(x.decode() for x in t.match(b(case["pub"]))) == sorted(case["set"])


def test_kat_router(golden):
    for kat in golden["kat_router"]:
        trie, routes = pytrie.Trie(), {}
        for topic, dest in kat["add"]:
            tb = b(topic)
            if pytrie.wildcard(tb) and tb not in routes:
                trie.insert(tb)
            routes.setdefault(tb, []).append(dest)
        got = sorted([t.decode(), d] for t, d in pytrie.match_routes(trie, routes, b(kat["topic"])))
        assert got == kat["sorted"]
        if "then_del" in kat:
            for topic, dest in kat["then_del"]:
                tb = b(topic)
                if pytrie.wildcard(tb) and routes.get(tb) == [dest]:
                    trie.delete(tb)
                routes[tb].remove(dest)
                if not routes[tb]:
                    del routes[tb]
            got = sorted([t.decode(), d] for t, d in pytrie.match_routes(trie, routes, b(kat["topic"])))
            assert got == kat["sorted_after"]
            node, exp = kat["lookup_after"]
            assert trie.lookup(b(node)) == exp


def test_o1_vectors_regression(golden):
    """O1 still produces exactly the committed vectors (order and E)."""
    for vec in golden["o1_vectors"]:
        t = O1()
        for f in vec["filters"]:
            t.insert(b(f))
        for row in vec["topics"]:
            got, e = t.match(b(row["topic"]), with_edges=True)
            assert [x.decode(L1) for x in got] == row["match"], (vec["name"], row["topic"])
            assert e == row["edge_reads"]


def _rand_case(rng):
    voc = rng.randint(1, 4)
    filters = set()
    for _ in range(rng.randint(1, 60)):
        k = rng.randint(1, 6)
        ws = []
        for i in range(k):
            r = rng.random()
            if i == k - 1 and r < 0.2:
                ws.append("#")
            elif r < 0.45:
                ws.append("+")
            elif r < 0.5:
                ws.append("")
            elif i == 0 and r < 0.55:
                ws.append("$S")
            else:
                ws.append("w%d" % rng.randrange(voc))
        filters.add("/".join(ws))
    topics = []
    for _ in range(20):
        k = rng.randint(1, 6)
        ws = ["" if rng.random() < 0.1 else ("$S" if i == 0 and rng.random() < 0.1 else "w%d" % rng.randrange(voc))
              for i in range(k)]
        topics.append("/".join(ws))
    return sorted(filters), topics


def test_o1_vs_pytrie_vs_o2_random():
    rng = random.Random(12345)
    for _ in range(150):
        filters, topics = _rand_case(rng)
        o1, py = O1(), pytrie.Trie()
        for f in filters:
            o1.insert(b(f))
            py.insert(b(f))
        for t in topics:
            got, e = o1.match(b(t), with_edges=True)
            assert got == py.match(b(t))
            assert e == py.edge_reads
            brute = {b(f) for f in filters if o2_topic_match(b(t), b(f))}
            assert set(got) == brute
            assert len(got) == len(set(got))


def test_o1_delete_matches_pytrie_random():
    rng = random.Random(7)
    for _ in range(60):
        filters, topics = _rand_case(rng)
        o1, py = O1(), pytrie.Trie()
        for f in filters:
            o1.insert(b(f))
            py.insert(b(f))
        dels = rng.sample(filters, len(filters) // 2) + ["w0/zz", "+/nope"]
        for f in dels:
            o1.delete(b(f))
            py.delete(b(f))
        for t in topics:
            assert o1.match(b(t)) == py.match(b(t))
        # every prefix node's bookkeeping agrees
        for f in filters:
            parts = f.split("/")
            for k in range(1, len(parts) + 1):
                nid = b("/".join(parts[:k]))
                assert o1.lookup(nid) == py.lookup(nid), nid


def test_o3_interned_equals_o1():
    """the optimized CPU baseline leg (oracle/o3_interned.c) returns O1's
    ordered lists: C1, a C5 sample ($ topics, '#'-heavy, fan-out > 500) and
    the O1 vectors (empty levels, 31-41 levels)"""
    import json
    import numpy as np
    from emqx_amd import emqx_topic as T
    from emqx_amd import workload as W
    from emqx_amd.engine import pack
    from oracle import O1, O3
    cases = [(W.filters(1), W.topics(1, n=20000))]
    f5 = [T.parse(f)[0] for f in W.unpack(*W.filters(5, n=30000))]
    cases.append((pack(list(dict.fromkeys(f5))), W.topics(5, n=300)))
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "o1_vectors.json")))
    for vec in g["vectors"] if isinstance(g, dict) and "vectors" in g else g:
        fs = list(dict.fromkeys(f.encode("latin-1") for f in vec["filters"]))
        cases.append((pack(fs), pack([r["topic"].encode("latin-1") for r in vec["topics"]])))
    for (fb, fo), (tb, to) in cases:
        o1, o3 = O1(), O3()
        o1.insert_many(fb, fo)
        o3.insert_many(fb, fo)
        a = o1.match_ids(tb, to, threads=4)
        b = o3.match_ids(tb, to, threads=4)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
