"""Route bag bookkeeping of emqx_router on the host side of the engine
(add_route / del_route with the reference's trie deltas, get_routes) against
the oracle's RouteTable (oracle/pytrie.py), on a host-only engine."""
import random

from emqx_amd import Engine
from emqx_amd.emqx_router import Router
from oracle import pytrie

DESTS = ["n1", "n2", ("g1", "n1"), ("g2", "n2")]


def _pool(rng, k):
    words = [b"a", b"b", b"", b"+", b"#", b"$SYS", b"c"]
    pool = set()
    while len(pool) < k:
        ws = [rng.choice(words) for _ in range(rng.randint(1, 4))]
        if b"#" in ws[:-1]:
            continue
        pool.add(b"/".join(ws))
    return sorted(pool)


def _prefixes(f):
    ws = f.split(b"/")
    return [b"/".join(ws[:i]) for i in range(1, len(ws) + 1)]


def test_route_bag_and_trie_deltas_vs_oracle():
    rng = random.Random(7)
    for _ in range(10):
        e = Engine(device=-1)
        r, o = Router(e, node="n1"), pytrie.RouteTable()
        pool = _pool(rng, 40)
        for _ in range(400):
            t, d = rng.choice(pool), rng.choice(DESTS)
            if rng.random() < 0.6:
                r.add_route(t, d)
                o.add_route(t, d)
            else:
                r.del_route(t, d)
                o.del_route(t, d)
        for t in pool:
            assert [x.dest for x in r.get_routes(t)] == o.get_routes(t), t
            assert r.has_routes(t) == bool(o.get_routes(t))
            for nid in _prefixes(t):
                assert e.lookup(nid) == o.trie.lookup(nid), nid
        assert e.route_count == sum(len(v) for v in o.routes.values())
        e.close()
