"""The in-place route image (engine.cpp, route image maintenance) under
random add / del churn, on a host-only engine: after every burst the image
must mirror the route bags exactly (tm_debug_check_routes: the kernel's probe
finds every topic, segments equal bags, filter entries, order labels), and
get_routes/1 must equal the oracle's bag (oracle/pytrie.RouteTable)."""
import random

import pytest

from emqx_amd import Engine
from oracle import pytrie


def topic_pool(rng, n):
    words = ["a", "b", "sensor", "x" * 9, "dev%d", "+", "#", "", "$SYS", "ab/cd"]
    out = set()
    while len(out) < n:
        lv = []
        for i in range(rng.randint(1, 6)):
            w = rng.choice(words)
            if w == "#" and i < 5:
                w = "h"
            lv.append(w % rng.randint(0, 50) if "%d" in w else w)
        out.add("/".join(lv))
    return sorted(out)


@pytest.mark.parametrize("seed", [1, 2])
def test_route_image_mirrors_bags_under_churn(seed):
    rng = random.Random(seed)
    e = Engine(device=-1)
    e.set_option("route_gc", 64)          # compactions happen in this test
    o = pytrie.RouteTable()
    topics = topic_pool(rng, 1500)
    dests = ["n%d" % i for i in range(40)] + [("g%d" % i, "n%d" % i) for i in range(5)]

    def dbytes(d):
        return (d if isinstance(d, str) else "%s|%s" % d).encode()

    live = {}
    for burst in range(30):
        for _ in range(400):
            t = rng.choice(topics)
            if rng.random() < 0.05:                       # a hot topic: a long bag (indexed)
                t = topics[burst % 7]
            d = rng.choice(dests)
            if rng.random() < 0.55:
                e.route_add(t.encode(), dbytes(d))
                o.add_route(t.encode(), d)
                live.setdefault(t, [])
                if d not in live[t]:
                    live[t].append(d)
            elif live:
                t = rng.choice(sorted(live))
                d = rng.choice(live[t])
                e.route_del(t.encode(), dbytes(d))
                o.del_route(t.encode(), d)
                live[t].remove(d)
                if not live[t]:
                    del live[t]
        if burst % 10 == 9:       # a filter deleted / re-inserted behind the router's back
            w = [t for t in live if "+" in t or t.endswith("#")]
            if w:
                t = rng.choice(w).encode()
                e.delete(t)
                e.debug_check_routes()
                e.insert(t)
        e.debug_check_routes()
        for t in rng.sample(topics, 50):
            got = e.get_routes(t.encode())
            assert [e.dest_bytes(x).decode() for x in got] == [dbytes(d).decode() for d in o.get_routes(t.encode())], t
    e.close()


def test_route_labels_follow_topic_order_through_relabels():
    """topics added in ascending, descending and clustered order (the list
    labelling's worst cases: no gap left, windows respread, universe grown
    past 2^16 labels)"""
    e = Engine(device=-1)
    asc = ["t/%06d" % i for i in range(20000)]
    for t in asc:
        e.route_add(t.encode(), b"n1")
    e.debug_check_routes()
    for t in reversed(["u/%06d" % i for i in range(3000)]):
        e.route_add(t.encode(), b"n1")
    for i in range(3000):
        e.route_add(("t/000100/%05d" % i).encode(), b"n2")    # all between two neighbours
    e.debug_check_routes()
    for t in asc[::2]:
        e.route_del(t.encode(), b"n1")
    e.debug_check_routes()
    e.close()
