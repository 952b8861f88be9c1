"""emqx_router:match_routes/1 on the GPU (trie walk + route expansion,
routes.hip) against the oracle (oracle/pytrie.py RouteTable; O1 for the trie
order at C1 scale): ordered lists of (route topic, dest), exact-topic routes
first, then each matched filter's routes in emqx_trie:match/1 order."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.emqx_router import Router, _enc  # noqa: E402
from oracle import O1, pytrie  # noqa: E402

pytestmark = pytest.mark.gpu

DESTS = ["n1", "n2", ("g1", "n1"), ("g2", "n2"), "n3"]


def _pool(rng, k):
    words = [b"a", b"b", b"", b"+", b"#", b"$SYS", b"c", b"d"]
    pool = set()
    while len(pool) < k:
        ws = [rng.choice(words) for _ in range(rng.randint(1, 5))]
        if b"#" in ws[:-1]:
            continue
        pool.add(b"/".join(ws))
    return sorted(pool)


def _topics(rng, k):
    words = [b"a", b"b", b"", b"$SYS", b"c", b"d", b"x"]
    return [b"/".join(rng.choice(words) for _ in range(rng.randint(1, 6))) for _ in range(k)]


def test_match_routes_random_ops_vs_oracle(gpu_device):
    rng = random.Random(11)
    for rep in range(6):
        e = Engine(device=gpu_device)
        if rep % 2:
            e.set_option("layout", 2)        # relayout on every commit: filter ids must survive
        r, o = Router(e, node="n1"), pytrie.RouteTable()
        pool = _pool(rng, 60)
        for step in range(600):
            t, d = rng.choice(pool), rng.choice(DESTS)
            if rng.random() < 0.65:
                r.add_route(t, d)
                o.add_route(t, d)
            else:
                r.del_route(t, d)
                o.del_route(t, d)
            if step % 150 == 149:
                topics = _topics(rng, 300) + pool    # publish topics, plus the route topics themselves
                got = r.match_routes_many(topics)
                for tp, row in zip(topics, got):
                    assert [(x.topic, x.dest) for x in row] == o.match_routes(tp), (rep, step, tp)
        e.close()


def test_match_routes_c1_scale_vs_o1(gpu_device):
    """C1 filters with 1-3 dests each + exact-topic routes; 20K topics"""
    rng = np.random.default_rng(5)
    fb, fo = W.filters(1)
    filters = W.unpack(fb, fo)
    tb, to = W.topics(1, n=20000)
    topics = W.unpack(tb, to)
    e = Engine(device=gpu_device)
    routes = {}
    for f in filters:
        for d in rng.choice(len(DESTS), size=int(rng.integers(1, 4)), replace=False):
            e.route_add(f, _enc(DESTS[d]))
            routes.setdefault(f, []).append(_enc(DESTS[d]))
    for t in topics[::7]:                                   # direct routes of some publish topics
        e.route_add(t, _enc("n9"))
        routes.setdefault(t, [])
        if _enc("n9") not in routes[t]:
            routes[t].append(_enc("n9"))
    counts, offs, src, dst = e.match_routes_batch(tb, to)
    o1 = O1()
    o1.insert_many(fb, fo)
    oc, oo, oi = o1.match_ids(tb, to, threads=4)
    # O1 ids are the filters' insertion sequence (C1 filters are distinct)
    k, total = 0, 0
    for t, tp in enumerate(topics):
        want = [(tp, d) for d in routes.get(tp, [])]
        for fid in oi[int(oo[t]):int(oo[t + 1])]:
            f = filters[int(fid)]
            want += [(f, d) for d in routes[f]]
        got = []
        for j in range(int(offs[t]), int(offs[t]) + int(counts[t])):
            s = int(src[j])
            got.append((tp if s == Engine.TOPIC_ROUTE else e.filter_bytes(s), e.dest_bytes(int(dst[j]))))
        assert got == want, tp
        total += len(want)
    assert total == len(src) and total > 100_000
    e.close()


def test_match_routes_device_api_and_empty(gpu_device):
    import torch
    from emqx_amd.engine import pack
    e = Engine(device=gpu_device)
    dev = torch.device("cuda", gpu_device)
    r = Router(e, node="n1")
    for t in [b"a/+", b"a/#", b"#", b"a/b"]:
        r.add_route(t, "n1")
    r.add_route(b"a/#", ("g", "n2"))
    topics = [b"a/b", b"$SYS/x", b"", b"a"]
    tb, to = pack(topics)
    n = len(topics)
    d_b = torch.from_numpy(tb.copy()).to(dev)
    d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    o = torch.empty(n + 1, dtype=torch.int64, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    src = torch.empty(64, dtype=torch.int32, device=dev)
    dst = torch.empty(64, dtype=torch.int32, device=dev)
    e.match_routes_batch_device(d_b, d_o, n, int(to[-1]), c, o, src, dst, 64, tot)
    torch.cuda.synchronize()
    want = [[(x.topic, x.dest) for x in row] for row in r.match_routes_many(topics)]
    oh, sh, dh = o.cpu().numpy(), src.cpu().numpy().view(np.uint32), dst.cpu().numpy().view(np.uint32)
    for t in range(n):
        got = [(topics[t] if int(sh[j]) == Engine.TOPIC_ROUTE else e.filter_bytes(int(sh[j])),
                r._dest(int(dh[j]))) for j in range(int(oh[t]), int(oh[t + 1]))]
        assert got == want[t]
    assert want[0] == [(b"a/b", "n1"), (b"a/+", "n1"), (b"a/#", "n1"), (b"a/#", ("g", "n2")), (b"#", "n1")]
    assert want[1] == []
    # no routes at all: every topic maps to an empty list
    e2 = Engine(device=gpu_device)
    e2.insert(b"a/+")
    counts, offs, s2, d2 = e2.match_routes_batch(tb, to)
    assert int(offs[-1]) == 0 and len(s2) == 0
    e2.close()
    e.close()
