"""emqx_broker:aggre/1 over emqx_router:match_routes/1 on the GPU (walk +
route expansion + aggre.hip) against the oracle (oracle/pytrie.py
RouteTable.match_deliveries = aggre(match_routes(T)), a clause-by-clause
transcription of src/emqx_broker.erl:194-206): ordered lists of
{To, Node} / {To, Group}, compared element for element."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.emqx_router import Router  # noqa: E402
from oracle import pytrie  # noqa: E402

pytestmark = pytest.mark.gpu

DESTS = ["n1", "n2", ("g1", "n1"), ("g1", "n2"), ("g2", "n2"), "n3", ("a", "n3"), "g1"]


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


def test_aggre_random_ops_vs_oracle(gpu_device):
    rng = random.Random(21)
    for rep in range(4):
        e = Engine(device=gpu_device)
        if rep % 2:
            e.set_option("layout", 2)
        r, o = Router(e, node="n1"), pytrie.RouteTable()
        pool = _pool(rng, 60)
        for step in range(600):
            t, d = rng.choice(pool), rng.choice(DESTS)
            if rng.random() < 0.7:
                r.add_route(t, d)
                o.add_route(t, d)
            else:
                r.del_route(t, d)
                o.del_route(t, d)
            if step % 150 == 149:
                topics = _topics(rng, 300) + pool
                got = r.match_deliveries_many(topics, tagged=True)
                for tp, row in zip(topics, got):
                    assert row == o.match_deliveries(tp), (rep, step, tp)
        e.close()


def test_aggre_long_lists_global_scratch(gpu_device):
    """route lists on every tm_aggre path: registers (<= 128), LDS (<= 512)
    and the global-scratch path (> 512)"""
    e = Engine(device=gpu_device)
    r, o = Router(e, node="n1"), pytrie.RouteTable()
    rng = random.Random(5)
    for f in [b"#", b"a/#", b"a/+", b"+/b", b"a/b"]:
        for k in range(rng.randint(150, 260)):
            d = ("g%d" % (k % 37), "n%d" % (k % 5)) if k % 3 == 0 else "n%d" % k
            r.add_route(f, d)
            o.add_route(f, d)
    for k in range(40):                       # a short list with groups: the register path
        d = ("g%d" % (k % 3), "n1") if k % 2 else "n%d" % (k % 7)
        r.add_route(b"$SYS/z", d)
        o.add_route(b"$SYS/z", d)
    topics = [b"a/b", b"a/c", b"x/b", b"a", b"$SYS/b", b"q", b"$SYS/z"]
    got = r.match_deliveries_many(topics, tagged=True)
    sizes = [len(o.match_routes(tp)) for tp in topics]
    # every kernel path: registers (<= 128 routes), LDS (<= 512), global scratch
    assert min(sizes) <= 128 and any(128 < x <= 512 for x in sizes) and max(sizes) > 512, sizes
    for tp, row in zip(topics, got):
        assert row == o.match_deliveries(tp), tp
    e.close()


def test_aggre_c1_scale_vs_oracle(gpu_device):
    """C1 filters with 1-3 dests (a third of them $share groups) + exact
    routes on some publish topics; 5K topics vs the oracle"""
    rng = np.random.default_rng(9)
    fb, fo = W.filters(1)
    filters = W.unpack(fb, fo)
    tb, to = W.topics(1, n=5000)
    topics = W.unpack(tb, to)
    e = Engine(device=gpu_device)
    r, o = Router(e, node="n1"), pytrie.RouteTable()
    for f in filters:
        for d in rng.choice(len(DESTS), size=int(rng.integers(1, 4)), replace=False):
            r.add_route(f, DESTS[d])
            o.add_route(f, DESTS[d])
    for t in topics[::7]:
        r.add_route(t, ("g9", "n2"))
        o.add_route(t, ("g9", "n2"))
    got = r.match_deliveries_many(topics, tagged=True)
    n = 0
    for tp, row in zip(topics, got):
        assert row == o.match_deliveries(tp), tp
        n += len(row)
    assert n > 10_000
    e.close()


def test_aggre_device_api_and_empty(gpu_device):
    import torch
    from emqx_amd.engine import pack
    e = Engine(device=gpu_device)
    dev = torch.device("cuda", gpu_device)
    r = Router(e, node="n1")
    for t in [b"a/+", b"a/#", b"#", b"a/b"]:
        r.add_route(t, "n1")
    r.add_route(b"a/#", ("g", "n2"))
    r.add_route(b"a/#", ("g", "n1"))
    topics = [b"a/b", b"$SYS/x", b"", b"a"]
    tb, to = pack(topics)
    n = len(topics)
    d_b = torch.from_numpy(tb.copy()).to(dev)
    d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    o = torch.empty(n + 1, dtype=torch.int64, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    to_d = torch.empty(64, dtype=torch.int32, device=dev)
    tg_d = torch.empty(64, dtype=torch.int32, device=dev)
    e.match_deliveries_batch_device(d_b, d_o, n, int(to[-1]), c, o, to_d, tg_d, 64, tot)
    torch.cuda.synchronize()
    want = r.match_deliveries_many(topics, tagged=True)
    oh, ch = o.cpu().numpy(), c.cpu().numpy()
    th, gh = to_d.cpu().numpy().view(np.uint32), tg_d.cpu().numpy().view(np.uint32)
    for t in range(n):
        got = [(topics[t] if int(th[j]) == Engine.TOPIC_ROUTE else e.filter_bytes(int(th[j])),
                e.target_bytes(int(gh[j]))) for j in range(int(oh[t]), int(oh[t]) + int(ch[t]))]
        assert int(ch[t]) <= int(oh[t + 1]) - int(oh[t])
        assert got == want[t]
    # match_routes(a/b) = a/b n1, a/+ n1, a/# n1, a/# {g,n2}, a/# {g,n1}, # n1: the last
    # group route is 5th, so '#' n1 leads and the usort of the first five follows
    assert want[0] == [(b"#", (0, b"n1")), (b"a/#", (0, b"n1")), (b"a/#", (1, b"g")), (b"a/+", (0, b"n1")),
                       (b"a/b", (0, b"n1"))]
    assert want[1] == []
    e2 = Engine(device=gpu_device)
    e2.insert(b"a/+")
    counts, offs, t2, g2 = e2.match_deliveries_batch(tb, to)
    assert int(offs[-1]) == 0 and len(t2) == 0
    e2.close()
    e.close()


def test_aggre_golden_vectors(gpu_device):
    """tests/golden/aggre_vectors.json (ORACLE-DERIVED: oracle aggre/1 over
    random route tables; no reference fixture exists, parity unpinned)"""
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "aggre_vectors.json")))
    for case in g["cases"]:
        e = Engine(device=gpu_device)
        r = Router(e, node="n1")
        for op, t, d in case["ops"]:
            dest = (d[1], d[2]) if d[0] == "group" else d[1]
            (r.add_route if op == "add" else r.del_route)(bytes.fromhex(t), dest)
        # valid publish names, then the out-of-domain wildcard names
        topics = [bytes.fromhex(t) for t in case["topics"] + case["ood_topics"]]
        got = r.match_deliveries_many(topics, tagged=True)
        for tp, row, want in zip(topics, got, case["deliveries"] + case["ood_deliveries"]):
            assert [[to.hex(), x[0], x[1].hex()] for to, x in row] == want, tp
        e.close()


def test_aggre_beyond_4096_group_routes(gpu_device):
    """a topic whose routes up to the last $share route exceed
    4096 takes tm_aggre_large's in-place row sort (was O(u^2) counting)"""
    e = Engine(device=gpu_device)
    r, o = Router(e, node="n1"), pytrie.RouteTable()
    rng = random.Random(44)
    for f, m in [(b"#", 6000), (b"a/#", 9500), (b"a/+", 300)]:
        for k in range(m):
            x = rng.randrange(1 << 30)
            d = ("g%d" % (x % 2900), "n%d" % (x % 3)) if k % 3 == 0 else "n%d" % (x % 7000)
            r.add_route(f, d)
            o.add_route(f, d)
    r.add_route(b"a/b", ("g7", "n2"))
    o.add_route(b"a/b", ("g7", "n2"))
    topics = [b"a/b", b"a", b"x/y", b"$SYS/a"]
    got = r.match_deliveries_many(topics, tagged=True)
    assert max(len(o.match_routes(tp)) for tp in topics) > 10000
    for tp, row in zip(topics, got):
        assert row == o.match_deliveries(tp), tp
    e.close()


def test_routes_enospc_small_batch_high_fanout(gpu_device):
    """out_cap > route workspace > ... with a 2-topic batch whose
    lists exceed the first call's default 64K cap: TM_ENOSPC, then exact"""
    from emqx_amd.engine import pack
    from emqx_amd import _lib as L
    e = Engine(device=gpu_device)
    n_routes = 70_000
    tb, to = pack([b"#"] * n_routes)
    db, do = pack([b"n%d" % i for i in range(n_routes)])
    e.route_add_many(tb, to, db, do)
    topics = [b"a/b", b"c"]
    pb, po = pack(topics)
    with pytest.raises(L.TopicMatchError) as ex:
        e.match_routes_batch(pb, po, out_cap=1 << 16)
    assert ex.value.code == L.TM_ENOSPC
    counts, offs, src, dst = e.match_routes_batch(pb, po)
    assert list(counts) == [n_routes, n_routes]
    assert list(dst[:n_routes]) == e.get_routes(b"#")
    assert list(dst[n_routes:]) == list(dst[:n_routes])
    with pytest.raises(L.TopicMatchError) as ex:
        e.match_deliveries_batch(pb, po, out_cap=1 << 16)
    assert ex.value.code == L.TM_ENOSPC
    counts, offs, to_, tg = e.match_deliveries_batch(pb, po)
    assert list(counts) == [n_routes, n_routes]     # node dests only: the fold reverses
    assert [e.target_bytes(int(x))[1] for x in tg[:3]] == [b"n69999", b"n69998", b"n69997"]
    e.close()


@pytest.mark.parametrize("double_buffer", [1, 0])
def test_route_image_churn_on_device_vs_oracle(gpu_device, double_buffer):
    """the in-place route image (engine.cpp) on the device under heavy churn:
    compactions (option route_gc tiny), exact-table regrowth, label
    relabels (topics added in order), a filter deleted and re-inserted
    behind the router's back; every burst's match_routes/1 and
    aggre(match_routes/1) equal the oracle's, with two image epochs and with
    one (double_buffer 0)"""
    rng = random.Random(31 + double_buffer)
    e = Engine(device=gpu_device)
    e.set_option("route_gc", 64)
    e.set_option("double_buffer", double_buffer)
    r, o = Router(e, node="n1"), pytrie.RouteTable()
    pool = _pool(rng, 400) + [b"t/%05d" % i for i in range(600)]
    live = {}
    for burst in range(12):
        for _ in range(700):
            t = rng.choice(pool)
            d = rng.choice(DESTS)
            if rng.random() < 0.6 or not live:
                r.add_route(t, d)
                o.add_route(t, d)
                live.setdefault(t, set()).add(d)
            else:
                t = rng.choice(sorted(live))
                d = rng.choice(sorted(live[t], key=str))
                r.del_route(t, d)
                o.del_route(t, d)
                live[t].discard(d)
                if not live[t]:
                    del live[t]
        if burst % 3 == 2:   # a wildcard filter deleted and re-inserted behind the router's back
            w = [t for t in live if b"+" in t or t.endswith(b"#")]
            if w:
                t = rng.choice(w)
                e.delete(t)
                e.insert(t)
        if burst % 4 == 3:
            e.debug_check_routes()
        topics = _topics(rng, 200) + [t for t in pool[:50] if b"+" not in t and b"#" not in t]
        got = r.match_deliveries_many(topics, tagged=True)
        for tp, row in zip(topics, got):
            assert row == o.match_deliveries(tp), (burst, tp)
        for tp, row in zip(topics, r.match_routes_many(topics)):
            assert [(x.topic, x.dest) for x in row] == o.match_routes(tp), (burst, tp)
    e.close()
